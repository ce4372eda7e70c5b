"""CPU tests of the drop-in boundary: libgrs.so loads, exports every symbol include/grs.h
declares, and validates arguments before touching a device (no compute calls here)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(REPO, "include", "grs.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(grs_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("grs_create", "grs_sort", "grs_sort_bits", "grs_destroy", "grs_last_timing",
                     "grs_gather_records", "grs_iota_u32", "grs_count_inversions"):
        assert required in names


def test_library_exports_every_declared_symbol():
    from gpuradixsort_amd import _lib

    L = _lib.lib()
    bound = {name for name, _, _ in _lib.SIGNATURES}
    for name in declared_functions():
        assert hasattr(L, name), f"libgrs.so does not export {name}"
        assert name in bound, f"_lib.SIGNATURES lacks {name}"


def test_version_and_status_strings():
    from gpuradixsort_amd import _lib

    L = _lib.lib()
    assert L.grs_version() == 410
    assert L.grs_status_string(0) == b"GRS_OK"
    assert L.grs_status_string(4) == b"GRS_ECAPACITY"


def test_create_validates_arguments_without_a_device():
    from gpuradixsort_amd import _lib

    L = _lib.lib()
    h = ctypes.c_void_p()
    assert L.grs_create(None, 10, 0, 0, 8, 0) == _lib.GRS_EINVAL
    assert L.grs_create(ctypes.byref(h), 10, 0, 0, 5, 0) == _lib.GRS_EINVAL      # radix 5
    assert L.grs_create(ctypes.byref(h), 10, 7, 0, 8, 0) == _lib.GRS_EINVAL      # key type
    assert L.grs_create(ctypes.byref(h), _lib.GRS_MAX_N + 1, 0, 0, 8, 0) == _lib.GRS_ECAPACITY
    assert L.grs_sort(None, None, None, 0, None) == _lib.GRS_EINVAL
    import torch

    if not torch.cuda.is_available():
        assert L.grs_create(ctypes.byref(h), 10, 0, 0, 8, 0) == _lib.GRS_ENODEV
        assert b"device" in L.grs_last_error()


def test_python_errors_are_loud():
    from gpuradixsort_amd import GrsError, _lib

    with pytest.raises(GrsError):
        _lib.check(_lib.GRS_EINVAL, "probe")


def test_extension_entry_points_validate_without_a_device():
    """§8f entry points reject bad arguments before any HIP call (no device needed)."""
    from gpuradixsort_amd import _lib

    L = _lib.lib()
    # key transform: key width and kind are checked; n = 0 and kind 0 are no-ops
    assert L.grs_key_transform(None, 10, 2, 1, 0, None) == _lib.GRS_EINVAL
    assert L.grs_key_transform(None, 10, 4, 3, 0, None) == _lib.GRS_EINVAL
    assert L.grs_key_transform(None, 10, 4, 1, 0, None) == _lib.GRS_EINVAL   # NULL keys
    assert L.grs_key_transform(None, 0, 4, 1, 0, None) == _lib.GRS_OK
    assert L.grs_key_transform(None, 10, 8, 0, 0, None) == _lib.GRS_OK
    # scan: scratch size grows with n; capacity, NULL and short-scratch checks
    assert L.grs_scan_scratch_bytes(0) == 16
    assert L.grs_scan_scratch_bytes(1) < L.grs_scan_scratch_bytes(1 << 24)
    assert L.grs_exclusive_scan_u32(None, None, 1 << 33, None, None, 0, None) == _lib.GRS_ECAPACITY
    assert L.grs_exclusive_scan_u32(None, None, 100, None, None, 0, None) == _lib.GRS_EINVAL
    fake = ctypes.c_void_p(1 << 20)   # never dereferenced: the size check fails first
    assert L.grs_exclusive_scan_u32(fake, fake, 100, None, fake, 4, None) == _lib.GRS_EINVAL
    # segmented sort: a sorter is required
    assert L.grs_sort_segmented(None, None, None, 10, None, 1, None) == _lib.GRS_EINVAL


def test_presorted_exchange_steps_validate_without_a_device():
    """The presorted exchange's step entry points reject bad arguments before any HIP call."""
    from gpuradixsort_amd import _lib

    L = _lib.lib()
    fake = ctypes.c_void_p(1 << 20)   # never dereferenced: validation fails first
    # bound of the encoded words: n keys + a 3-word directory entry per 256-key block and bucket
    assert L.grs_shard_encode_words_max(0, 8) == 3 * 8
    assert L.grs_shard_encode_words_max(1 << 20, 8) == (1 << 20) + 3 * ((1 << 20) // 256 + 8)
    assert L.grs_shard_sample(fake, 10, 2, 4, fake, fake, None) == _lib.GRS_EINVAL      # key bytes
    assert L.grs_shard_sample(fake, 10, 4, 0, fake, fake, None) == _lib.GRS_EINVAL      # no samples
    assert L.grs_shard_sample(None, 10, 4, 4, fake, fake, None) == _lib.GRS_EINVAL      # NULL keys
    assert L.grs_shard_encode(None, fake, 10, fake, fake, 2, 0, fake, 1 << 20, fake, None) == _lib.GRS_EINVAL
    wo = (ctypes.c_uint64 * 2)()
    ln = (ctypes.c_uint32 * 2)()
    assert L.grs_shard_decode_merge(None, fake, 2, wo, ln, fake, 10, None) == _lib.GRS_EINVAL
    t = _lib.grs_sharded_timing()
    assert L.grs_sharded_last_timing(None, ctypes.byref(t)) == _lib.GRS_EINVAL


def test_options_api_without_device():
    """grs_set_option / grs_get_option validate their arguments before touching a device: a
    NULL sorter is GRS_EINVAL (the options replace round 2's environment knobs)."""
    import ctypes

    from gpuradixsort_amd._lib import OPTIONS, lib

    L = lib()
    v = ctypes.c_int()
    for name, (opt, _) in OPTIONS.items():
        assert L.grs_set_option(None, opt, 0) == 1, name
        assert L.grs_get_option(None, opt, ctypes.byref(v)) == 1, name
