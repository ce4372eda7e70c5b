"""The error path end to end: a look-back spin that gives up must surface as GRS_ETIMEOUT
through every boundary, and the sorter must sort correctly again right after.

The reference reports nothing here: its scan silently overflows past 2^20 items
(PrefixScanBuffer.comp:36) and its shader errors are only printed
(ShaderStorage.cpp:338-339).  libgrs bounds every spin and keeps a sticky error word; the
test hook GRS_OPT_FAULT_TILE (include/grs.h) makes tile v of every pass withhold its
look-back tile words, so the later tiles of its look-back group hit the bound.
"""
import os
import subprocess

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(REPO, "gpuradixsort_amd", "grs_demo")
ETIMEOUT = 6

# (key_bits, pairs, radix_bits, options): every pass kernel and tile shape the library launches
SHAPES = [
    (32, False, 8, {}),                               # small tiles (4 per CU) at 2^22
    (32, False, 8, {"tile": "big"}),                  # big tiles, grs_onesweep_v4
    (32, False, 8, {"tile": "big", "xl": "always"}),  # XL two-round tiles
    (32, False, 8, {"tile": "big", "pass": "v6"}),    # persistent pass
    (32, True, 8, {"tile": "big"}),                   # u32 pairs, record passes
    (64, False, 8, {"tile": "big"}),                  # u64 keys
    (32, False, 4, {"tile": "big"}),                  # 4-bit digits (C2's kernel)
    (32, False, 4, {"tile": "big", "pass": "fused"}),  # 4-bit digits, every pass in one launch
    (32, False, 8, {"rank": "match", "tile": "big"}),  # ballot-match fallback
    # the MSD-first schedule (the default from 48M keys) at a size where H2 samples and P2
    # scatters into sampled regions: P1 (grs_onesweep_region) and P2 (grs_onesweep_seg) time out
    (32, False, 8, {"msd": "always"}),
    (32, True, 8, {"msd": "always"}),
    (64, False, 8, {"msd": "always"}),
]
MSD_N = (1 << 27) + 3


def _input(gpu, n, key_bits, pairs, seed):
    import gpuradixsort_amd as grs

    k = torch.empty(n, dtype=torch.uint32 if key_bits == 32 else torch.uint64, device=gpu)
    grs.fill_splitmix(k, seed)
    v = None
    if pairs:
        v = torch.empty(n, dtype=torch.uint32, device=gpu)
        grs.iota_u32(v)
    return k, v


def _expected(k, v):
    """The stable sort of (k, v), computed on the host (numpy: torch cannot index u32)."""
    kh = k.cpu().numpy()
    order = np.argsort(kh, kind="stable")
    return kh[order], (v.cpu().numpy()[order] if v is not None else None)


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: f"{s[0]}{'p' if s[1] else ''}-rb{s[2]}-"
                         + "-".join(f"{a}={b}" for a, b in s[3].items()))
def test_timeout_surfaces_then_sorter_recovers(gpu, shape):
    import gpuradixsort_amd as grs
    from gpuradixsort_amd._lib import GrsError

    key_bits, pairs, rb, opts = shape
    n = MSD_N if opts.get("msd") == "always" else 1 << 22
    s = grs.RadixSorter(n, key_bits=key_bits, pairs=pairs, radix_bits=rb, options=opts)
    assert s.get_option("fault_tile") == -1
    # all-ones keys first: the sorter's scratch then holds the largest digit everywhere, so
    # the slots a timed-out pass leaves unwritten hand the later passes more keys of the last
    # digit than the upfront histogram counted (runs past n without the pass's clamp)
    k, v = _input(gpu, n, key_bits, pairs, 10)
    k.view(torch.int32 if key_bits == 32 else torch.int64).fill_(-1)
    s.sort(k, v)
    s.check_error()
    assert s.check_guards() == 0
    s.set_option("fault_tile", 0)
    assert s.get_option("fault_tile") == 0
    # the keys (and values) sit at the front of larger buffers whose tails must stay untouched
    guard = 1 << 16
    kbuf = torch.empty(n + guard, dtype=torch.uint32 if key_bits == 32 else torch.uint64,
                       device=gpu)
    grs.fill_splitmix(kbuf, 11)
    ktail = kbuf[n:].clone()
    k = kbuf[:n]
    v = vbuf = None
    if pairs:
        vbuf = torch.empty(n + guard, dtype=torch.uint32, device=gpu)
        grs.iota_u32(vbuf)
        v = vbuf[:n]
    s.sort(k, v)
    with pytest.raises(GrsError) as e:
        s.check_error()
    assert e.value.status == ETIMEOUT
    assert (kbuf[n:].cpu().numpy() == ktail.cpu().numpy()).all(), "a timed-out sort wrote past n"
    if pairs:
        assert (vbuf[n:].cpu().numpy() == np.arange(n, n + guard)).all(), \
            "a timed-out sort wrote values past n"
    # the error word is sticky until read: the check above cleared it
    s.check_error()
    # and a timed-out sort stays inside the sorter's own scratch arrays too
    assert s.check_guards() == 0, "a timed-out sort wrote past a scratch array (guard band)"

    # the same sorter, hook off: the next sort is bit-exact (status buffers, tickets and the
    # alternating control blocks are consistent after a timed-out sort)
    s.set_option("fault_tile", -1)
    k, v = _input(gpu, n, key_bits, pairs, 12)
    ek, ev = _expected(k, v)
    s.sort(k, v)
    s.check_error()
    assert s.check_guards() == 0
    assert (k.cpu().numpy() == ek).all()
    if pairs:
        assert (v.cpu().numpy() == ev).all()
    s.close()
    del k, v, kbuf, vbuf
    torch.cuda.empty_cache()


def test_device_wide_check_reports_timeout(gpu):
    """grs_check_error (device-wide synchronisation) reports the same sticky word."""
    import gpuradixsort_amd as grs
    from gpuradixsort_amd._lib import GrsError

    n = 1 << 22
    s = grs.RadixSorter(n, options={"fault_tile": 3})
    k, _ = _input(gpu, n, 32, False, 13)
    s.sort(k)
    with pytest.raises(GrsError) as e:
        s.check_error(device_wide=True)
    assert e.value.status == ETIMEOUT
    s.set_option("fault_tile", -1)
    k, _ = _input(gpu, n, 32, False, 14)
    ek, _ = _expected(k, None)
    s.sort(k)
    s.check_error(device_wide=True)
    assert (k.cpu().numpy() == ek).all()


def test_python_parallel_sort_raises_then_recovers(gpu):
    """The reference-shaped Python mirror: ParallelSort.Sort() blocks and raises."""
    import gpuradixsort_amd as grs
    from gpuradixsort_amd._lib import GrsError

    n = 3_000_001
    k, _ = _input(gpu, n, 32, False, 15)
    ssbo = grs.OriginalDataSsbo(n)
    ssbo.Upload(k.cpu())
    ps = grs.ParallelSort(ssbo)
    ps._sorter.set_option("fault_tile", 0)
    with pytest.raises(GrsError) as e:
        ps.Sort()
    assert e.value.status == ETIMEOUT
    ps._sorter.set_option("fault_tile", -1)
    ssbo.Upload(k.cpu())
    ps.Sort()
    ek, _ = _expected(k, None)
    assert (ssbo.Download().numpy() == ek).all()


def test_cpp_facade_demo_exits_nonzero_on_timeout(gpu):
    """The C++ facade's blocking Sort() throws grs::Error(GRS_ETIMEOUT); grs_demo prints it
    and exits 2 (the reference's call pattern, main.cpp:152-160, with the fault hook set)."""
    r = subprocess.run([DEMO, "fault", "3000001", "7"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "GRS_ETIMEOUT" in r.stderr
    # and the same binary without the hook sorts exactly
    r = subprocess.run([DEMO, "3000001", "7"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "sorted=yes" in r.stdout, r.stdout + r.stderr
