"""ctypes binding of libgrs.so (the C-ABI declared in include/grs.h).

The library is built in-tree (`make -C gpuradixsort_amd/csrc`, or `__graft_entry__.build()`)
and is the ONLY compute path of this package: there is no CPU fallback.  If the shared
object is missing, `lib()` raises; on a machine without a GPU the library still loads (so the
exported-symbol checks run on CPU) and every compute call returns GRS_ENODEV.

torch is imported before the library is loaded on purpose: torch ships its own
libamdhip64.so.7, and loading it first makes libgrs bind to that same HIP runtime (same
soname), so device pointers and streams from torch are valid inside libgrs.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_size_t, c_uint32, c_uint64, c_ulonglong, c_void_p

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libgrs.so")

GRS_OK, GRS_EINVAL, GRS_ENOMEM, GRS_EHIP, GRS_ECAPACITY, GRS_ENODEV, GRS_ETIMEOUT, GRS_ERCCL = range(8)
GRS_KEY_U32, GRS_KEY_U64 = 0, 1
GRS_RCCL_ID_BYTES = 128
GRS_MAX_N = (1 << 32) - (1 << 16)


class GrsError(RuntimeError):
    def __init__(self, status: int, what: str, detail: str = ""):
        self.status = status
        names = ["GRS_OK", "GRS_EINVAL", "GRS_ENOMEM", "GRS_EHIP", "GRS_ECAPACITY", "GRS_ENODEV",
                 "GRS_ETIMEOUT", "GRS_ERCCL"]
        name = names[status] if 0 <= status < len(names) else str(status)
        super().__init__(f"{what}: {name}" + (f" ({detail})" if detail else ""))


class grs_timing(ctypes.Structure):
    _fields_ = [("passes", c_int), ("total_ms", c_float), ("hist_ms", c_float),
                ("pass_ms", c_float * 16), ("copy_ms", c_float), ("kind", c_int)]


class grs_sharded_timing(ctypes.Structure):
    _fields_ = [("total_ms", c_float), ("before_ms", c_float), ("exchange_ms", c_float),
                ("after_ms", c_float), ("bytes_sent", c_uint64), ("bytes_received", c_uint64),
                ("presorted", c_int)]


class grs_key_extract(ctypes.Structure):
    _fields_ = [("kind", c_int), ("offset", c_uint32), ("transform", c_int),
                ("lo", c_float * 3), ("hi", c_float * 3)]


GRS_EXTRACT_FIELD, GRS_EXTRACT_MORTON3 = 0, 1

# grs_option (include/grs.h) by the names RadixSorter(options=...) takes, with the value names
# each accepts besides plain ints
OPTIONS = {
    "tile": (1, {"size": -1, "small": 0, "big": 1}),
    "xl": (2, {"size": -1, "never": 0, "always": 1}),
    "pass": (3, {"auto": 0, "v4": 4, "v6": 6, "fused": 8}),
    "records": (4, {"arrays": 0, "scratch": 1, "split": 2}),
    "rank": (5, {"probe": 0, "match": 1}),
    "sharded_path": (6, {"auto": 0, "general": 1}),
    "sharded_send": (7, {"regions": 0, "contig": 1, "shrunk": 2}),
    "exchange": (8, {"auto": 0, "partition": 1, "presorted": 2, "chunked": 3}),
    "merge": (9, {"rounds": 0, "kway": 1}),
    "fault_tile": (10, {"off": -1}),   # test hook: tile v of every pass never publishes
    "msd": (11, {"size": -1, "never": 0, "always": 1, "exact_p2": 2}),
    "seg_route": (12, {"shape": 0, "passes": 1, "composite": 2}),
    "h2_chunk": (13, {"size": 0}),
    "h2_piece": (14, {"default": 0}),
    "p3": (15, {"per_segment": 0, "persistent": 1, "whole_keys": 2}),
    "x_chunks": (16, {"default": 0}),
}

# (name, restype, argtypes) of every symbol include/grs.h declares
SIGNATURES = [
    ("grs_version", c_int, []),
    ("grs_status_string", c_char_p, [c_int]),
    ("grs_last_error", c_char_p, []),
    ("grs_create", c_int, [POINTER(c_void_p), c_size_t, c_int, c_int, c_int, c_int]),
    ("grs_destroy", None, [c_void_p]),
    ("grs_scratch_bytes", c_size_t, [c_void_p]),
    ("grs_debug_check_guards", c_int, [c_void_p, POINTER(c_uint64)]),
    ("grs_debug_msd_flags", c_int, [c_void_p, POINTER(c_uint32)]),
    ("grs_rank_mode", c_int, [c_void_p]),
    ("grs_lds_order_check", c_int, [c_int, c_int, c_int, POINTER(c_ulonglong)]),
    ("grs_set_option", c_int, [c_void_p, c_int, c_int]),
    ("grs_get_option", c_int, [c_void_p, c_int, POINTER(c_int)]),
    ("grs_pass_kernel", c_char_p, [c_void_p, c_size_t]),
    ("grs_sort", c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    ("grs_sort_bits", c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_int, c_void_p]),
    ("grs_set_profiling", c_int, [c_void_p, c_int]),
    ("grs_last_timing", c_int, [c_void_p, POINTER(grs_timing)]),
    ("grs_timing_history", c_int, [c_void_p, c_int, POINTER(grs_timing)]),
    ("grs_check_error", c_int, [c_void_p]),
    ("grs_stream_check_error", c_int, [c_void_p, c_void_p]),
    ("grs_partition", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p,
                              c_int, c_void_p, c_void_p]),
    ("grs_partition_ranges", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                     c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    ("grs_partition_regions", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                      c_void_p, c_void_p, c_int, c_size_t, c_void_p, c_void_p]),
    ("grs_sort_sharded", c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p,
                                 c_size_t, POINTER(c_size_t), c_void_p, c_void_p]),
    ("grs_sharded_last_timing", c_int, [c_void_p, POINTER(grs_sharded_timing)]),
    ("grs_sharded_redo_count", c_int, [c_void_p, POINTER(c_uint64)]),
    ("grs_rccl_unique_id", c_int, [c_void_p]),
    ("grs_rccl_comm_init", c_int, [POINTER(c_void_p), c_void_p, c_int, c_int, c_int]),
    ("grs_rccl_comm_destroy", None, [c_void_p]),
    ("grs_shard_splitters_host", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                         c_void_p, c_void_p]),
    ("grs_shard_plan_host", c_int, [c_void_p, c_int, c_int, POINTER(c_uint64), POINTER(c_uint64),
                                    POINTER(c_uint64)]),
    ("grs_shard_bounds_host", c_int, [c_void_p, c_size_t, c_int, c_void_p, c_void_p, c_int,
                                      POINTER(c_uint64)]),
    ("grs_shard_chunk_plan_host", c_int, [c_void_p, c_int, c_int, c_int, c_uint64, POINTER(c_uint64),
                                          POINTER(c_uint64), POINTER(c_uint64)]),
    ("grs_shard_samples_per_rank", c_int, [c_int]),
    ("grs_shard_sample", c_int, [c_void_p, c_size_t, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    ("grs_shard_encode_words_max", c_size_t, [c_size_t, c_int]),
    ("grs_shard_encode", c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_int, c_int,
                                 c_void_p, c_size_t, c_void_p, c_void_p]),
    ("grs_shard_decode_merge", c_int, [c_void_p, c_void_p, c_int, POINTER(c_uint64),
                                       POINTER(c_uint32), c_void_p, c_size_t, c_void_p]),
    ("grs_copy_u32", c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    ("grs_iota_u32", c_int, [c_void_p, c_size_t, c_uint32, c_void_p]),
    ("grs_gather_records", c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_size_t, c_void_p]),
    ("grs_fill_splitmix", c_int, [c_void_p, c_size_t, c_int, c_uint64, c_uint64, c_void_p]),
    ("grs_fill_permutation", c_int, [c_void_p, c_size_t, c_int, c_uint64, c_uint64, c_uint64, c_void_p]),
    ("grs_count_inversions", c_int, [c_void_p, c_size_t, c_int, POINTER(c_uint64), c_void_p]),
    ("grs_sort_host", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                              c_void_p]),
    ("grs_key_transform", c_int, [c_void_p, c_size_t, c_int, c_int, c_int, c_void_p]),
    ("grs_sort_records", c_int, [c_void_p, c_void_p, c_size_t, c_size_t, POINTER(grs_key_extract),
                                 c_void_p]),
    ("grs_records_key_buffers", c_int, [c_void_p, c_size_t, c_size_t, POINTER(c_void_p),
                                        POINTER(c_void_p)]),
    ("grs_sort_records_by_keys", c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_void_p, c_void_p,
                                         c_void_p]),
    ("grs_scan_scratch_bytes", c_size_t, [c_size_t]),
    ("grs_exclusive_scan_u32", c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_size_t,
                                       c_void_p]),
    ("grs_scan_check_error", c_int, [c_void_p, c_void_p]),
    ("grs_sort_segmented", c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_int,
                                   c_void_p]),
]

_LIB = None


def lib() -> ctypes.CDLL:
    """Load libgrs.so once (after torch, see module doc) and declare its signatures."""
    global _LIB
    if _LIB is not None:
        return _LIB
    import torch  # noqa: F401  (binds libgrs to torch's HIP runtime; see module doc)

    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C gpuradixsort_amd/csrc` or "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    L = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


def check(status: int, what: str) -> None:
    if status != GRS_OK:
        detail = lib().grs_last_error()
        raise GrsError(status, what, detail.decode() if detail else "")
