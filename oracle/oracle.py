"""Parity oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the CPU baseline, never as the thing measured or shipped.

Contents (each restates the reference, amdreallyfast/GpuRadixSort, file:line cited):
  * ref_parallel_sort      the reference's GLSL path K1..K5 (oracle/ref_restatement.c), valid
                           for N <= 1,048,576 (the reference's capacity, PrefixScanBuffer.comp:36)
  * blelloch_scan          ParallelPrefixScan.comp:56-141's group scan (PrefixScan.xlsx KAT)
  * stable_sort            independent C merge sort (small N) / numpy stable argsort (any N)
  * splitmix keys          SURVEY.md §8(d) generator, numpy and C twins
  * cpu_sort               std::sort / __gnu_parallel::sort (BASELINE.md §4 CPU baseline)
  * ref_device_scan        K3a + K3b composed as ParallelSort.cpp:253-274 drives them
  * key_transform_np,
    segmented_sort_np,
    morton3_np,
    extract_keys_np        checkers for the §8f extensions (order-preserving key bits,
                           segmented sort, the K1 key-extraction hook): numpy restatements;
                           the reference names Morton codes as its purpose (ParallelSort.h:13-31)
                           but defines none, so these are "parity unpinned"
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
REF_CAPACITY = 1024 * 1024

_L = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
        u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
        L.ref_padded_count.restype = ctypes.c_uint32
        L.ref_padded_count.argtypes = [ctypes.c_uint32]
        L.ref_blelloch_scan_group.restype = ctypes.c_uint32
        L.ref_blelloch_scan_group.argtypes = [u32p, ctypes.c_uint32]
        L.ref_parallel_sort.restype = ctypes.c_int
        L.ref_parallel_sort.argtypes = [u32p, ctypes.c_uint32, ctypes.c_void_p]
        L.oracle_stable_sort_u32.restype = ctypes.c_int
        L.oracle_stable_sort_u32.argtypes = [u32p, u32p, ctypes.c_size_t]
        L.oracle_stable_sort_u64.restype = ctypes.c_int
        L.oracle_stable_sort_u64.argtypes = [u64p, u32p, ctypes.c_size_t]
        L.oracle_fill_splitmix_u32.restype = None
        L.oracle_fill_splitmix_u32.argtypes = [u32p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_fill_splitmix_u64.restype = None
        L.oracle_fill_splitmix_u64.argtypes = [u64p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64]
        L.cpu_hardware_concurrency.restype = ctypes.c_int
        L.cpu_hardware_concurrency.argtypes = []
        L.cpu_sort_u32.restype = None
        L.cpu_sort_u32.argtypes = [u32p, ctypes.c_size_t, ctypes.c_int]
        L.cpu_sort_u64.restype = None
        L.cpu_sort_u64.argtypes = [u64p, ctypes.c_size_t, ctypes.c_int]
        L.cpu_stable_sort_pairs_u32.restype = None
        L.cpu_stable_sort_pairs_u32.argtypes = [u32p, u32p, ctypes.c_size_t, ctypes.c_int]
        _L = L
    return _L


# ---- the reference's algorithm ------------------------------------------------------------

def padded_count(n: int) -> int:
    """P = ceil(N/1024)*1024 (PrefixSumSsbo.cpp:125-127)."""
    return int(lib().ref_padded_count(n))


def blelloch_scan(values) -> tuple[np.ndarray, int]:
    """Exclusive scan of one power-of-two group, ParallelPrefixScan.comp:56-141."""
    a = np.ascontiguousarray(values, dtype=np.uint32).copy()
    total = lib().ref_blelloch_scan_group(a, a.size)
    return a, int(total)


def ref_parallel_sort(keys) -> tuple[np.ndarray, np.ndarray]:
    """The reference's Sort(): returns (sorted keys, carried original index per slot)."""
    a = np.ascontiguousarray(keys, dtype=np.uint32).copy()
    perm = np.zeros(max(a.size, 1), dtype=np.uint32)
    r = lib().ref_parallel_sort(a, a.size, perm.ctypes.data)
    if r == -1:
        raise ValueError(f"N={a.size} exceeds the reference's capacity of {REF_CAPACITY}")
    if r != 0:
        raise MemoryError("ref_parallel_sort: allocation failed")
    return a, perm[: a.size]


def ref_device_scan(values) -> tuple[np.ndarray, int]:
    """The reference's device-wide exclusive scan: K3a scans each 1024-item group of the
    zero-padded input (ParallelPrefixScan.comp:56-141, PrefixSumSsbo.cpp:125-127), K3b scans
    the group totals in one 1024-wide group (ParallelPrefixScan.comp:151-196), and the
    group's prefix is added to each item (SortIntermediateData.comp:46-48 reads them so).
    uint32 arithmetic wraps mod 2^32 as in GLSL.  Valid for N <= 1,048,576."""
    a = np.ascontiguousarray(values, dtype=np.uint32)
    n = a.size
    if n > REF_CAPACITY:
        raise ValueError("beyond the reference's capacity")
    if n == 0:
        return a.copy(), 0
    p = padded_count(n)
    padded = np.zeros(p, dtype=np.uint32)
    padded[:n] = a
    groups = p // 1024
    sums = np.zeros(1024, dtype=np.uint32)
    for g in range(groups):
        out, tot = blelloch_scan(padded[g * 1024:(g + 1) * 1024])
        padded[g * 1024:(g + 1) * 1024] = out
        sums[g] = tot
    gscan, total = blelloch_scan(sums)
    with np.errstate(over="ignore"):
        padded += np.repeat(gscan[:groups], 1024)
    return padded[:n], int(total)


# ---- §8f extensions: checkers -------------------------------------------------------------

def key_transform_np(a: np.ndarray) -> np.ndarray:
    """Order-preserving unsigned image of signed / IEEE-754 keys (grs_key_transform)."""
    bits = a.dtype.itemsize * 8
    ut = np.uint32 if bits == 32 else np.uint64
    u = a.view(ut).copy()
    sign = ut(1) << ut(bits - 1)
    if a.dtype.kind == "i":
        return u ^ sign
    if a.dtype.kind == "f":
        neg = (u & sign) != 0
        return np.where(neg, ~u, u | sign).astype(ut)
    return u


def segmented_sort_np(keys: np.ndarray, offsets: np.ndarray, vals=None):
    """Every segment [off[s], off[s+1]) stably sorted on its own."""
    k = keys.copy()
    v = None if vals is None else vals.copy()
    for s in range(len(offsets) - 1):
        lo, hi = int(offsets[s]), int(offsets[s + 1])
        o = np.argsort(keys[lo:hi], kind="stable")
        k[lo:hi] = keys[lo:hi][o]
        if v is not None:
            v[lo:hi] = vals[lo:hi][o]
    return k, v


# ---- independent stable sorts -------------------------------------------------------------

def stable_sort_c(keys) -> tuple[np.ndarray, np.ndarray]:
    """C merge sort (oracle/ref_restatement.c): (sorted keys, stable permutation)."""
    k = np.ascontiguousarray(keys).copy()
    perm = np.zeros(k.size, dtype=np.uint32)
    if k.dtype == np.uint32:
        lib().oracle_stable_sort_u32(k, perm, k.size)
    elif k.dtype == np.uint64:
        lib().oracle_stable_sort_u64(k, perm, k.size)
    else:
        raise TypeError(k.dtype)
    return k, perm


def stable_argsort(keys: np.ndarray) -> np.ndarray:
    """numpy's stable sort (radix/timsort), the oracle for N beyond the C merge sort."""
    return np.argsort(keys, kind="stable").astype(np.uint32)


# ---- synthetic keys ------------------------------------------------------

SEED_BASE = 0x6A09E667F3BCC908
_M = (1 << 64) - 1


def config_seed(config_id: int) -> int:
    """seed = 0x6A09E667F3BCC908 + config id.  The north-star leg (id 6) has
    C3's n and key width, and splitmix64(seed ^ i) over i < 2^28 only permutes the seed's low
    28 bits, so a seed differing from C3's in those bits alone would give C3's key multiset: its
    seed also differs in bit 48 (round 4)."""
    s = SEED_BASE + config_id
    if config_id == 6:
        s += 1 << 48
    return s & _M


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x += np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return x


def splitmix_keys(n: int, key_bits: int, seed: int, first: int = 0) -> np.ndarray:
    """key[i] = splitmix64(seed ^ (first + i)) truncated to key_bits (C implementation)."""
    if key_bits == 32:
        out = np.empty(n, dtype=np.uint32)
        lib().oracle_fill_splitmix_u32(out, n, seed & _M, first)
    else:
        out = np.empty(n, dtype=np.uint64)
        lib().oracle_fill_splitmix_u64(out, n, seed & _M, first)
    return out


# ---- CPU baseline ---------------------------------------------------------------------------

def hardware_concurrency() -> int:
    """std::thread::hardware_concurrency() of this host."""
    return int(lib().cpu_hardware_concurrency())


def cpu_sort(keys: np.ndarray, threads: int = 1) -> None:
    """In-place std::sort (threads == 1) or __gnu_parallel::sort."""
    if keys.dtype == np.uint32:
        lib().cpu_sort_u32(keys, keys.size, threads)
    else:
        lib().cpu_sort_u64(keys, keys.size, threads)


def cpu_stable_sort_pairs(keys: np.ndarray, vals: np.ndarray, threads: int = 1) -> None:
    lib().cpu_stable_sort_pairs_u32(keys, vals, keys.size, threads)


def _spread(v: np.ndarray, bits: int) -> np.ndarray:
    """Spread the low `bits` bits of v to every third bit (Morton interleave)."""
    v = v.astype(np.uint64) & np.uint64((1 << bits) - 1)
    out = np.zeros_like(v)
    for b in range(bits):
        out |= ((v >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b)
    return out


def morton3_np(xyz: np.ndarray, lo, hi, key_bits: int = 32) -> np.ndarray:
    """Morton code of float32 positions (N, 3): per axis floor((v - lo) / (hi - lo) * 2^B)
    clamped to [0, 2^B) with NaN / non-positive -> 0 (B = 10 for u32 keys, 21 for u64),
    bits interleaved x, y, z from the top — grs_sort_records' GRS_EXTRACT_MORTON3, computed
    in float32 exactly as the device does."""
    bits = 10 if key_bits == 32 else 21
    xyz = np.asarray(xyz, np.float32)
    cells = []
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        for a in range(3):
            t = (xyz[:, a] - np.float32(lo[a])) / (np.float32(hi[a]) - np.float32(lo[a]))
            q = np.zeros(t.shape, np.uint64)
            pos = t > np.float32(0)
            top = t >= np.float32(1)
            mid = pos & ~top
            q[mid] = (t[mid] * np.float32(1 << bits)).astype(np.uint64)
            q[top] = (1 << bits) - 1
            q = np.minimum(q, np.uint64((1 << bits) - 1))
            cells.append(q)
    code = (_spread(cells[0], bits) << np.uint64(2)) | (_spread(cells[1], bits) << np.uint64(1)) \
        | _spread(cells[2], bits)
    return code.astype(np.uint32 if key_bits == 32 else np.uint64)


def extract_keys_np(records: np.ndarray, offset: int, key_bits: int = 32, transform: int = 0):
    """Key field of every record (uint8 array (N, record_bytes)) at byte `offset`, as the
    unsigned key grs_sort_records sorts by (transform: 0 unsigned, 1 signed, 2 IEEE float)."""
    kb = key_bits // 8
    raw = np.ascontiguousarray(records[:, offset:offset + kb]).view(
        np.uint32 if kb == 4 else np.uint64).reshape(-1)
    if transform == 0:
        return raw.copy()
    return key_transform_np(raw.view(
        (np.int32 if kb == 4 else np.int64) if transform == 1 else (np.float32 if kb == 4 else np.float64)))
