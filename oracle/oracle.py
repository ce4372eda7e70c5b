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
    segmented_sort_np      checkers for the §8f extensions (order-preserving key bits,
                           segmented sort): numpy restatements, no reference counterpart
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
    return (SEED_BASE + config_id) & _M


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

def cpu_sort(keys: np.ndarray, threads: int = 1) -> None:
    """In-place std::sort (threads == 1) or __gnu_parallel::sort."""
    if keys.dtype == np.uint32:
        lib().cpu_sort_u32(keys, keys.size, threads)
    else:
        lib().cpu_sort_u64(keys, keys.size, threads)


def cpu_stable_sort_pairs(keys: np.ndarray, vals: np.ndarray, threads: int = 1) -> None:
    lib().cpu_stable_sort_pairs_u32(keys, vals, keys.size, threads)
