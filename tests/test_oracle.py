"""CPU tests of the parity oracle: pinned to the reference's own known-answer data
(tests/golden/, lifted from PrefixScan.xlsx and main.cpp:128-143) before it is trusted, then
cross-checked against two independent stable sorts."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_xlsx_blelloch_scan_kat():
    """ParallelPrefixScan.comp:56-141 restated == the hand trace in PrefixScan.xlsx."""
    kat = load("prefix_scan_xlsx.json")
    out, total = oracle.blelloch_scan(kat["input"])
    assert out.tolist() == kat["exclusive_scan"]
    assert total == kat["total"] == 16
    # and it is the plain exclusive prefix sum
    assert out.tolist() == np.concatenate([[0], np.cumsum(kat["input"])[:-1]]).tolist()


def test_xlsx_upsweep_state():
    """Row 50 of the sheet = the up-sweep tree after 'set last item to 0' (line 103)."""
    kat = load("prefix_scan_xlsx.json")
    a = list(kat["input"])
    n = len(a)
    mult = 1
    pairs = n >> 1
    while pairs > 0:
        for tid in range(pairs):
            lo, hi = mult * (2 * tid + 1) - 1, mult * (2 * tid + 2) - 1
            a[hi] += a[lo]
        mult *= 2
        pairs >>= 1
    a[n - 1] = 0
    assert a == kat["upsweep_after_zero"]


def test_main_cpp_16key_kat():
    kat = load("main_cpp_16key.json")
    assert kat["input"] == [12, 1, 9, 2, 0, 11, 7, 3, 4, 15, 8, 5, 14, 13, 10, 6]
    keys, perm = oracle.ref_parallel_sort(kat["input"])
    assert keys.tolist() == kat["sorted"] == list(range(16))
    assert perm.tolist() == kat["perm"]


def test_padded_count():
    """P = ceil(N/1024)*1024 (PrefixSumSsbo.cpp:125-127)."""
    assert oracle.padded_count(0) == 0
    assert oracle.padded_count(1) == 1024
    assert oracle.padded_count(1024) == 1024
    assert oracle.padded_count(1025) == 2048
    assert oracle.padded_count(1_000_000) == 1_000_448


def test_reference_capacity_is_enforced():
    oracle.ref_parallel_sort(np.zeros(1024 * 1024, np.uint32))
    with pytest.raises(ValueError):
        oracle.ref_parallel_sort(np.zeros(1024 * 1024 + 1, np.uint32))


def _dists(n, rng):
    yield "uniform", rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    yield "perm", rng.permutation(n).astype(np.uint32)          # main.cpp:120-125
    yield "all_equal", np.full(n, 7, np.uint32)
    yield "all_ffffffff", np.full(n, 0xFFFFFFFF, np.uint32)     # not confused with padding
    yield "sorted", np.sort(rng.integers(0, 2**32, n, dtype=np.uint64)).astype(np.uint32)
    yield "reversed", np.arange(n, 0, -1, dtype=np.uint32)
    yield "16_unique", rng.integers(0, 16, n).astype(np.uint32) * np.uint32(0x10000001)
    yield "mixed_ff", np.where(rng.random(n) < 0.3, 0xFFFFFFFF, rng.integers(0, 100, n)).astype(np.uint32)


@pytest.mark.parametrize("n", [0, 1, 2, 1023, 1024, 1025, 5000, 65536])
def test_restatement_equals_stable_sort(n):
    """The reference's output order == std::stable_sort by key: keys and
    the carried _globalIndexOfOriginalData, including genuine 0xffffffff keys."""
    rng = np.random.default_rng(n + 1)
    for name, keys in _dists(n, rng):
        rk, rp = oracle.ref_parallel_sort(keys)
        ck, cp = oracle.stable_sort_c(keys)
        np_perm = oracle.stable_argsort(keys)
        assert (rk == ck).all(), name
        assert (rp == cp).all(), name
        assert (rp == np_perm).all(), name
        assert (rk == keys[np_perm]).all(), name


def test_restatement_at_capacity():
    rng = np.random.default_rng(5)
    keys = rng.integers(0, 2**32, 1024 * 1024, dtype=np.uint64).astype(np.uint32)
    rk, rp = oracle.ref_parallel_sort(keys)
    perm = oracle.stable_argsort(keys)
    assert (rp == perm).all() and (rk == keys[perm]).all()


def test_splitmix_c_matches_numpy():
    for kb in (32, 64):
        seed = oracle.config_seed(3)
        c = oracle.splitmix_keys(1000, kb, seed, first=12345)
        x = oracle.splitmix64_np(np.uint64(seed) ^ (np.arange(1000, dtype=np.uint64) + np.uint64(12345)))
        assert (c == x.astype(c.dtype)).all()


def test_small_config_digests():
    """digests.json (committed) for C1/C2 reproduce from the seeds with numpy."""
    d = load("digests.json")
    for name in ("c1_64k_u32", "c1_64k_u32_pairs", "c2_16m_u32"):
        rec = d[name]
        keys = oracle.splitmix_keys(rec["n"], rec["key_bits"], rec["seed"])
        if rec["pairs"]:
            perm = oracle.stable_argsort(keys)
            assert hashlib.sha256(perm.tobytes()).hexdigest() == rec["sha256_perm"]
            keys = keys[perm]
        else:
            keys = np.sort(keys)
        assert hashlib.sha256(keys.tobytes()).hexdigest() == rec["sha256_keys"]


def test_cpu_sort_wrappers():
    """The host std::sort plumbing path (BASELINE.json configs[0]: 64K u32 keys)."""
    rec = load("digests.json")["c1_64k_u32"]
    keys = oracle.splitmix_keys(rec["n"], 32, rec["seed"])
    for threads in (1, 4):
        k = keys.copy()
        oracle.cpu_sort(k, threads)
        assert hashlib.sha256(k.tobytes()).hexdigest() == rec["sha256_keys"]
    rec = load("digests.json")["c1_64k_u32_pairs"]
    k = keys.copy()
    v = np.arange(k.size, dtype=np.uint32)
    oracle.cpu_stable_sort_pairs(k, v, 2)
    assert hashlib.sha256(v.tobytes()).hexdigest() == rec["sha256_perm"]


def test_ref_device_scan_pinned_by_xlsx_and_cumsum():
    """K3a + K3b composed (oracle.ref_device_scan) == the PrefixScan.xlsx hand trace, and ==
    an independent cumsum (mod 2^32) across group boundaries."""
    kat = load("prefix_scan_xlsx.json")
    out, total = oracle.ref_device_scan(kat["input"])
    assert out.tolist() == kat["exclusive_scan"] and total == kat["total"]
    rng = np.random.default_rng(5)
    for n in (1, 1023, 1024, 1025, 3000, 1 << 16):
        a = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        out, total = oracle.ref_device_scan(a)
        c = (np.cumsum(a.astype(np.uint64)) - a.astype(np.uint64)) & 0xFFFFFFFF
        assert np.array_equal(out, c.astype(np.uint32))
        assert total == int(a.astype(np.uint64).sum() & 0xFFFFFFFF)


def test_key_transform_np_orders_like_numpy():
    rng = np.random.default_rng(2)
    for dt in (np.int32, np.int64):
        a = rng.integers(np.iinfo(dt).min, np.iinfo(dt).max, 5000, dtype=dt)
        assert np.array_equal(a[np.argsort(oracle.key_transform_np(a), kind="stable")],
                              np.sort(a, kind="stable"))
    for dt in (np.float32, np.float64):
        a = (rng.standard_normal(5000) * 1e3).astype(dt)
        a[:4] = [np.inf, -np.inf, 0.0, -0.0]
        assert np.array_equal(a[np.argsort(oracle.key_transform_np(a), kind="stable")],
                              np.sort(a, kind="stable"))
