"""GPU parity tests: libgrs's HIP sort (through the C-ABI) against the oracle.

Bar: bit-exact keys AND the exact stable permutation (payload = input index, the reference's
_globalIndexOfOriginalData).  N <= 1,048,576 u32 cases are checked against the restatement
of the reference's own GLSL path (oracle.ref_parallel_sort); larger and u64 cases against
stable sorts (C merge sort / numpy stable argsort); full BASELINE sizes against committed
SHA-256 digests of the expected output plus size-independent properties.
"""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_SORTERS = {}


def sorter(key_bits, pairs, radix_bits, capacity):
    import gpuradixsort_amd as grs

    k = (key_bits, pairs, radix_bits)
    s = _SORTERS.get(k)
    if s is None or s.capacity < capacity:
        if s is not None:
            s.close()
        s = grs.RadixSorter(max(capacity, 1 << 20), key_bits=key_bits, pairs=pairs,
                            radix_bits=radix_bits)
        _SORTERS[k] = s
    return s


def to_dev(a: np.ndarray, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def gpu_sort(keys: np.ndarray, pairs: bool, radix_bits: int, dev, begin_bit=0, end_bit=None):
    kb = keys.dtype.itemsize * 8
    s = sorter(kb, pairs, radix_bits, keys.size)
    k = to_dev(keys, dev)
    v = to_dev(np.arange(keys.size, dtype=np.uint32), dev) if pairs else None
    s.sort(k, v, begin_bit=begin_bit, end_bit=end_bit)
    torch.cuda.synchronize()
    s.check_error()
    return k.cpu().numpy(), (v.cpu().numpy() if pairs else None)


def distributions(n, kb, rng):
    dt = np.uint32 if kb == 32 else np.uint64
    top = np.iinfo(dt).max
    yield "uniform", rng.integers(0, top, n, dtype=dt, endpoint=True)
    yield "perm", rng.permutation(n).astype(dt)                 # main.cpp:120-125
    yield "all_equal", np.full(n, 7, dt)
    yield "all_max", np.full(n, top, dt)                        # 0xffffffff is a real key
    yield "sorted", np.sort(rng.integers(0, top, n, dtype=dt, endpoint=True))
    yield "reversed", np.arange(n, 0, -1).astype(dt)
    yield "16_unique", (rng.integers(0, 16, n).astype(dt) * dt(0x10000001))
    yield "mixed_max", np.where(rng.random(n) < 0.3, top, rng.integers(0, 100, n)).astype(dt)
    yield "low_entropy", (rng.integers(0, top, n, dtype=dt, endpoint=True)
                          & rng.integers(0, top, n, dtype=dt, endpoint=True)
                          & rng.integers(0, top, n, dtype=dt, endpoint=True))


# Tile edges of the pass (grs_capi.hip BigTile / SmallTile): small tiles 4096 (u32 keys),
# 2048 (u32 pairs, u64 keys), 1536 (u64 pairs); big tiles 36864 / 17408 / 11264 (ballot-match
# fallback 32768 / 16384 / 10240); look-back groups of 8 tiles.  Sizes up to 2^20 run the small tiles by default; test_tile_shapes pins
# the big ones.
SIZES = [0, 1, 2, 63, 64, 65, 1023, 1024, 1025, 1535, 1537, 2047, 2049, 4095, 4096, 4097,
         12289, 16383, 16385, 32769, 36865, 65536, 98305, 131073, 262145, 1 << 20]


@pytest.mark.parametrize("radix_bits", [4, 8])
@pytest.mark.parametrize("pairs", [False, True])
@pytest.mark.parametrize("n", SIZES)
def test_u32_matches_reference_path(gpu, n, pairs, radix_bits):
    """u32, N <= 2^20: keys and stable permutation == the reference's GLSL path."""
    rng = np.random.default_rng(1000 + n)
    for name, keys in distributions(n, 32, rng):
        if n > 65536 and name not in ("uniform", "perm", "16_unique"):
            continue
        rk, rp = oracle.ref_parallel_sort(keys)
        gk, gv = gpu_sort(keys, pairs, radix_bits, gpu)
        assert np.array_equal(gk, rk), f"{name}: keys differ"
        if pairs:
            assert np.array_equal(gv, rp), f"{name}: permutation differs (stability)"


@pytest.mark.parametrize("radix_bits", [4, 8])
@pytest.mark.parametrize("pairs", [False, True])
@pytest.mark.parametrize("n", [0, 1, 65, 4097, 12289, 100003, 1 << 20])
def test_u64_matches_stable_sort(gpu, n, pairs, radix_bits):
    rng = np.random.default_rng(2000 + n)
    for name, keys in distributions(n, 64, rng):
        if n > 65536 and name not in ("uniform", "16_unique", "mixed_max"):
            continue
        perm = oracle.stable_argsort(keys)
        gk, gv = gpu_sort(keys, pairs, radix_bits, gpu)
        assert np.array_equal(gk, keys[perm]), f"{name}: keys differ"
        if pairs:
            assert np.array_equal(gv, perm), f"{name}: permutation differs"


def test_lds_lane_order_at_scale(gpu):
    """The property the atomic ranking relies on, checked at scale on the device through the
    C-ABI (grs_lds_order_check): 5 digit patterns x 4 counter layouts x 2048 workgroups x 8
    waves x 256 items x 64 lanes (5.4 G returning atomics), every returned value compared with
    a ballot-match rank.  The sorter's create-time probe is a 24-atomic spot check of this."""
    import ctypes

    from gpuradixsort_amd._lib import check, lib

    bad = ctypes.c_ulonglong(1)
    check(lib().grs_lds_order_check(gpu.index, 2048, 256, ctypes.byref(bad)), "grs_lds_order_check")
    assert bad.value == 0


def test_rank_mode_is_atomic_on_gfx950(gpu):
    """The LDS lane-order probe passes on MI355X, so the atomic-rank pass runs."""
    s = sorter(32, False, 8, 1 << 20)
    assert s.rank_mode == "atomic"
    assert s.pass_kernel_for(1 << 20) == "grs_onesweep_v4"   # small tiles
    assert sorter(32, True, 8, 1 << 20).pass_kernel == "grs_onesweep_v4"
    # big tiles: persistent pass where a CU sees at most 4 tiles or digits are 4-bit
    assert s.pass_kernel_for(1 << 24) == "grs_onesweep_v6"
    assert s.pass_kernel_for(1 << 27) == "grs_onesweep_v4"
    assert sorter(32, False, 4, 1 << 20).pass_kernel_for(1 << 24) == "grs_onesweep_v6"


@pytest.mark.parametrize("tile", ["big", "small"])
@pytest.mark.parametrize("kb,pairs", [(32, False), (32, True), (64, False), (64, True)])
def test_tile_shapes(gpu, monkeypatch, tile, kb, pairs):
    """Option tile pins the big (1024-thread) or small (256-thread) tile shape whatever the size:
    bit-exact across each shape's tile edges and look-back group edges (8 tiles), ragged
    last groups, both digit widths."""
    import gpuradixsort_amd as grs

    # u64 pairs: 22K-pair tiles reordered in two rounds of 11K (t // 2 is the round edge)
    big = {(32, False): 36864, (32, True): 17408, (64, False): 17408, (64, True): 22528}
    small = {(32, False): 4096, (32, True): 2048, (64, False): 2048, (64, True): 1536}
    t = (big if tile == "big" else small)[(kb, pairs)]
    rng = np.random.default_rng(kb * 10 + pairs)
    dt = np.uint32 if kb == 32 else np.uint64
    sizes = (1, t // 2 - 1, t // 2 + 1, t - 1, t + 1, 8 * t - 1, 8 * t + 1, 8 * t * 9 + 3,
             17 * t + 5)
    s = grs.RadixSorter(max(sizes), key_bits=kb, pairs=pairs, radix_bits=8, options={"tile": tile})
    s4 = grs.RadixSorter(max(sizes), key_bits=kb, pairs=pairs, radix_bits=4, options={"tile": tile})
    for n in sizes:
        keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
        keys[::31] = keys[0]   # ties across tiles
        keys[::97] = np.iinfo(dt).max
        perm = oracle.stable_argsort(keys)
        for srt in (s, s4):
            k = to_dev(keys, gpu)
            v = to_dev(np.arange(n, dtype=np.uint32), gpu) if pairs else None
            srt.sort(k, v)
            srt.check_error()
            assert np.array_equal(k.cpu().numpy(), keys[perm]), (n, srt.radix_bits)
            if pairs:
                assert np.array_equal(v.cpu().numpy(), perm), (n, srt.radix_bits)
    s.close()
    s4.close()


@pytest.mark.parametrize("kb,pairs,t,records", [(32, False, 768 * 64, "2"), (32, True, 768 * 40, "2"),
                                                (32, True, 768 * 40, "1"), (32, True, 768 * 40, "0"),
                                                (64, False, 768 * 44, "2")])
def test_xl_tiles(gpu, monkeypatch, kb, pairs, t, records):
    """Option xl=always pins the two-round XL tiles (768 threads; LDS holds half the tile per round)
    at every big-tile size: bit-exact across tile, round and look-back group edges (the
    library uses them from 32 tiles per CU).  u32 pairs: the passes write 8-byte (key, value)
    records -- into the scratch, and (records=2, even n, 4 passes) split over the caller's
    two arrays for the middle passes; records=1: the scratch only; 0: two arrays
    throughout; a 24-bit sort (3 passes) keeps two arrays and copies back."""
    import gpuradixsort_amd as grs

    h = t // 2
    rng = np.random.default_rng(48 + kb + pairs)
    dt = np.uint32 if kb == 32 else np.uint64
    # odd and even sizes: split records need an even n
    sizes = (1, 2, h - 1, h, h + 1, t - 1, t, t + 1, t + h + 3, t + h + 4, 8 * t - 1, 8 * t,
             8 * t + 1, 8 * t * 5 + h + 7, 8 * t * 5 + h + 8)
    s = grs.RadixSorter(max(sizes), key_bits=kb, pairs=pairs,
                        options={"xl": "always", "tile": "big", "records": int(records)})
    assert s.pass_kernel_for(max(sizes)) == "grs_onesweep_v4"
    for n in sizes:
        keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
        keys[::29] = keys[0]
        keys[::101] = np.iinfo(dt).max
        perm = oracle.stable_argsort(keys)
        k = to_dev(keys, gpu)
        v = to_dev(np.arange(n, dtype=np.uint32), gpu) if pairs else None
        s.sort(k, v)
        s.check_error()
        assert np.array_equal(k.cpu().numpy(), keys[perm]), n
        if pairs:
            assert np.array_equal(v.cpu().numpy(), perm), n
    if pairs:   # bits [0, 24): 3 passes, no record passes, result copied back;
        #             bits [8, 24): 2 passes, record passes in between
        n = sizes[-1]
        for lo, hi in ((0, 24), (8, 24)):
            keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
            perm = oracle.stable_argsort((keys >> np.uint32(lo)) & np.uint32((1 << (hi - lo)) - 1))
            k = to_dev(keys, gpu)
            v = to_dev(np.arange(n, dtype=np.uint32), gpu)
            s.sort(k, v, begin_bit=lo, end_bit=hi)
            s.check_error()
            assert np.array_equal(k.cpu().numpy(), keys[perm]), (lo, hi)
            assert np.array_equal(v.cpu().numpy(), perm), (lo, hi)
    s.close()


@pytest.mark.parametrize("records", ["1", "2"])
def test_big_tile_record_passes(gpu, monkeypatch, records):
    """The one-round big-tile v4 pass with record flags (launch_rec kinds 1-4: 8-byte (key,
    value) records in the scratch, and for even n split over the caller's two arrays): the
    library takes it between ~2^24 and ~2^28 u32 pairs.  Options xl=never, tile=big, pass=v4
    pin it at test sizes; odd and even n (split records need an even n); payload == the
    stable permutation."""
    import gpuradixsort_amd as grs

    t = 1024 * 17
    h = t // 2
    rng = np.random.default_rng(170 + int(records))
    sizes = (2, 3, h, h + 1, t, t + 1, 8 * t, 8 * t + 1, 8 * t * 3 + h + 7, 8 * t * 3 + h + 8,
             2_000_000, 2_000_001)
    s = grs.RadixSorter(max(sizes), key_bits=32, pairs=True,
                        options={"xl": "never", "tile": "big", "pass": "v4",
                                 "records": int(records)})
    assert s.pass_kernel_for(max(sizes)) == "grs_onesweep_v4"
    for n in sizes:
        keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        keys[::29] = keys[0]
        keys[::101] = 0xFFFFFFFF
        perm = oracle.stable_argsort(keys)
        k = to_dev(keys, gpu)
        v = to_dev(np.arange(n, dtype=np.uint32), gpu)
        s.sort(k, v)
        s.check_error()
        assert np.array_equal(k.cpu().numpy(), keys[perm]), n
        assert np.array_equal(v.cpu().numpy(), perm), n
    s.close()


@pytest.mark.parametrize("shape", ["xl", "big"])
@pytest.mark.parametrize("offset", [1, 2])
def test_pairs_offset_views(gpu, monkeypatch, shape, offset):
    """u32 pairs sorted through views at a storage offset (keys[offset:], vals[offset:]):
    offset 1 leaves the arrays only 4-byte aligned, so the record passes that move 8-byte
    records on the caller's arrays must fall back to two arrays (run_sort's alignment gate);
    offset 2 is 8-byte aligned and keeps the split records.  Even n past the record-pass
    thresholds; payload == the stable permutation, and the elements before the view stay."""
    import gpuradixsort_amd as grs

    opts = {"tile": "big", "records": "split"}
    opts.update({"xl": "always"} if shape == "xl" else {"xl": "never", "pass": "v4"})
    rng = np.random.default_rng(90 + offset)
    n = 1_000_002
    s = grs.RadixSorter(n, key_bits=32, pairs=True, options=opts)
    keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    keys[::31] = 12345
    perm = oracle.stable_argsort(keys)
    kb = torch.full((n + offset,), 0xABCDEF, dtype=torch.int32, device=gpu)
    vb = torch.full((n + offset,), 0x13579B, dtype=torch.int32, device=gpu)
    k, v = kb[offset:], vb[offset:]
    assert (k.data_ptr() % 8 == 0) == (offset % 2 == 0)
    k.copy_(torch.from_numpy(keys.view(np.int32)).to(gpu))
    v.copy_(torch.arange(n, dtype=torch.int32, device=gpu))
    s.sort(k, v)
    s.check_error()
    assert np.array_equal(k.cpu().numpy().view(np.uint32), keys[perm])
    assert np.array_equal(v.cpu().numpy().view(np.uint32), perm)
    assert kb[:offset].eq(0xABCDEF).all() and vb[:offset].eq(0x13579B).all()
    s.close()


def test_misaligned_u64_keys_rejected(gpu):
    """u64 keys must be 8-byte aligned: a 4-byte-offset pointer returns GRS_EINVAL instead of
    issuing misaligned 8-byte accesses."""
    import ctypes

    import gpuradixsort_amd as grs
    from gpuradixsort_amd._lib import lib

    s = grs.RadixSorter(1024, key_bits=64, pairs=False)
    buf = torch.zeros(2048 + 2, dtype=torch.int32, device=gpu)
    rc = lib().grs_sort(s._h, ctypes.c_void_p(buf.data_ptr() + 4), ctypes.c_void_p(0), 1024,
                        ctypes.c_void_p(0))
    assert rc != 0 and "aligned" in lib().grs_last_error().decode()
    s.close()


def test_ballot_match_fallback(gpu, monkeypatch):
    """Option rank=match forces ballot-match ranking (the path taken if the LDS order probe
    ever fails): same bit-exact results, both tile shapes."""
    import gpuradixsort_amd as grs

    rng = np.random.default_rng(5)
    for tile in ("big", "small"):
        for kb, pairs, rb in ((32, False, 8), (32, True, 4), (64, True, 8), (64, False, 4)):
            dt = np.uint32 if kb == 32 else np.uint64
            keys = rng.integers(0, np.iinfo(dt).max, 300_007, dtype=dt, endpoint=True)
            keys[::5] = 77
            perm = oracle.stable_argsort(keys)
            s = grs.RadixSorter(keys.size, key_bits=kb, pairs=pairs, radix_bits=rb,
                                options={"rank": "match", "tile": tile})
            assert s.rank_mode == "match"
            k = to_dev(keys, gpu)
            v = to_dev(np.arange(keys.size, dtype=np.uint32), gpu) if pairs else None
            s.sort(k, v)
            s.check_error()
            assert np.array_equal(k.cpu().numpy(), keys[perm]), (tile, kb, pairs, rb)
            if pairs:
                assert np.array_equal(v.cpu().numpy(), perm)
            s.close()


@pytest.mark.parametrize("pass_kernel", ["v6", "fused"])
@pytest.mark.parametrize("kb,pairs,rb", [(32, False, 8), (32, True, 8), (64, False, 8),
                                          (64, True, 8), (32, False, 4), (64, True, 4)])
def test_persistent_pass(gpu, monkeypatch, kb, pairs, rb, pass_kernel):
    """Option pass=v6: the persistent big-tile pass (grs_onesweep_v6: resident workgroups loop
    over tickets, the next tile's loads issued behind the reorder) gives the same bit-exact
    results across tile edges, for every key/payload type and both digit widths (u64 pairs at
    8-bit digits keep the two-round v4 pass, whose second round needs the registers the
    prefetch would take).  pass=fused: every pass in one launch of those workgroups with a grid
    barrier between passes (grs_onesweep_fused; u32 pairs at 8-bit digits keep v6 and their
    record passes)."""
    import gpuradixsort_amd as grs

    rng = np.random.default_rng(11 + kb + pairs + rb)
    dt = np.uint32 if kb == 32 else np.uint64
    for n in (1, 16383, 32769, 36865, 8 * 36864 + 1, 1_000_003, 3 * 1024 * 1024 + 7):
        keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
        keys[::7] = np.iinfo(dt).max
        keys[1::13] = 3
        perm = oracle.stable_argsort(keys)
        s = grs.RadixSorter(n, key_bits=kb, pairs=pairs, radix_bits=rb,
                            options={"pass": pass_kernel, "tile": "big"})
        if pass_kernel == "fused" and not (kb == 64 and pairs and rb == 8) and not (kb == 32 and pairs and rb == 8):
            assert s.pass_kernel_for(max(n, 2)) in ("grs_onesweep_fused", "grs_onesweep_v4"), n
        k = to_dev(keys, gpu)
        v = to_dev(np.arange(n, dtype=np.uint32), gpu) if pairs else None
        s.sort(k, v)
        s.check_error()
        assert np.array_equal(k.cpu().numpy(), keys[perm]), n
        if pairs:
            assert np.array_equal(v.cpu().numpy(), perm), n
        s.close()


def test_golden_16key_kat(gpu):
    kat = json.load(open(os.path.join(GOLDEN, "main_cpp_16key.json")))
    keys = np.array(kat["input"], np.uint32)
    for rb in (4, 8):
        gk, gv = gpu_sort(keys, True, rb, gpu)
        assert gk.tolist() == kat["sorted"] and gv.tolist() == kat["perm"]


def test_bit_ranges(gpu):
    """grs_sort_bits: sort on key bits [b, e) only, stably (the reference's bit loop,
    ParallelSort.cpp:236, made a parameter)."""
    rng = np.random.default_rng(7)
    keys = rng.integers(0, 2**32, 300_001, dtype=np.uint64).astype(np.uint32)
    for b, e in ((0, 12), (5, 17), (16, 32), (3, 4), (0, 31)):
        sub = (keys >> np.uint32(b)) & np.uint32((1 << (e - b)) - 1)
        perm = oracle.stable_argsort(sub)
        for rb in (4, 8):
            gk, gv = gpu_sort(keys, True, rb, gpu, b, e)
            assert np.array_equal(gv, perm) and np.array_equal(gk, keys[perm]), (b, e, rb)


def test_larger_u32(gpu):
    rng = np.random.default_rng(11)
    for n in ((1 << 20) + 1, 3_000_017):
        keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        keys[::97] = 0xFFFFFFFF
        perm = oracle.stable_argsort(keys)
        for rb in (4, 8):
            gk, gv = gpu_sort(keys, True, rb, gpu)
            assert np.array_equal(gv, perm) and np.array_equal(gk, keys[perm])


def _digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name,radix_bits", [("c1_64k_u32", 8), ("c1_64k_u32_pairs", 8),
                                             ("c2_16m_u32", 4)])
def test_config_digests_small(gpu, name, radix_bits):
    import gpuradixsort_amd as grs

    rec = json.load(open(os.path.join(GOLDEN, "digests.json")))[name]
    n, kb, pairs = rec["n"], rec["key_bits"], rec["pairs"]
    k = torch.empty(n, dtype=torch.uint32, device=gpu)
    grs.fill_splitmix(k, rec["seed"])   # device generator == oracle generator
    assert np.array_equal(k.cpu().numpy(), oracle.splitmix_keys(n, kb, rec["seed"]))
    s = sorter(kb, pairs, radix_bits, n)
    v = None
    if pairs:
        v = torch.empty(n, dtype=torch.uint32, device=gpu)
        grs.iota_u32(v)
    s.sort(k, v)
    torch.cuda.synchronize()
    assert _digest(k.cpu().numpy()) == rec["sha256_keys"]
    if pairs:
        assert _digest(v.cpu().numpy()) == rec["sha256_perm"]


@pytest.mark.parametrize("name,radix_bits", [("ns_256m_u32", 8), ("c3_256m_u32_pairs", 8),
                                             ("c5_256m_u64", 8)])
def test_config_digests_full_size(gpu, name, radix_bits):
    """Full BASELINE sizes: exact SHA-256 of the expected output, plus the properties
    (sortedness via the device inversion counter)."""
    import gpuradixsort_amd as grs

    digests = json.load(open(os.path.join(GOLDEN, "digests.json")))
    if name not in digests:
        pytest.fail(f"{name} digest missing: run tests/golden/make_golden.py --large")
    rec = digests[name]
    n, kb, pairs = rec["n"], rec["key_bits"], rec["pairs"]
    dt = torch.uint32 if kb == 32 else torch.uint64
    k = torch.empty(n, dtype=dt, device=gpu)
    grs.fill_splitmix(k, rec["seed"])
    v = None
    if pairs:
        v = torch.empty(n, dtype=torch.uint32, device=gpu)
        grs.iota_u32(v)
    s = grs.RadixSorter(n, key_bits=kb, pairs=pairs, radix_bits=radix_bits)
    s.sort(k, v)
    torch.cuda.synchronize()
    s.check_error()
    assert grs.count_inversions(k) == 0
    assert _digest(k.cpu().numpy()) == rec["sha256_keys"]
    if pairs:
        assert _digest(v.cpu().numpy()) == rec["sha256_perm"]
    s.close()
    del k, v
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kb,pairs,rb,n", [(32, True, 8, 16384 * 256 + 13), (64, False, 8, 16384 * 256 + 13),
                                         (64, True, 8, 10240 * 256 + 13), (32, False, 8, 32768 * 256 + 13),
                                         (64, True, 4, 10240 * 256 + 13), (32, True, 4, 16384 * 256 + 13)])
def test_status_sizing_at_the_small_big_boundary(gpu, kb, pairs, rb, n):
    """Sizes just past (smaller big tile) x CUs, where the sort still takes small tiles: the
    look-back status was sized for fewer of them and the sort was refused (GRS_ECAPACITY) before
    round 6.  Default options, a sorter of exactly n, the stable sort out."""
    rng = np.random.default_rng(n + kb)
    dt = np.uint32 if kb == 32 else np.uint64
    keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
    keys[::7] = keys[3]
    import gpuradixsort_amd as grs

    s = grs.RadixSorter(n, key_bits=kb, pairs=pairs, radix_bits=rb)   # capacity exactly n
    k = to_dev(keys, gpu)
    v = to_dev(np.arange(n, dtype=np.uint32), gpu) if pairs else None
    s.sort(k, v)
    s.check_error()
    perm = np.argsort(keys, kind="stable")
    assert np.array_equal(k.cpu().numpy(), keys[perm])
    if pairs:
        assert np.array_equal(v.cpu().numpy(), perm.astype(np.uint32))
    assert s.check_guards() == 0
    s.close()


def test_capacity_and_argument_errors(gpu):
    import gpuradixsort_amd as grs

    s = grs.RadixSorter(1000, key_bits=32, pairs=False)
    k = torch.zeros(2000, dtype=torch.uint32, device=gpu)
    with pytest.raises(grs.GrsError, match="ECAPACITY"):
        s.sort(k)
    with pytest.raises(grs.GrsError, match="EINVAL"):
        s.sort(k, n=10, begin_bit=8, end_bit=8)
    s.sort(k, n=0)   # N = 0 is a no-op (PrefixSumSsbo.cpp:121-124)


def test_repeated_sorts_reuse_scratch(gpu):
    """Sort() twice on one controller (main.cpp:159-160): the second call must still be
    exact (status/ticket re-initialisation between calls)."""
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 2**32, 777_777, dtype=np.uint64).astype(np.uint32)
    perm = oracle.stable_argsort(keys)
    for _ in range(3):
        gk, gv = gpu_sort(keys, True, 8, gpu)
        assert np.array_equal(gv, perm)


def test_control_blocks_alternate_across_calls(gpu):
    """A sort launches no memset: its histogram kernel zeroes the OTHER of the sorter's two
    control blocks for the next call, and a partition (which clears and dirties the first
    block itself) makes the next sort clear it again.  Interleave sorts of different sizes,
    digit widths and bit ranges with partitions on one sorter, on one stream, without
    synchronising in between, and check every result."""
    import gpuradixsort_amd as grs

    rng = np.random.default_rng(12)
    s = grs.RadixSorter(300_000, key_bits=32, pairs=True, radix_bits=8)
    s4 = grs.RadixSorter(300_000, key_bits=32, pairs=True, radix_bits=4)
    jobs = []
    for step, n in enumerate((300_000, 1, 65_537, 0, 123_457, 300_000, 4_096)):
        keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        k = to_dev(keys, gpu)
        v = to_dev(np.arange(n, dtype=np.uint32), gpu)
        if step % 3 == 1:     # a bit-range sort (bits [8, 24))
            s.sort(k, v, begin_bit=8, end_bit=24)
            perm = np.argsort((keys >> 8) & 0xFFFF, kind="stable")
        elif step % 3 == 2:   # a partition, then a sort on the same sorter
            ko, vo = torch.empty_like(k), torch.empty_like(v)
            sp = np.sort(rng.integers(0, 2**32, 5, dtype=np.uint64).astype(np.uint32))
            cnt = torch.zeros(6, dtype=torch.uint32, device=gpu)
            s.partition(k, ko, sp, cnt, v, vo)
            bucket = np.searchsorted(sp, keys, side="right")
            jobs.append(("partition", ko, vo, keys, np.argsort(bucket, kind="stable")))
            s.sort(k, v)
            perm = np.argsort(keys, kind="stable")
        else:
            (s4 if step % 2 else s).sort(k, v)
            perm = np.argsort(keys, kind="stable")
        jobs.append(("sort", k, v, keys, perm))
    torch.cuda.synchronize()
    s.check_error()
    s4.check_error()
    for what, k, v, keys, perm in jobs:
        assert np.array_equal(k.cpu().numpy(), keys[perm]), what
        assert np.array_equal(v.cpu().numpy(), perm), what


@pytest.mark.parametrize("kb", [32, 64])
@pytest.mark.parametrize("pairs", [False, True])
def test_partition_is_stable_range_split(gpu, kb, pairs):
    """grs_partition (the multi-GPU exchange's local step): bucket = #splitters <= key,
    buckets contiguous in order, input order kept inside each bucket."""
    import gpuradixsort_amd as grs

    rng = np.random.default_rng(kb + pairs)
    dt = np.uint32 if kb == 32 else np.uint64
    for n, nsplit in ((1, 1), (1000, 3), (100_003, 7), (777_777, 15), (50_000, 0)):
        keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
        keys[::13] = np.iinfo(dt).max
        sp = np.sort(rng.choice(keys, nsplit)) if nsplit else np.zeros(0, dt)
        bucket = np.searchsorted(sp, keys, side="right")
        perm = np.argsort(bucket, kind="stable")
        s = grs.RadixSorter(n, key_bits=kb, pairs=pairs, radix_bits=8)
        k = to_dev(keys, gpu)
        ko = torch.empty_like(k)
        v = vo = None
        if pairs:
            v = to_dev(np.arange(n, dtype=np.uint32), gpu)
            vo = torch.empty_like(v)
        cnt = torch.zeros(nsplit + 1, dtype=torch.uint32, device=gpu)
        s.partition(k, ko, sp, cnt, v, vo)
        torch.cuda.synchronize()
        assert np.array_equal(cnt.cpu().numpy(), np.bincount(bucket, minlength=nsplit + 1))
        assert np.array_equal(ko.cpu().numpy(), keys[perm])
        if pairs:
            assert np.array_equal(vo.cpu().numpy(), perm)


@pytest.mark.parametrize("kb", [32, 64])
@pytest.mark.parametrize("pairs", [False, True])
def test_partition_regions_with_ties(gpu, kb, pairs):
    """grs_partition_regions (the exchange's send step): bucket b at keys_out[b * region], no
    bucket histogram; splitters with index thresholds split runs of equal keys, and splitter
    keys sharing a 12-bit prefix exercise the compares behind the LDS bucket table
    (SplitterIdxDigit::fill_lut).  Then a region too small: the count shows the spill."""
    import gpuradixsort_amd as grs

    rng = np.random.default_rng(100 + kb + pairs)
    dt = np.uint32 if kb == 32 else np.uint64
    sh = dt(kb - 12)
    for n, nsplit in ((1, 1), (5000, 3), (300_007, 7), (777_777, 15)):
        keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
        keys[::11] = keys[0]                              # a run of equal keys across buckets
        keys[1::17] = (dt(5) << sh) | dt(3)               # many keys in one shared prefix
        cand = np.concatenate([keys[:1], [(dt(5) << sh) | dt(3), (dt(5) << sh) | dt(1)],
                               rng.choice(keys, 16)]).astype(dt)
        sp = np.sort(rng.choice(cand, nsplit))
        th = rng.integers(0, n + 1, nsplit).astype(np.uint32)
        idx = np.arange(n, dtype=np.uint64)
        bucket = np.zeros(n, np.int64)
        for b in range(nsplit):
            bucket += (sp[b] < keys) | ((sp[b] == keys) & (th[b] <= idx))
        counts = np.bincount(bucket, minlength=nsplit + 1)
        region = int(counts.max()) + 64
        s = grs.RadixSorter(n, key_bits=kb, pairs=pairs, radix_bits=8)
        k = to_dev(keys, gpu)
        ko = torch.empty(nsplit * region + n, dtype=k.dtype, device=gpu)
        v = vo = None
        if pairs:
            v = to_dev(np.arange(n, dtype=np.uint32), gpu)
            vo = torch.empty(nsplit * region + n, dtype=torch.uint32, device=gpu)
        cnt = torch.zeros(nsplit + 1, dtype=torch.uint32, device=gpu)
        s.partition_regions(k, ko, sp, cnt, region, thresholds=th, vals=v, vals_out=vo)
        torch.cuda.synchronize()
        s.check_error()
        assert np.array_equal(cnt.cpu().numpy(), counts), n
        ko_h = ko.cpu().numpy()
        vo_h = vo.cpu().numpy() if pairs else None
        for b in range(nsplit + 1):
            sel = np.nonzero(bucket == b)[0]
            got = ko_h[b * region: b * region + sel.size]
            assert np.array_equal(got, keys[sel]), (n, b)
            if pairs:
                assert np.array_equal(vo_h[b * region: b * region + sel.size], sel.astype(np.uint32)), (n, b)
        if n > 1000:   # a region smaller than the largest bucket: its count says so
            small = int(counts.max()) - 1
            ko2 = torch.empty(nsplit * small + n, dtype=k.dtype, device=gpu)
            vo2 = torch.empty(nsplit * small + n, dtype=torch.uint32, device=gpu) if pairs else None
            s.partition_regions(k, ko2, sp, cnt, small, thresholds=th, vals=v, vals_out=vo2)
            torch.cuda.synchronize()
            s.check_error()
            c2 = cnt.cpu().numpy()
            assert np.array_equal(c2, counts) and int(c2.max()) > small
        s.close()
