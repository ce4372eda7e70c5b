"""GPU parity of the §8f extensions, through the C-ABI:

  * grs_exclusive_scan_u32  vs the restated reference scan (K3a + K3b, oracle.ref_device_scan)
                            for N <= 2^20, the PrefixScan.xlsx KAT, and numpy cumsum mod 2^32
                            beyond the reference's capacity
  * grs_key_transform       signed / float keys sorted through the unsigned sort vs numpy's
                            order of the original values (parity unpinned: the reference has
                            no signed or float keys, ReadMeRadixSort.txt:71-80)
  * grs_sort_segmented      vs per-segment numpy stable argsort (parity unpinned: the
                            reference has no segmented sort)
Bit-exact throughout (integer work).
"""
import json
import os

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cumsum_excl(a: np.ndarray):
    c = np.cumsum(a.astype(np.uint64)) - a.astype(np.uint64)
    return (c & 0xFFFFFFFF).astype(np.uint32), int(a.astype(np.uint64).sum() & 0xFFFFFFFF)


def gpu_scan(a: np.ndarray, dev, in_place=False):
    import gpuradixsort_amd as grs

    x = torch.from_numpy(a.view(np.int32).copy()).to(dev)
    total = torch.full((1,), -1, dtype=torch.int32, device=dev)
    out = grs.exclusive_scan_u32(x, x if in_place else None, total=total)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32), int(total.cpu().numpy().view(np.uint32)[0])


def test_scan_xlsx_kat(gpu):
    kat = json.load(open(os.path.join(GOLDEN, "prefix_scan_xlsx.json")))
    out, total = gpu_scan(np.asarray(kat["input"], dtype=np.uint32), gpu)
    assert out.tolist() == kat["exclusive_scan"]
    assert total == kat["total"]


@pytest.mark.parametrize("n", [1, 2, 1023, 1024, 1025, 4095, 4096, 4097, 65537, 1 << 20])
def test_scan_vs_reference_restatement(gpu, n):
    rng = np.random.default_rng(n)
    for a in (rng.integers(0, 2, n, dtype=np.uint32),                 # the reference's 0/1 bits
              rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)):  # wraps mod 2^32
        want, wtot = oracle.ref_device_scan(a)
        out, total = gpu_scan(a, gpu)
        assert np.array_equal(out, want)
        assert total == wtot


@pytest.mark.parametrize("n", [(1 << 22) - 1, 1 << 22, (1 << 24) + 5, 100_000_007])
def test_scan_large_in_place(gpu, n):
    """In place, around and above the switch from 8K- to 32K-item tiles (2^22 items)."""
    rng = np.random.default_rng(7)
    a = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want, wtot = cumsum_excl(a)
    out, total = gpu_scan(a, gpu, in_place=True)
    assert np.array_equal(out, want)
    assert total == wtot


def test_scan_empty_and_all_max(gpu):
    out, total = gpu_scan(np.zeros(0, dtype=np.uint32), gpu)
    assert out.size == 0 and total == 0
    a = np.full(300_001, 0xFFFFFFFF, dtype=np.uint32)
    out, total = gpu_scan(a, gpu)
    want, wtot = cumsum_excl(a)
    assert np.array_equal(out, want) and total == wtot


# ---- key transforms ----------------------------------------------------------------------

def sort_transformed(a: np.ndarray, dev):
    """a (signed / float numpy array) -> sorted through transform + unsigned sort + inverse,
    plus the stable permutation."""
    import gpuradixsort_amd as grs

    bits = a.dtype.itemsize * 8
    t = torch.from_numpy(a.copy()).to(dev)
    u = t.view(torch.int32 if bits == 32 else torch.int64)
    grs.key_transform(t)
    s = grs.RadixSorter(max(a.size, 1), key_bits=bits, pairs=True)
    v = torch.arange(a.size, dtype=torch.int32, device=dev)
    s.sort(u, v)
    grs.key_transform(t, inverse=True)
    torch.cuda.synchronize()
    s.check_error()
    s.close()
    return t.cpu().numpy(), v.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("dtype", [np.int32, np.int64, np.float32, np.float64])
def test_key_transform_sort(gpu, dtype):
    rng = np.random.default_rng(3)
    n = 300_017
    if np.dtype(dtype).kind == "i":
        info = np.iinfo(dtype)
        a = rng.integers(info.min, info.max, n, dtype=dtype, endpoint=True)
        a[:5] = [info.min, info.max, 0, -1, 1]
    else:
        a = (rng.standard_normal(n) * 1e6).astype(dtype)
        a[::97] = a[::97].round()          # ties
        a[:6] = [np.inf, -np.inf, 0.0, -0.0, np.finfo(dtype).tiny, -np.finfo(dtype).max]
    out, perm = sort_transformed(a, gpu)
    order = np.argsort(oracle.key_transform_np(a), kind="stable")
    assert np.array_equal(out.view(np.uint8), a[order].view(np.uint8))   # bit-exact
    assert np.array_equal(perm, order.astype(np.uint32))
    # and the values are in numpy's numeric order (no NaNs here; -0 sorts before +0)
    assert np.array_equal(out, np.sort(a, kind="stable"))


def test_key_transform_nan_and_roundtrip(gpu):
    import gpuradixsort_amd as grs

    a = np.array([1.0, np.nan, -np.nan, -np.inf, np.inf, -0.0, 0.0, -2.5], dtype=np.float32)
    out, _ = sort_transformed(a, gpu)
    bits = out.view(np.uint32)
    assert np.isnan(out[0]) and np.signbit(out[0])       # -NaN first
    assert np.isnan(out[-1]) and not np.signbit(out[-1])  # +NaN last
    assert out[1] == -np.inf and out[-2] == np.inf
    assert out[2] == -2.5 and bits[3] == 0x80000000 and bits[4] == 0   # -0 before +0
    # transform + inverse is the identity on every bit pattern
    x = torch.from_numpy(np.random.default_rng(1).integers(0, 2**32, 1 << 16, dtype=np.uint64)
                         .astype(np.uint32).view(np.float32)).to(gpu)
    y = x.clone()
    grs.key_transform(y)
    grs.key_transform(y, inverse=True)
    assert torch.equal(x.view(torch.int32), y.view(torch.int32))


# ---- segmented sort ------------------------------------------------------------------------

def random_offsets(n, nseg, rng, empty=True):
    cuts = np.sort(rng.integers(0, n + 1, nseg - 1))
    off = np.concatenate([[0], cuts, [n]]).astype(np.uint32)
    if empty and nseg > 3:
        off[2] = off[1]                  # an empty segment
    return off


@pytest.mark.parametrize("kb", [32, 64])
@pytest.mark.parametrize("n,nseg", [(1, 1), (1000, 1), (100_003, 7), (300_000, 4096),
                                    (1 << 20, 100_000), (300_000, 200)])
def test_segmented_sort(gpu, kb, n, nseg):
    import gpuradixsort_amd as grs

    rng = np.random.default_rng(n + nseg + kb)
    dt = np.uint32 if kb == 32 else np.uint64
    keys = rng.integers(0, 1 << 12, n, dtype=dt)       # many ties: stability matters
    vals = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    off = random_offsets(n, nseg, rng)
    want_k, want_v = oracle.segmented_sort_np(keys, off, vals)
    s = grs.RadixSorter(n, key_bits=kb, pairs=True)
    k = torch.from_numpy(keys.view(np.int32 if kb == 32 else np.int64).copy()).to(gpu)
    v = torch.from_numpy(vals.view(np.int32).copy()).to(gpu)
    o = torch.from_numpy(off.view(np.int32)).to(gpu)
    s.sort_segmented(k, o, v)
    torch.cuda.synchronize()
    s.check_error()
    assert np.array_equal(k.cpu().numpy().view(dt), want_k)
    assert np.array_equal(v.cpu().numpy().view(np.uint32), want_v)
    # keys only (no payload pointer) gives the same keys
    k2 = torch.from_numpy(keys.view(np.int32 if kb == 32 else np.int64).copy()).to(gpu)
    s.sort_segmented(k2, o)
    torch.cuda.synchronize()
    assert np.array_equal(k2.cpu().numpy().view(dt), want_k)
    s.close()


@pytest.mark.parametrize("rank", ["probe", "match"])
@pytest.mark.parametrize("kb", [32, 64])
@pytest.mark.parametrize("lengths", [[4096] * 5, [4095, 1, 2, 3, 4096, 0, 17], [4096, 4097, 5],
                                     [300, 1000, 513, 2, 0, 1024, 511],
                                     [16384, 9000, 8192, 1, 8193], [16385, 3]],
                         ids=["all_4096", "ragged", "one_4097", "mixed_bounds", "to_16k", "one_16385"])
def test_segmented_sort_short_segment_bound(gpu, kb, lengths, rank):
    """Segments at the LDS paths' bounds (4096 items for the bitonic fallback, 16384 / 8192 for the
    block radix sort of u32 / u64 keys), ragged and empty ones, lengths around every LDS size,
    and one item past a bound (the general path takes the whole call); rank "probe" = the block
    radix sort (lane-ordered LDS atomics, probed), "match" = the bitonic fallback."""
    import gpuradixsort_amd as grs

    rng = np.random.default_rng(sum(lengths) + kb)
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.uint32)
    n = int(off[-1])
    dt = np.uint32 if kb == 32 else np.uint64
    keys = rng.integers(0, 64, n, dtype=dt)              # heavy ties
    keys[::5] = np.iinfo(dt).max                         # the largest key beside the padding
    vals = np.arange(n, dtype=np.uint32)
    want_k, want_v = oracle.segmented_sort_np(keys, off, vals)
    s = grs.RadixSorter(n, key_bits=kb, pairs=True, options={"rank": rank})
    k = torch.from_numpy(keys.view(np.int32 if kb == 32 else np.int64).copy()).to(gpu)
    v = torch.from_numpy(vals.view(np.int32).copy()).to(gpu)
    o = torch.from_numpy(off.view(np.int32)).to(gpu)
    s.sort_segmented(k, o, v)
    torch.cuda.synchronize()
    s.check_error()
    assert np.array_equal(k.cpu().numpy().view(dt), want_k)
    assert np.array_equal(v.cpu().numpy().view(np.uint32), want_v)
    s.close()


# tile of the segmented onesweep pass (grs_capi.hip BigTile: 1024 threads x ITEMS) per
# (key bits, payload); look-back groups are GRS_LB_GROUP = 8 tiles
SEG_TILE = {(32, True): 1024 * 17, (32, False): 1024 * 36, (64, True): 1024 * 22, (64, False): 1024 * 17}


@pytest.mark.parametrize("path", ["default", "lsd"])
@pytest.mark.parametrize("pairs", [True, False], ids=["pairs", "keys"])
@pytest.mark.parametrize("kb", [32, 64])
@pytest.mark.parametrize("case", ["tile_edges", "group_edges", "one_long_many_short", "two_segments",
                                  "skewed_runs"])
def test_segmented_sort_long_segments(gpu, kb, pairs, case, path):
    """Segments longer than the LDS sorts take: lengths at the 16K LDS bound, one tile (solo,
    no look-back) and one past it, two tiles, at and around a look-back group of 8 tiles,
    empty segments between, against oracle.segmented_sort_np; full-range keys with a
    heavy-tie subset so every byte and the stability matter.  Path "default": segments of 4K
    keys and more on average take the top-byte scatter + LDS sorts (grs_seg_runs: merged
    runs, the primary and mid shapes, the segmented-LSD fallback for runs past LDS, which
    "skewed_runs" reaches with a 200K-key run); "lsd" (GRS_OPT_MSD = never): the segmented LSD
    (grs_seg_plan, grs_seg_hist, one grs_onesweep_seg launch per byte)."""
    import gpuradixsort_amd as grs

    T = SEG_TILE[(kb, pairs)]
    dt = np.uint32 if kb == 32 else np.uint64
    top = dt(kb - 8)
    skew = None
    if case == "tile_edges":
        lengths = [16384, 16385, T - 1, T, 0, T + 1, 2 * T, 2 * T + 1, 1, 0, 3 * T - 7]
    elif case == "group_edges":
        lengths = [8 * T - 1, 8 * T, 0, 8 * T + 1, 9 * T + 5, 17 * T + 3]
    elif case == "one_long_many_short":
        lengths = [3] * 20000 + [5 * T + 11] + [0, 1, 2] * 3000
    elif case == "two_segments":
        lengths = [1, 40 * T + 99]
    else:
        # top bytes per segment: six runs of 10000 (the mid shape), one run of 200000 (the
        # fallback, several tiles), uniform (merged runs), two runs of 15000
        lengths = [60000, 200000, 5000, 30000]
        skew = [np.repeat(np.arange(6), 10000), np.full(200000, 0x41), None, np.repeat([0x80, 0x81], 15000)]
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.uint32)
    n = int(off[-1])
    rng = np.random.default_rng(n + kb + pairs)
    keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
    ties = rng.random(n) < 0.4
    keys[ties] = rng.integers(0, 16, int(ties.sum())).astype(dt) * (np.iinfo(dt).max // dt(15))
    if skew is not None:
        for i, tb in enumerate(skew):
            if tb is not None:
                seg = slice(int(off[i]), int(off[i + 1]))
                low = keys[seg] & ((dt(1) << top) - dt(1))
                keys[seg] = (rng.permutation(tb).astype(dt) << top) | low
    vals = np.arange(n, dtype=np.uint32)
    want_k, want_v = oracle.segmented_sort_np(keys, off, vals)
    s = grs.RadixSorter(n, key_bits=kb, pairs=True)
    if path == "lsd":
        s.set_option("msd", "never")
    k = torch.from_numpy(keys.view(np.int32 if kb == 32 else np.int64).copy()).to(gpu)
    v = torch.from_numpy(vals.view(np.int32).copy()).to(gpu) if pairs else None
    o = torch.from_numpy(off.view(np.int32)).to(gpu)
    for rep in range(2):                 # the second call reuses the planner's scratch
        if rep:
            k.copy_(torch.from_numpy(keys.view(np.int32 if kb == 32 else np.int64).copy()))
            if pairs:
                v.copy_(torch.from_numpy(vals.view(np.int32).copy()))
        s.sort_segmented(k, o, v)
        torch.cuda.synchronize()
        s.check_error()
        assert np.array_equal(k.cpu().numpy().view(dt), want_k), (case, rep)
        if pairs:
            assert np.array_equal(v.cpu().numpy().view(np.uint32), want_v), (case, rep)
    s.close()


def test_segmented_sort_needs_payload_sorter(gpu):
    import gpuradixsort_amd as grs

    s = grs.RadixSorter(16, key_bits=32, pairs=False)
    k = torch.zeros(16, dtype=torch.int32, device=gpu)
    o = torch.tensor([0, 16], dtype=torch.int32, device=gpu)
    with pytest.raises(ValueError):
        s.sort_segmented(k, o)
    s.close()


# ---- host-buffer sort (BASELINE C1 plumbing) ------------------------------------------------

def test_sort_host_c1_matches_reference_path(gpu):
    """C1: 64K uniform u32 keys through grs_sort_host == the restated reference path."""
    import gpuradixsort_amd as grs

    keys = oracle.splitmix_keys(65536, 32, oracle.config_seed(1))
    want_k, want_p = oracle.ref_parallel_sort(keys)
    s = grs.RadixSorter(65536, key_bits=32, pairs=True)
    k = keys.copy()
    v = np.arange(k.size, dtype=np.uint32)
    s.sort_host(k, v)
    assert np.array_equal(k, want_k) and np.array_equal(v, want_p)
    s.close()
    s = grs.RadixSorter(65536, key_bits=32)
    k = keys.copy()
    s.sort_host(k)
    assert np.array_equal(k, want_k)
    with pytest.raises(ValueError):
        s.sort_host(k, v)          # payload on a keys-only sorter
    s.close()


def test_sort_host_u64_and_empty(gpu):
    import gpuradixsort_amd as grs

    keys = oracle.splitmix_keys(300_001, 64, oracle.config_seed(5))
    s = grs.RadixSorter(keys.size, key_bits=64)
    k = keys.copy()
    s.sort_host(k)
    assert np.array_equal(k, np.sort(keys))
    s.sort_host(np.zeros(0, dtype=np.uint64))
    s.close()


@pytest.mark.parametrize("kb", [32, 64])
def test_sort_host_segmented_sort_host_on_one_sorter(gpu, kb):
    """Scratch ownership of one pair sorter across entry points (the round-1 advisor's
    use-after-free): grs_sort_host -> grs_sort_segmented -> grs_sort_host -> destroy, each
    result bit-exact."""
    import gpuradixsort_amd as grs

    dt = np.uint32 if kb == 32 else np.uint64
    rng = np.random.default_rng(kb)
    n = 300_007
    s = grs.RadixSorter(n, key_bits=kb, pairs=True)
    for rnd in range(2):
        keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
        keys[::9] = 3
        vals = np.arange(n, dtype=np.uint32)
        perm = oracle.stable_argsort(keys)
        hk, hv = keys.copy(), vals.copy()
        s.sort_host(hk, hv)
        assert np.array_equal(hk, keys[perm]) and np.array_equal(hv, perm), rnd
        # segmented sort on the same sorter (allocates its own scratch)
        offs = np.array([0, 1000, 1000, 77_777, n], np.uint32)
        k = torch.from_numpy(keys).to(gpu)
        v = torch.from_numpy(vals).to(gpu)
        o = torch.from_numpy(offs).to(gpu)
        s.sort_segmented(k, o, v)
        s.check_error()
        exp_k, exp_v = keys.copy(), vals.copy()
        for a, b in zip(offs[:-1], offs[1:]):
            p = oracle.stable_argsort(keys[a:b])
            exp_k[a:b], exp_v[a:b] = keys[a:b][p], vals[a:b][p]
        assert np.array_equal(k.cpu().numpy(), exp_k) and np.array_equal(v.cpu().numpy(), exp_v)
        hk, hv = keys.copy(), vals.copy()
        s.sort_host(hk, hv)
        assert np.array_equal(hk, keys[perm]) and np.array_equal(hv, perm), rnd
    s.close()


def test_stream_check_error_and_checked_facade(gpu):
    """grs_stream_check_error on a clean stream returns OK (the look-back never timed out);
    the checked facades (ParallelSort.Sort) go through it."""
    import gpuradixsort_amd as grs

    st = torch.cuda.Stream()
    s = grs.RadixSorter(1 << 20, key_bits=32)
    k = torch.empty(1 << 20, dtype=torch.uint32, device=gpu)
    grs.fill_splitmix(k, 17)
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        s.sort(k, stream=st)
        s.check_error(st)
    assert grs.count_inversions(k) == 0
    s.check_error(device_wide=True)
    ssbo = grs.OriginalDataSsbo(1000)
    ssbo.Upload(np.arange(1000)[::-1].copy())
    grs.ParallelSort(ssbo).Sort()
    assert ssbo.Download().numpy().tolist() == list(range(1000))
