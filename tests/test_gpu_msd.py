"""GPU tests of the MSD-first sort (grs_msd.hpp; GRS_OPT_MSD): u32 keys, u32 pairs, u64 keys.

The MSD sort is a different schedule of the same stable sort: two stable scatters by the top
two bytes, then each 16-bit segment sorted by its low 16 bits in LDS, and a segmented LSD for
segments longer than LDS takes.  Its output must equal the reference's (the stable sort by key,
ParallelSort.cpp:236-298 restated by oracle.ref_parallel_sort) bit for bit.  Keys only: the MSD
path is the u32 keys-without-payload sort, so the check is the sorted multiset -- the same
output order as the reference's path, which test_u32_matches_reference_path pins for the LSD
schedule.

Every sort here is followed by the sorter's guard-band check (grs_debug_check_guards): the
scratch arrays the MSD kernels write (second buffer, region buffer, tables, status buffers)
end in guard bands, and a kernel that writes past one fails the test even when its output
happens to come out right (round 5's P2 region spill did exactly that).
"""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

_S = {}


def msd_sorter(capacity, mode="always", key_bits=32, pairs=False):
    import gpuradixsort_amd as grs

    key = (mode, key_bits, pairs)
    s = _S.get(key)
    if s is None or s.capacity < capacity:
        if s is not None:
            s.close()
            _S.pop(key)
        for other in list(_S):   # one sorter at a time of the large ones (HBM)
            if _S[other].capacity >= (1 << 26):
                _S.pop(other).close()
        s = grs.RadixSorter(max(capacity, 1 << 20), key_bits=key_bits, pairs=pairs, radix_bits=8)
        s.set_option("msd", mode)
        _S[key] = s
    return s


def run(keys: np.ndarray, dev, mode="always"):
    s = msd_sorter(keys.size, mode)
    k = torch.from_numpy(np.ascontiguousarray(keys)).to(dev)
    s.sort(k)
    torch.cuda.synchronize()
    s.check_error()
    assert s.check_guards() == 0, "a kernel wrote past a scratch array (guard band)"
    return k.cpu().numpy()


def dists(n, rng):
    top = 0xFFFFFFFF
    yield "uniform", rng.integers(0, top, n, dtype=np.uint32, endpoint=True)
    yield "perm", rng.permutation(n).astype(np.uint32)
    yield "all_equal", np.full(n, 7, np.uint32)
    yield "all_max", np.full(n, top, np.uint32)
    yield "sorted", np.sort(rng.integers(0, top, n, dtype=np.uint32, endpoint=True))
    yield "reversed", np.arange(n, 0, -1).astype(np.uint32)
    yield "16_unique", (rng.integers(0, 16, n).astype(np.uint32) * np.uint32(0x10000001))
    yield "mixed_max", np.where(rng.random(n) < 0.3, top, rng.integers(0, 100, n)).astype(np.uint32)
    yield "low_entropy", (rng.integers(0, top, n, dtype=np.uint32, endpoint=True)
                          & rng.integers(0, top, n, dtype=np.uint32, endpoint=True)
                          & rng.integers(0, top, n, dtype=np.uint32, endpoint=True))
    yield "narrow_24bit", rng.integers(0, 1 << 24, n, dtype=np.uint32)
    yield "narrow_29bit", rng.integers(0, 1 << 29, n, dtype=np.uint32)


PIECE = 256   # keys of one piece of H2's sample (2^GRS_H2_PIECE_LOG, grs_msd.hpp)

SIZES = [1, 2, 3, 64, 1000, 4097, 5121, 36865, 65537, 300007, 1 << 20]


@pytest.mark.parametrize("n", SIZES)
def test_msd_matches_reference_path(gpu, n):
    """Forced MSD schedule, every distribution: keys == the restated reference path."""
    rng = np.random.default_rng(5000 + n)
    for name, keys in dists(n, rng):
        if n > 65537 and name not in ("uniform", "perm", "16_unique", "mixed_max", "narrow_29bit"):
            continue
        want = oracle.ref_parallel_sort(keys)[0]
        got = run(keys, gpu)
        assert np.array_equal(got, want), f"{name} n={n}"


def _segment_keys(rng, sizes):
    """Keys whose 16-bit prefixes p_i hold exactly sizes[i] keys each (random low halves),
    shuffled: exercises P3's capacity edge and the fallback (solo and multi-tile segments)."""
    parts = []
    for i, c in enumerate(sizes):
        prefix = np.uint32((i * 2654435761) & 0xFFFF) << np.uint32(16)
        parts.append(prefix | rng.integers(0, 1 << 16, c, dtype=np.uint32))
    keys = np.concatenate(parts)
    rng.shuffle(keys)
    # one key of prefix 0xFFFF at the end: the keys vary in their top bit, so the MSD digits
    # stay the top two bytes (the span-adaptive digit would otherwise move below a constant top)
    return np.append(keys, np.uint32(0xFFFFFFFF))


@pytest.mark.parametrize("sizes", [
    [5120, 5121, 1, 2, 4096],                  # P3 shape A edge (n < 2^26: shape A)
    [5121] * 7 + [100],                        # solo fallback segments
    [36864, 36865, 73729, 200000, 3],          # one-tile, two-tile and multi-tile fallbacks
    [1 << 20],                                 # one segment of everything
    [6000, 10000, 18432, 18433, 100],          # the mid list (the larger LDS shape) and past it
])
def test_msd_segment_edges(gpu, sizes):
    rng = np.random.default_rng(sum(sizes))
    keys = _segment_keys(rng, sizes)
    got = run(keys, gpu)
    assert np.array_equal(got, np.sort(keys))


@pytest.mark.parametrize("pairs", [False, True])
def test_msd_persistent_p3_option(gpu, pairs):
    """Option p3=persistent (grs_msd_local_pf, an A/B variant): the same keys and permutation as
    the stable sort, through the mid and big lists and at a size with many segments."""
    import gpuradixsort_amd as grs

    rng = np.random.default_rng(77 + pairs)
    cases = [_segment_keys(rng, [5120, 5121, 1, 2, 4096]),
             _segment_keys(rng, [6000, 10000, 18432, 18433, 100, 36865]),
             rng.integers(0, 1 << 32, (1 << 22) + 3, dtype=np.uint64).astype(np.uint32)]
    s = grs.RadixSorter(1 << 23, key_bits=32, pairs=pairs, radix_bits=8)
    s.set_option("msd", "always")
    s.set_option("p3", "persistent")
    for keys in cases:
        k = torch.from_numpy(keys).to(gpu)
        v = torch.arange(keys.size, dtype=torch.int64, device=gpu).to(torch.uint32) if pairs else None
        s.sort(k, v)
        s.check_error()
        perm = np.argsort(keys, kind="stable")
        assert np.array_equal(k.cpu().numpy(), keys[perm])
        if pairs:
            assert np.array_equal(v.cpu().numpy(), perm.astype(np.uint32))
    assert s.check_guards() == 0
    s.close()


@pytest.mark.parametrize("n", [1 << 24, (1 << 26) + 12345])
def test_msd_larger(gpu, n):
    """Sizes where the MSD schedule is (or is about to be) the default: uniform and narrow
    ranges, by the default option and forced, against torch.sort."""
    rng = np.random.default_rng(n)
    for name, keys in (("uniform", rng.integers(0, 1 << 32, n, dtype=np.uint32)),
                       ("narrow_27bit", rng.integers(0, 1 << 27, n, dtype=np.uint32)),
                       ("16_unique", rng.integers(0, 16, n).astype(np.uint32) << np.uint32(28))):
        k = torch.from_numpy(keys).to(gpu)
        want = torch.sort(k.view(torch.int32).to(torch.int64) & 0xFFFFFFFF)[0]
        for mode in ("size", "always"):
            got = run(keys, gpu, mode)
            assert np.array_equal(got.astype(np.int64), want.cpu().numpy()), (name, mode)


def test_msd_profile_kind(gpu):
    """The profiled MSD sort reports its phases (grs_timing.kind = 1)."""
    s = msd_sorter(1 << 22)
    s.set_profiling(1)
    k = torch.randint(0, 1 << 31, (1 << 22,), dtype=torch.int64, device=gpu).to(torch.int32)
    s.sort(k.view(torch.uint32))
    t = s.timing()
    s.set_profiling(0)
    assert t["kind"] == "msd" and t["passes"] == 6, t
    assert all(x >= 0 for x in t["pass_ms"]) and t["total_ms"] > 0


def test_msd_region_spill_redo(gpu):
    """The first scatter writes each top-byte run into a region sized from a sample of 2^20
    keys (64-key chunks at evenly spaced positions).  Keys that put every sampled chunk in
    bucket 0 and everything else in bucket 255 make bucket 255's run outgrow its region: the
    sort must detect it and redo the scatter with exact counts (grs_msd_redo_plan), bit-exact."""
    n = 1 << 22
    chunks, w = 16384, 64
    rng = np.random.default_rng(77)
    keys = (np.uint32(0xFF) << np.uint32(24)) | rng.integers(0, 1 << 24, n, dtype=np.uint32)
    pos = (np.arange(chunks, dtype=np.uint64) * np.uint64(n - w) // np.uint64(chunks - 1)).astype(np.int64)
    idx = (pos[:, None] + np.arange(w)[None, :]).ravel()
    keys[idx] = rng.integers(0, 1 << 24, idx.size, dtype=np.uint32)   # bucket 0
    got = run(keys, gpu)
    assert np.array_equal(got, np.sort(keys))
    # and the sorter keeps working (the spill flag lives in the per-call control block)
    keys2 = rng.integers(0, 1 << 32, n, dtype=np.uint32)
    assert np.array_equal(run(keys2, gpu), np.sort(keys2))


def test_msd_p1_region_spill_stays_in_bounds(gpu):
    """7120 keys of top byte 0xFF where the sample never looks: digit 255's P1 region (4096 keys,
    the last region, ending 1024 elements before the second buffer does) is outgrown by ~3000
    keys.  The run clamp must hold the run inside the buffer (guard bands intact: a build
    without the clamp overwrites them, tools/diag/canary_no_clamp.py) and the exact redo must
    sort it -- keys only and u32 pairs."""
    import gpuradixsort_amd as grs

    n, chunks = 1 << 22, 16384
    rng = np.random.default_rng(4243)
    keys = rng.integers(0, 0xFF000000, n, dtype=np.uint64).astype(np.uint32)
    starts = (np.arange(chunks, dtype=np.uint64) * np.uint64(n - 64) // np.uint64(chunks - 1)).astype(np.int64)
    seen = np.zeros(n, bool)
    seen[(starts[:, None] + np.arange(64)[None, :]).ravel()] = True
    hot = rng.choice(np.flatnonzero(~seen), 4096 + 3024, replace=False)
    keys[hot] = np.uint32(0xFF000000) | rng.integers(0, 1 << 24, hot.size, dtype=np.uint32)
    perm = np.argsort(keys, kind="stable")
    for pairs in (False, True):
        s = grs.RadixSorter(n, key_bits=32, pairs=pairs, radix_bits=8)   # capacity n: regions fill alt
        s.set_option("msd", "always")
        k = torch.from_numpy(keys).to(gpu)
        v = torch.arange(n, dtype=torch.int32, device=gpu).view(torch.uint32) if pairs else None
        s.sort(k, v)
        s.check_error()
        assert s.check_guards() == 0, pairs
        assert np.array_equal(k.cpu().numpy(), keys[perm]), pairs
        if pairs:
            assert np.array_equal(v.cpu().numpy(), perm.astype(np.uint32))
        s.close()


def run_typed(keys: np.ndarray, dev, pairs: bool, mode="always"):
    kb = keys.dtype.itemsize * 8
    s = msd_sorter(keys.size, mode, kb, pairs)
    k = torch.from_numpy(np.ascontiguousarray(keys)).to(dev)
    v = torch.arange(keys.size, dtype=torch.int64, device=dev).to(torch.int32).view(torch.uint32) if pairs else None
    s.sort(k, v)
    torch.cuda.synchronize()
    s.check_error()
    assert s.check_guards() == 0, "a kernel wrote past a scratch array (guard band)"
    return k.cpu().numpy(), (v.cpu().numpy() if pairs else None)


@pytest.mark.parametrize("n", [1, 2, 64, 4097, 5121, 65537, 300007, 1 << 20])
def test_msd_pairs_match_reference_path(gpu, n):
    """u32 keys + u32 payload (the reference's IntermediateData {key, index}): keys AND the
    stable permutation == the restated reference path (ParallelSort.cpp:236-298)."""
    rng = np.random.default_rng(6000 + n)
    for name, keys in dists(n, rng):
        if n > 65537 and name not in ("uniform", "perm", "16_unique", "mixed_max"):
            continue
        rk, rp = oracle.ref_parallel_sort(keys)
        gk, gv = run_typed(keys, gpu, True)
        assert np.array_equal(gk, rk), f"{name} n={n}: keys"
        assert np.array_equal(gv, rp), f"{name} n={n}: permutation (stability)"


@pytest.mark.parametrize("n", [1, 3, 64, 4097, 5121, 65537, 300007, 1 << 20])
def test_msd_u64_matches_stable_sort(gpu, n):
    """u64 keys (6 LDS rounds below the 16-bit prefix; 6-pass segmented fallback)."""
    rng = np.random.default_rng(7000 + n)
    top = np.iinfo(np.uint64).max
    cases = [("uniform", rng.integers(0, top, n, dtype=np.uint64, endpoint=True)),
             ("all_equal", np.full(n, 9, np.uint64)),
             ("16_unique", rng.integers(0, 16, n).astype(np.uint64) * np.uint64(0x1000000000000001)),
             ("narrow_40bit", rng.integers(0, 1 << 40, n, dtype=np.uint64)),
             ("mixed_max", np.where(rng.random(n) < 0.3, top, rng.integers(0, 100, n)).astype(np.uint64))]
    for name, keys in cases:
        gk, _ = run_typed(keys, gpu, False)
        assert np.array_equal(gk, np.sort(keys)), f"{name} n={n}"


@pytest.mark.parametrize("kb,pairs", [(32, True), (64, False)])
def test_msd_typed_segment_edges_and_spill(gpu, kb, pairs):
    """The fallback (solo and multi-tile segments) and the region redo for u32 pairs and u64."""
    rng = np.random.default_rng(kb + pairs)
    dt = np.uint32 if kb == 32 else np.uint64
    sizes = [5120, 5121, 10240, 10241, 17408, 17409, 40000, 3]
    parts = []
    for i, c in enumerate(sizes):
        prefix = dt((i * 2654435761) & 0xFFFF) << dt(kb - 16)
        parts.append(prefix | rng.integers(0, 1 << 16, c).astype(dt))
    keys = np.concatenate(parts)
    rng.shuffle(keys)
    gk, gv = run_typed(keys, gpu, pairs)
    perm = oracle.stable_argsort(keys)
    assert np.array_equal(gk, keys[perm])
    if pairs:
        assert np.array_equal(gv, perm.astype(np.uint32))
    # region spill: sampled chunks in bucket 0, the rest in bucket 255
    n, chunks, w = 1 << 22, 16384, 64
    keys = (dt(0xFF) << dt(kb - 8)) | rng.integers(0, 1 << 24, n).astype(dt)
    pos = (np.arange(chunks, dtype=np.uint64) * np.uint64(n - w) // np.uint64(chunks - 1)).astype(np.int64)
    idx = (pos[:, None] + np.arange(w)[None, :]).ravel()
    keys[idx] = rng.integers(0, 1 << 24, idx.size).astype(dt)
    gk, gv = run_typed(keys, gpu, pairs)
    perm = oracle.stable_argsort(keys)
    assert np.array_equal(gk, keys[perm])
    if pairs:
        assert np.array_equal(gv, perm.astype(np.uint32))


@pytest.mark.parametrize("n", [(1 << 27) + 77, 1 << 28])
def test_msd_sampled_p2(gpu, n):
    """Sorts large enough that H2 counts a sample of P1's output (one 256-key piece in 2 / 4) and
    P2 scatters into regions sized from it (grs_msd_plan3), P3 reading the region buffer:
    uniform, narrow (few top-byte buckets, long regions), few-unique and sorted keys."""
    rng = np.random.default_rng(n)
    cases = (("uniform", rng.integers(0, 1 << 32, n, dtype=np.uint32)),
             ("narrow_27bit", rng.integers(0, 1 << 27, n, dtype=np.uint32)),
             ("16_unique", rng.integers(0, 16, n).astype(np.uint32) * np.uint32(0x10001001)),
             ("sorted", (np.arange(n, dtype=np.uint64) * 15).astype(np.uint32)))
    for name, keys in cases:
        k = torch.from_numpy(keys).to(gpu)
        want = torch.sort(k.view(torch.int32).to(torch.int64) & 0xFFFFFFFF)[0].cpu().numpy()
        got = run(keys, gpu, "always")
        assert np.array_equal(got.astype(np.int64), want), name
        del k


def test_msd_p2_region_spill(gpu):
    """A sample that misses a bin: every key in top-byte bucket 0 and, by 256-key piece of P1's
    output (2^GRS_H2_PIECE_LOG), byte 2 = 0 in the sampled pieces (even ones: one in two is sampled at 2^27) and 255
    in the others, so bin (0, 255) outgrows its region: P2's last tiles flag it, the exact
    histogram and pass run (gated on the flag) and P3 sorts in place -- bit-exact, and the
    sorter's next sort is too."""
    n = 1 << 27
    rng = np.random.default_rng(31)
    piece = (np.arange(n, dtype=np.int64) // PIECE) % 2
    keys = np.where(piece == 0, 0, 255).astype(np.uint32) << np.uint32(16)
    keys |= rng.integers(0, 1 << 16, n, dtype=np.uint32)
    keys[-1] |= np.uint32(1 << 31)   # the top byte varies: P1 / P2 stay on bytes 3 / 2
    got = run(keys, gpu, "always")
    assert np.array_equal(got, np.sort(keys))
    keys2 = rng.integers(0, 1 << 32, n, dtype=np.uint32)
    assert np.array_equal(run(keys2, gpu, "always"), np.sort(keys2))


@pytest.mark.parametrize("kb,pairs", [(32, False), (32, True), (64, False)])
def test_msd_exact_p2_hook(gpu, kb, pairs):
    """Option msd = exact_p2 (a test hook: P2's regions refused) runs the exact redo -- the gated
    exact histogram and the persistent exact pass in place -- at a sampled size, bit-exact."""
    n = (1 << 27) + 3
    rng = np.random.default_rng(kb * 7 + pairs)
    dt = np.uint32 if kb == 32 else np.uint64
    keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
    keys[::5] = keys[0]
    gk, gv = run_typed(keys, gpu, pairs, "exact_p2")
    perm = np.argsort(keys, kind="stable")
    assert np.array_equal(gk, keys[perm])
    if pairs:
        assert np.array_equal(gv, perm.astype(np.uint32))


def test_msd_pairs_sampled_p2(gpu):
    """u32 pairs at a sampled size (P2 into sampled regions): keys and the stable permutation
    bit-exact, also through a P2 region spill -- the case whose runs the region pass must hold
    inside the region buffer (the run clamp, grs_pass.hpp) before the exact redo."""
    import gpuradixsort_amd as grs

    n = (1 << 27) + 77
    for other in list(_S):
        _S.pop(other).close()
    s = grs.RadixSorter(n, key_bits=32, pairs=True, radix_bits=8)
    try:
        s.set_option("msd", "always")
        rng = np.random.default_rng(4242)
        piece = (np.arange(n, dtype=np.int64) // PIECE) % 2
        spill = (np.where(piece == 0, 0, 255).astype(np.uint32) << np.uint32(16)) | \
            rng.integers(0, 1 << 16, n, dtype=np.uint32)
        spill[-1] |= np.uint32(1 << 31)   # the top byte varies: P1 / P2 stay on bytes 3 / 2
        dup = rng.integers(0, 1 << 32, n, dtype=np.uint32)
        dup[::3] = dup[1]
        for name, keys in (("dup", dup), ("p2_spill", spill)):
            k = torch.from_numpy(keys).to(gpu)
            v = torch.arange(n, dtype=torch.int32, device=gpu).view(torch.uint32)
            s.sort(k, v)
            torch.cuda.synchronize()
            s.check_error()
            assert s.check_guards() == 0, name
            perm = np.argsort(keys, kind="stable")
            assert np.array_equal(k.cpu().numpy(), keys[perm]), name
            assert np.array_equal(v.cpu().numpy(), perm.astype(np.uint32)), name
            del k, v
    finally:
        s.close()
