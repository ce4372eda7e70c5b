"""GPU tests of the MSD sort's span-adaptive top digit (grs_msd.hpp msd_top_shift) on the
reference's own input distribution.

The reference sorts 0..N-1 shuffled (main.cpp:119-125).  Such keys vary in their low log2(N)
bits only, so a top-byte MSD scatter would leave 16 buckets at N = 2^28 and 16-bit segments of
65536 keys, past every LDS shape.  The MSD schedule therefore takes its two scatter digits from
the keys' highest VARYING bits (OR(keys) & OR(~keys)): a guess from 4096 sampled keys, checked
exactly by the first scatter's tiles, with a redo at the exact digit when the guess missed a
varying bit.  Every case must equal the stable sort (and the reference's path where the oracle
runs in seconds).
"""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

GUESS_CHUNKS = 64   # GRS_MSD_GUESS_CHUNKS: 64-key chunks every sample block reads for the guess


def _sorter(n, key_bits=32, pairs=False, mode="always"):
    import gpuradixsort_amd as grs

    s = grs.RadixSorter(max(n, 1 << 20), key_bits=key_bits, pairs=pairs, radix_bits=8)
    s.set_option("msd", mode)
    return s


def _sort_np(keys, dev, pairs=False, mode="always"):
    kb = keys.dtype.itemsize * 8
    s = _sorter(keys.size, kb, pairs, mode)
    k = torch.from_numpy(np.ascontiguousarray(keys)).to(dev)
    v = torch.arange(keys.size, dtype=torch.int32, device=dev).view(torch.uint32) if pairs else None
    s.sort(k, v)
    torch.cuda.synchronize()
    s.check_error()
    assert s.check_guards() == 0, "a kernel wrote past a scratch array (guard band)"
    s.close()
    return k.cpu().numpy(), (v.cpu().numpy() if pairs else None)


def _guess_positions(n):
    """Indices the span guess reads (grs_msd_sample): 64 chunks of 64 keys, evenly spaced."""
    if n <= GUESS_CHUNKS * 64:
        return np.arange(n)
    c = np.arange(GUESS_CHUNKS, dtype=np.uint64)
    starts = (c * np.uint64(n - 64) // np.uint64(GUESS_CHUNKS - 1)).astype(np.int64)
    return (starts[:, None] + np.arange(64)[None, :]).ravel()


@pytest.mark.parametrize("n", [4096, 65537, 300007, 1 << 20])
@pytest.mark.parametrize("pairs", [False, True])
def test_permutation_matches_reference_path(gpu, n, pairs):
    """The reference's own input, forced MSD schedule: keys and the stable permutation ==
    the restated reference path (ParallelSort.cpp:236-298)."""
    rng = np.random.default_rng(n + pairs)
    keys = rng.permutation(n).astype(np.uint32)
    rk, rp = oracle.ref_parallel_sort(keys)
    gk, gv = _sort_np(keys, gpu, pairs)
    assert np.array_equal(gk, rk)
    if pairs:
        assert np.array_equal(gv, rp)


@pytest.mark.parametrize("kb,pairs", [(32, False), (32, True), (64, False)])
def test_guess_misses_a_varying_bit(gpu, kb, pairs):
    """Keys below 2^20 except a few with the top bit set, placed where the 4096-key guess does
    not look: the guess picks the digit at bits 12..19, P1's exact span finds bit kb-1, and the
    redo scatters again at the top digit -- bit-exact, and the sorter's next sort too."""
    n = 1 << 22
    dt = np.uint32 if kb == 32 else np.uint64
    rng = np.random.default_rng(kb * 3 + pairs)
    keys = rng.integers(0, 1 << 20, n).astype(dt)
    seen = np.zeros(n, bool)
    seen[_guess_positions(n)] = True
    free = np.flatnonzero(~seen)
    hot = rng.choice(free, 7, replace=False)
    keys[hot] |= dt(1) << dt(kb - 1)
    gk, gv = _sort_np(keys, gpu, pairs)
    perm = np.argsort(keys, kind="stable")
    assert np.array_equal(gk, keys[perm])
    if pairs:
        assert np.array_equal(gv, perm.astype(np.uint32))
    keys2 = rng.integers(0, 1 << 20, n).astype(dt)
    assert np.array_equal(_sort_np(keys2, gpu, pairs)[0], np.sort(keys2))


@pytest.mark.parametrize("name", ["offset_range", "low_16", "low_12", "mid_bits", "two_values",
                                  "top_only", "sparse_high"])
def test_narrow_spans(gpu, name):
    """Spans the top digit adapts to: an offset range (constant high bits that are not zero),
    keys below 2^16 / 2^12 (the lowest digit, one or no LDS round), a band of middle bits, two
    values, keys differing in the top byte only, and sparse high bits."""
    n = (1 << 22) + 13
    rng = np.random.default_rng(len(name))
    if name == "offset_range":
        keys = np.uint32(0xA5000000) + rng.integers(0, 1 << 24, n, dtype=np.uint32)
    elif name == "low_16":
        keys = rng.integers(0, 1 << 16, n, dtype=np.uint32)
    elif name == "low_12":
        keys = rng.integers(0, 1 << 12, n, dtype=np.uint32)
    elif name == "mid_bits":
        keys = (rng.integers(0, 1 << 14, n, dtype=np.uint32) << np.uint32(9)) | np.uint32(0x80000001)
    elif name == "two_values":
        keys = np.where(rng.random(n) < 0.5, 0x12345678, 0x12345679).astype(np.uint32)
    elif name == "top_only":
        keys = rng.integers(0, 256, n, dtype=np.uint32) << np.uint32(24)
    else:
        keys = rng.integers(0, 1 << 18, n, dtype=np.uint32)
        keys[rng.integers(0, n, 1000)] |= np.uint32(1 << 30)
    for pairs in (False, True):
        gk, gv = _sort_np(keys, gpu, pairs)
        perm = np.argsort(keys, kind="stable")
        assert np.array_equal(gk, keys[perm]), (name, pairs)
        if pairs:
            assert np.array_equal(gv, perm.astype(np.uint32)), name


@pytest.mark.parametrize("bits", [40, 33, 20])
def test_u64_narrow_spans(gpu, bits):
    """u64 keys of a narrow span: fewer LDS rounds in P3 (ceil((top - 8) / 8))."""
    n = (1 << 21) + 5
    rng = np.random.default_rng(bits)
    keys = rng.integers(0, 1 << bits, n, dtype=np.uint64) + np.uint64(0x0123000000000000)
    gk, _ = _sort_np(keys, gpu)
    assert np.array_equal(gk, np.sort(keys))


@pytest.mark.parametrize("n,pairs", [(1 << 28, False), (1 << 28, True), ((1 << 27) + 77, False),
                                     (1 << 30, False)])
def test_reference_distribution_full_size(gpu, n, pairs):
    """The reference's input at BASELINE sizes (ns / C3 / C4) through the DEFAULT schedule: the
    sorted keys are exactly 0..n-1, and the payload is the inverse permutation
    (keys_in[payload] == 0..n-1)."""
    import gpuradixsort_amd as grs

    k = torch.empty(n, dtype=torch.uint32, device=gpu)
    grs.fill_permutation(k, 0x5EED + n)
    orig = k.clone() if pairs else None
    v = None
    if pairs:
        v = torch.empty(n, dtype=torch.uint32, device=gpu)
        grs.iota_u32(v)
    s = grs.RadixSorter(n, key_bits=32, pairs=pairs)
    s.sort(k, v)
    s.check_error()
    # no sampled region overflowed, and the guess found the span -- except when n is just above a
    # power of two: the 77 keys with the top bit are not among the guess's 4096, so P1 runs twice
    rare_top = n & (n - 1) != 0 and (n - (1 << (n.bit_length() - 1))) < n // 1000
    assert s.msd_flags() == {"p1_redo": rare_top, "p2_exact": False, "top_shift": (n - 1).bit_length() - 8}
    assert s.check_guards() == 0
    s.close()
    ar = torch.arange(n, dtype=torch.int64, device=gpu)
    assert torch.equal(k.view(torch.int32).to(torch.int64) & 0xFFFFFFFF, ar)
    if pairs:
        idx = v.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        assert torch.equal(orig.view(torch.int32).to(torch.int64)[idx] & 0xFFFFFFFF, ar)
    del k, v, orig, ar
    torch.cuda.empty_cache()


@pytest.mark.parametrize("total", [1 << 20, 1000003, 4096])
def test_fill_permutation_is_a_permutation(gpu, total):
    """grs_fill_permutation: every value of [0, total) once, in a scrambled order, and slices
    (first_index) agree with the whole."""
    import gpuradixsort_amd as grs

    k = torch.empty(total, dtype=torch.uint32, device=gpu)
    grs.fill_permutation(k, 99)
    h = k.cpu().numpy()
    assert np.array_equal(np.sort(h), np.arange(total, dtype=np.uint32))
    assert (np.diff(h.astype(np.int64)) == 1).mean() < 0.01
    part = torch.empty(total // 3, dtype=torch.uint32, device=gpu)
    grs.fill_permutation(part, 99, total=total, first_index=total // 3)
    assert np.array_equal(part.cpu().numpy(), h[total // 3: total // 3 + total // 3])


def _lsd_cases(n, kb, rng):
    """Inputs whose LSD digits are partly constant: the passes grs_pass_plan elides."""
    dt = np.uint32 if kb == 32 else np.uint64
    top = np.iinfo(dt).max
    yield "perm", rng.permutation(n).astype(dt)                       # main.cpp:119-125
    yield "all_equal", np.full(n, 0x5A, dt)                          # every pass constant
    yield "low_byte", rng.integers(0, 256, n).astype(dt)             # 3 (7) trivial top passes
    yield "hole", ((rng.integers(0, top, n, dtype=dt, endpoint=True) & dt(~(0xFF << 16) & top))
                   | dt(0xAB << 16))                                 # a constant middle byte
    yield "top_only", rng.integers(0, 256, n).astype(dt) << dt(kb - 8)   # low passes constant


@pytest.mark.parametrize("radix_bits", [4, 8])
@pytest.mark.parametrize("kb,pairs", [(32, False), (32, True), (64, False), (64, True)])
def test_lsd_elides_constant_digits(gpu, radix_bits, kb, pairs):
    """The LSD schedule (below 48M keys, and every 4-bit sort) skips the passes whose digit is
    the same for every key, or turns an odd run of them into one copy (grs_pass_plan): keys and
    the stable permutation must come out as the stable sort, at a small-tile and a big-tile size,
    with the sorter's guard bands intact."""
    import gpuradixsort_amd as grs

    for n in (300_007, (1 << 22) + 1):
        rng = np.random.default_rng(n + kb + radix_bits + pairs)
        s = grs.RadixSorter(n, key_bits=kb, pairs=pairs, radix_bits=radix_bits)
        for name, keys in _lsd_cases(n, kb, rng):
            k = torch.from_numpy(keys).to(gpu)
            v = torch.arange(n, dtype=torch.int32, device=gpu).view(torch.uint32) if pairs else None
            s.sort(k, v)
            s.check_error()
            perm = np.argsort(keys, kind="stable")
            assert np.array_equal(k.cpu().numpy(), keys[perm]), (name, n)
            if pairs:
                assert np.array_equal(v.cpu().numpy(), perm.astype(np.uint32)), (name, n)
        assert s.check_guards() == 0
        s.close()


def test_lsd_plan_c2_reference_input(gpu):
    """BASELINE C2's size and digit width (2^24 u32 keys, 4-bit LSD) on the reference's input:
    sorted to 0..n-1 exactly, and faster than the same sort of uniform keys (passes 6 and 7 see
    one digit and are skipped)."""
    import gpuradixsort_amd as grs

    n = 1 << 24
    s = grs.RadixSorter(n, key_bits=32, radix_bits=4)
    k = torch.empty(n, dtype=torch.uint32, device=gpu)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = {}
    for dist in ("uniform", "perm"):
        ts = []
        for i in range(6):
            if dist == "perm":
                grs.fill_permutation(k, 7 + i)
            else:
                grs.fill_splitmix(k, 7 + i)
            e0.record()
            s.sort(k)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms[dist] = sorted(ts[1:])[2]
    s.check_error()
    assert torch.equal(k.view(torch.int32).to(torch.int64), torch.arange(n, device=gpu))
    assert ms["perm"] < ms["uniform"], ms
    s.close()


@pytest.mark.parametrize("case", ["uniform", "span_redo", "spill_redo"])
@pytest.mark.parametrize("pairs", [False, True])
def test_h2_sample_paths(gpu, case, pairs):
    """Sorts large enough to sample H2 (2^27 + 3 keys): uniform keys (no redo, no exact P2), and
    H2's piece sample over a redone P1's exact layout -- a varying top bit the span guess
    misses, or a run past its sampled region (every key of one top digit sits where the sample
    does not look).  Keys and the stable permutation == torch's stable sort."""
    import gpuradixsort_amd as grs

    n = (1 << 27) + 3
    g = torch.Generator(device=gpu).manual_seed(27 + pairs)
    if case == "uniform":
        k64 = torch.randint(0, 1 << 32, (n,), generator=g, device=gpu, dtype=torch.int64)
    elif case == "span_redo":
        k64 = torch.randint(0, 1 << 20, (n,), generator=g, device=gpu, dtype=torch.int64)
        seen = np.zeros(n, bool)
        seen[_guess_positions(n)] = True
        hot = np.random.default_rng(5).choice(np.flatnonzero(~seen), 9, replace=False)
        k64[torch.from_numpy(hot).to(gpu)] |= 1 << 31
    else:
        # top byte 0x00 everywhere except one contiguous block of top byte 0xFF between the
        # sample's evenly spaced chunks (sampled share ~0, so its region is the pad alone)
        k64 = torch.randint(0, 1 << 24, (n,), generator=g, device=gpu, dtype=torch.int64)
        k64[100:100 + 8000] |= 0xFF << 24   # (between the sample's chunks at 0 and 8192)
        k64[n - 1] |= 1 << 31
    k = k64.to(torch.int32).view(torch.uint32)
    v = None
    if pairs:
        v = torch.empty(n, dtype=torch.uint32, device=gpu)
        grs.iota_u32(v)
    s = grs.RadixSorter(n, key_bits=32, pairs=pairs)
    s.sort(k, v)
    s.check_error()
    f = s.msd_flags()
    assert f["p1_redo"] == (case != "uniform"), f
    assert not f["p2_exact"], f
    assert s.check_guards() == 0
    s.close()
    want, perm = torch.sort(k64, stable=True)
    assert torch.equal(k.view(torch.int32).to(torch.int64) & 0xFFFFFFFF, want)
    if pairs:
        assert torch.equal(v.view(torch.int32).to(torch.int64) & 0xFFFFFFFF, perm)
    del k, v, k64, want, perm
    torch.cuda.empty_cache()
