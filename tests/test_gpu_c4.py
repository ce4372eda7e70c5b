"""GPU tests of BASELINE config C4 (2^30 uint32 keys, 8 shards) on one MI355X.

  * the whole 2^30-key input in ONE device call (the look-back words hold 32-bit prefixes, so
    one call takes up to GRS_MAX_N = 2^32 - 2^16 items), against the committed digest;
  * the 8-rank pipeline of grs_sort_sharded replayed on one GPU: eight 2^27-key shards, the
    same sampling and tie-breaking splitters (libgrs's host twin of the device step), one
    grs_partition_ranges per shard, buckets concatenated in source-rank order, eight local
    sorts -- the concatenation must match the same digest, and the destinations must be
    balanced.
Digest: tests/golden/digests.json c4_1b_u32 (SHA-256 of the sorted splitmix64 keys, computed
by the oracle in tests/golden/make_golden.py)."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _rec():
    return json.load(open(os.path.join(GOLDEN, "digests.json")))["c4_1b_u32"]


def _host_sha_update(h, t: torch.Tensor, chunk=1 << 27):
    for i in range(0, t.numel(), chunk):
        h.update(t[i:i + chunk].cpu().numpy().tobytes())


def test_c4_one_call_2pow30(gpu):
    import gpuradixsort_amd as grs

    rec = _rec()
    n = rec["n"]
    assert n == 1 << 30
    k = torch.empty(n, dtype=torch.uint32, device=gpu)
    grs.fill_splitmix(k, rec["seed"])
    s = grs.RadixSorter(n, key_bits=32)
    s.sort(k)
    s.check_error()
    assert grs.count_inversions(k) == 0
    h = hashlib.sha256()
    _host_sha_update(h, k)
    assert h.hexdigest() == rec["sha256_keys"]
    assert k[:4].cpu().tolist() == rec["head"] and k[-4:].cpu().tolist() == rec["tail"]
    s.close()
    del k
    torch.cuda.empty_cache()


def test_c4_eight_shard_pipeline_on_one_gpu(gpu):
    import gpuradixsort_amd as grs
    from gpuradixsort_amd._lib import check, lib

    L = lib()
    rec = _rec()
    G, n = 8, rec["n"] // 8
    S = L.grs_shard_samples_per_rank(G)
    part = grs.RadixSorter(n, key_bits=32)
    shard = torch.empty(n, dtype=torch.uint32, device=gpu)
    # 1. samples of every shard (grs_shard_samples: position floor(i * n / S)), rank-major
    pos = (torch.arange(S, dtype=torch.int64) * n) // S
    ak, ap = [], []
    for r in range(G):
        grs.fill_splitmix(shard, rec["seed"], first_index=r * n)
        ak.append(shard.index_select(0, pos.to(gpu)).cpu().numpy())
        ap.append(pos.numpy().astype(np.uint32))
    ak, ap = np.concatenate(ak), np.ascontiguousarray(np.concatenate(ap))
    order = np.lexsort((np.arange(G * S), ak))
    sk = np.ascontiguousarray(ak[order])
    sj = np.ascontiguousarray(order.astype(np.uint32))
    # 2. per shard: its splitters + thresholds (host twin of grs_shard_splitters), partition
    parts, counts = [], []
    for r in range(G):
        spl = np.zeros(G - 1, np.uint32)
        th = np.zeros(G - 1, np.uint32)
        check(L.grs_shard_splitters_host(sk.ctypes.data, sj.ctypes.data, ap.ctypes.data, 4, G, S, r,
                                         spl.ctypes.data, th.ctypes.data), "splitters")
        grs.fill_splitmix(shard, rec["seed"], first_index=r * n)
        out = torch.empty_like(shard)
        cnt = torch.zeros(G, dtype=torch.uint32, device=gpu)
        check(L.grs_partition_ranges(part._h, ctypes.c_void_p(shard.data_ptr()), None,
                                     ctypes.c_void_p(out.data_ptr()), None, n,
                                     spl.ctypes.data, th.ctypes.data, G - 1,
                                     ctypes.c_void_p(cnt.data_ptr()), None), "partition")
        part.check_error()
        parts.append(out)
        counts.append(cnt.cpu().numpy().astype(np.int64))
    mat = np.stack(counts)                      # mat[r][b]: shard r's bucket b
    assert mat.sum() == G * n
    dest = mat.sum(0)
    assert dest.max() / dest.mean() <= 1.1, dest
    # 3. per destination: buckets in source-rank order, local stable sort, digest in order
    local = grs.RadixSorter(int(dest.max()), key_bits=32)
    h = hashlib.sha256()
    off = np.concatenate([np.zeros((G, 1), np.int64), np.cumsum(mat, 1)], 1)
    for b in range(G):
        buf = torch.cat([parts[r][off[r, b]:off[r, b + 1]] for r in range(G)])
        local.sort(buf)
        local.check_error()
        assert grs.count_inversions(buf) == 0
        _host_sha_update(h, buf)
        del buf
    assert h.hexdigest() == rec["sha256_keys"]
    part.close()
    local.close()
    del parts, shard
    torch.cuda.empty_cache()


def _checksums(k: torch.Tensor):
    """Order-independent checksums of a uint32 tensor: the sum of its values and the sum of
    their images under a multiplicative hash, both as int32 reinterpretations summed in int64."""
    v = k.view(torch.int32)
    s1 = int(v.sum(dtype=torch.int64).item())
    h = v * -1640531535                         # 0x9E3779B1, wrapping in int32
    s2 = int(h.sum(dtype=torch.int64).item())
    del h
    return s1, s2


def test_max_n_one_call(gpu):
    """GRS_MAX_N = 2^32 - 2^16 keys in ONE call (the largest the +1-encoded 32-bit look-back
    prefixes and 32-bit tile positions allow): sorted, and the same multiset (checksums), at
    the size where any 32-bit index overflow in the kernels would show."""
    import gpuradixsort_amd as grs
    from gpuradixsort_amd._lib import GRS_MAX_N

    import time

    n = GRS_MAX_N
    t0 = time.time()

    def note(what):
        print(f"  max_n: {what} at {time.time() - t0:.2f} s", flush=True)

    k = torch.empty(n, dtype=torch.uint32, device=gpu)
    grs.fill_splitmix(k, 0x6A09E667F3BCC908 + 4, first_index=1 << 40)
    torch.cuda.synchronize()
    note("filled")
    before = _checksums(k)
    note("checksummed")
    s = grs.RadixSorter(n, key_bits=32)
    note("sorter created")
    s.sort(k)
    s.check_error()
    note("sorted")
    assert grs.count_inversions(k) == 0
    note("inversions counted")
    assert _checksums(k) == before
    s.close()
    del k
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n,dist", [(1_500_000_000, "perm"), ((1 << 31) + 12345, "uniform")])
def test_msd_past_c4(gpu, n, dist):
    """u32 keys past 1.13G (16-bit segments of 23K-33K keys: P3's 36K-key shape): still the MSD
    schedule (grs_debug_msd_flags answers, no redo, no exact P2), sorted and the same multiset;
    the reference's shuffled 0..n-1 (1.5G: 32768-key segments) sorts to exactly 0..n-1."""
    import gpuradixsort_amd as grs

    k = torch.empty(n, dtype=torch.uint32, device=gpu)
    if dist == "perm":
        grs.fill_permutation(k, 0x5EED)
    else:
        grs.fill_splitmix(k, 0x6A09E667F3BCC908 + 5)
    before = _checksums(k)
    s = grs.RadixSorter(n, key_bits=32)
    s.sort(k)
    s.check_error()
    f = s.msd_flags()
    assert not f["p1_redo"] and not f["p2_exact"], f
    assert s.check_guards() == 0
    s.close()
    assert grs.count_inversions(k) == 0
    assert _checksums(k) == before
    if dist == "perm":
        assert int(k[:1].view(torch.int32).item()) == 0 and int(k[-1:].view(torch.int32).item()) == n - 1
    del k
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kb", [32, 64])
def test_max_n_pairs_one_call(gpu, kb):
    """GRS_MAX_N (key, index) pairs in one call, u32 and u64 keys: keys sorted and
    keys_in[payload] == keys_out (the payload is the stable permutation)."""
    import gpuradixsort_amd as grs
    from gpuradixsort_amd._lib import GRS_MAX_N

    n = GRS_MAX_N
    kdt = torch.uint32 if kb == 32 else torch.uint64
    k = torch.empty(n, dtype=kdt, device=gpu)
    grs.fill_splitmix(k, 0x6A09E667F3BCC908 + 3, first_index=1 << 41)
    orig = k.clone()
    v = torch.empty(n, dtype=torch.uint32, device=gpu)
    grs.iota_u32(v)
    s = grs.RadixSorter(n, key_bits=kb, pairs=True)
    s.sort(k, v)
    s.check_error()
    s.close()                                   # frees the sorter's scratch before the check
    assert grs.count_inversions(k) == 0
    iv = torch.int32 if kb == 32 else torch.int64
    idx = v.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    del v
    gathered = orig.view(iv)[idx]
    del idx, orig
    assert torch.equal(gathered, k.view(iv))
    del k, gathered
    torch.cuda.empty_cache()


def test_c4_presorted_eight_ranks_on_one_gpu(gpu):
    """The presorted exchange of C4 at full size, eight ranks replayed on one GPU through the
    C-ABI steps: each 2^27-key shard sorted, sampled, split by the tie-breaking splitters and
    encoded; each receiver decodes and merges the eight encoded runs it gets.  The ranks'
    outputs concatenated must hash to the committed digest; the encoding must be about a byte
    per key; the receivers must be balanced.  Each receiver's runs are also merged by the
    one-pass k-way merge (option "merge"), which must give the same keys."""
    import gpuradixsort_amd as grs
    from gpuradixsort_amd import _lib
    from gpuradixsort_amd.sharded import shard_decode_merge, shard_encode, shard_sample

    rec = _rec()
    G, n = 8, rec["n"] // 8
    S = int(_lib.lib().grs_shard_samples_per_rank(G))
    s = grs.RadixSorter(n + n // 4, key_bits=32)
    shards, sks, sps = [], [], []
    for r in range(G):
        k = torch.empty(n, dtype=torch.uint32, device=gpu)
        grs.fill_splitmix(k, rec["seed"], first_index=r * n)
        s.sort(k)
        shards.append(k)
        sk, sp = shard_sample(k, n, S)
        sks.append(sk)
        sps.append(sp)
    gk, gp = torch.cat(sks), torch.cat(sps)
    sends, mat = [], []
    for r in range(G):
        send, sz = shard_encode(s, shards[r], n, gk, gp, G, r)
        sends.append(send)
        mat.append(sz.cpu().numpy().astype(np.int64))
    del shards
    mat = np.stack(mat)
    words = mat[:, 1::2]
    assert 4 * words.sum() / (G * n) < 1.1
    h = hashlib.sha256()
    sizes = []
    out = torch.empty(n + n // 4, dtype=torch.uint32, device=gpu)
    out_k = torch.empty_like(out)
    for r in range(G):
        parts, offs, lens, off = [], [], [], 0
        for p in range(G):
            start, w = int(words[p, :r].sum()), int(words[p, r])
            parts.append(sends[p][start:start + w])
            offs.append(off)
            lens.append(int(mat[p, 2 * r]))
            off += w
        recv = torch.cat(parts)
        m = shard_decode_merge(s, recv, offs, lens, out)
        s.set_option("merge", "kway")
        assert shard_decode_merge(s, recv, offs, lens, out_k) == m
        s.set_option("merge", "rounds")
        s.check_error()
        assert torch.equal(out[:m], out_k[:m]), f"k-way merge differs at receiver {r}"
        sizes.append(m)
        _host_sha_update(h, out[:m])
        del recv
    assert sum(sizes) == rec["n"]
    assert max(sizes) / (sum(sizes) / G) <= 1.02, sizes
    assert h.hexdigest() == rec["sha256_keys"]
    s.close()


@pytest.mark.parametrize("name", ["all_equal", "sorted", "reversed", "few_unique", "low_bits"])
def test_c4_size_distributions(gpu, name):
    """2^30 keys of structured distributions in one call: sorted, and the same multiset
    (sum and sum of squares of the keys)."""
    import gpuradixsort_amd as grs

    n = 1 << 30
    k = torch.empty(n, dtype=torch.uint32, device=gpu)
    if name == "all_equal":
        k.fill_(7)
    else:
        grs.fill_splitmix(k, 0xC4C4C4C4 + len(name))
        if name == "sorted":
            s0 = grs.RadixSorter(n, key_bits=32)
            s0.sort(k)
            s0.close()
        elif name == "reversed":
            s0 = grs.RadixSorter(n, key_bits=32)
            s0.sort(k)
            s0.close()
            k = torch.flip(k.view(torch.int32), [0]).view(torch.uint32).contiguous()
        elif name == "few_unique":
            k = ((k.view(torch.int32) & 3) * 0x40000001).view(torch.uint32)   # 4 keys, top and low bits
        elif name == "low_bits":   # every key below 2^12: the top passes see one digit
            k = (k.view(torch.int32) & 0xFFF).view(torch.uint32).contiguous()

    def checks(t):
        s1 = s2 = 0
        for i in range(0, n, 1 << 27):
            c = t[i:i + (1 << 27)].view(torch.int32).to(torch.int64) & 0xFFFFFFFF
            s1 += int(c.sum().item())
            s2 += int((c * c).remainder_(1 << 61).sum().item())   # int64 sums wrap: compare mod 2^64
        return s1, s2 % (1 << 64)
    before = checks(k)
    s = grs.RadixSorter(n, key_bits=32)
    s.sort(k)
    s.check_error()
    assert grs.count_inversions(k) == 0
    assert checks(k) == before
    s.close()


@pytest.mark.parametrize("dist", ["lists", "narrow28", "perm"])
def test_p3_low_halves_lists(gpu, dist):
    """P3 on the low 16 bits in LDS (grs_msd_local16, the u32 P3 from ~0.6G keys, 512 x 34 slots)
    against the whole-key kernel (option p3 = whole_keys) on the same 700M keys: identical
    output, sorted, the same multiset, no guard word touched.  lists: uniform keys with one
    16-bit segment pushed past 17408 keys into the mid list (~18K keys) and one into the fallback
    (~41K); narrow28: keys below 2^28 (the top digit at bit 20, P3's bits 12..15 constant in a
    segment); perm: the reference's 0..n-1 shuffled (top digit at bit 22)."""
    import gpuradixsort_amd as grs

    n = 700_000_000
    src = torch.empty(n, dtype=torch.uint32, device=gpu)
    if dist == "perm":
        grs.fill_permutation(src, 0x5EED7)
    else:
        grs.fill_splitmix(src, 0x3C6EF372FE94F82B)
    v = src.view(torch.int32)
    if dist == "lists":
        v[:7300] = (v[:7300] & 0xFFFF) | (0x1234 << 16)
        v[7300:37300] = (v[7300:37300] & 0xFFFF) | (0x4321 << 16)
    elif dist == "narrow28":
        v &= (1 << 28) - 1
    before = _checksums(src)
    outs = []
    for mode in ("per_segment", "whole_keys"):
        k = src.clone()
        s = grs.RadixSorter(n, key_bits=32)
        s.set_option("p3", mode)
        s.sort(k)
        s.check_error()
        assert s.check_guards() == 0, mode
        f = s.msd_flags()
        s.close()
        outs.append(k)
    del src
    assert torch.equal(outs[0], outs[1])
    assert grs.count_inversions(outs[0]) == 0
    assert _checksums(outs[0]) == before
    if dist == "lists":
        hi = (outs[0].view(torch.int32) >> 16) & 0xFFFF
        assert int((hi == 0x1234).sum().item()) > 17408 and int((hi == 0x4321).sum().item()) > 36864
        del hi
    else:
        assert f["top_shift"] == (20 if dist == "narrow28" else 22), f
    if dist == "perm":
        assert int(outs[0][:1].view(torch.int32).item()) == 0 and int(outs[0][-1:].view(torch.int32).item()) == n - 1
    del outs
    torch.cuda.empty_cache()
