"""GPU tests of the presorted exchange of grs_sort_sharded (gpuradixsort_amd/csrc/grs_codec.hpp)
through its transport-independent C-ABI steps (include/grs.h): G ranks are simulated on ONE
device -- every rank's shard is sorted, sampled, split and encoded by libgrs, the "exchange" is a
device copy of each bucket's encoded words into the receiver's buffer (the same words RCCL would
carry), and every receiver decodes and merges them.  The ranks' outputs concatenated must be the
sorted input, and the splitters (ties broken by global index) must balance duplicate-heavy
inputs.  The RCCL transport itself runs at world size 1 in tests/test_gpu_sharded.py."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dist(name, n, rng):
    if name == "uniform":
        return rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    if name == "all_equal":
        return np.full(n, 7, np.uint32)
    if name == "few_unique":
        return rng.choice(np.array([3, 0xFFFFFFFF, 1 << 20, 0], np.uint32), n)
    if name == "skewed":       # most keys in a narrow band, some far away
        k = rng.integers(1000, 3000, n, dtype=np.uint64).astype(np.uint32)
        k[::97] = rng.integers(0, 2**32, k[::97].size, dtype=np.uint64).astype(np.uint32)
        return k
    if name == "max_gaps":     # deltas of 2^31 and more: 32-bit widths
        k = rng.integers(0, 2, n, dtype=np.uint64).astype(np.uint32) * np.uint32(0xFFFFFFFF)
        return k
    if name == "sorted_desc":
        return np.sort(rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32))[::-1].copy()
    raise ValueError(name)


def sim_presorted(shards, gpu, cap=None, merge="rounds"):
    """Simulate grs_sort_sharded's presorted exchange over len(shards) ranks on one device.
    Returns the ranks' outputs (numpy) and the G x 2G size matrix.  merge: the receive side's
    2-way rounds ("rounds", the default) or its one k-way pass ("kway")."""
    import gpuradixsort_amd as grs
    from gpuradixsort_amd import _lib
    from gpuradixsort_amd.sharded import shard_decode_merge, shard_encode, shard_sample

    G = len(shards)
    S = int(_lib.lib().grs_shard_samples_per_rank(G))
    total = sum(len(s) for s in shards)
    cap = cap or max(total, 1)
    sorter = grs.RadixSorter(cap, key_bits=32, device=gpu.index, options={"merge": merge})
    sorted_, sks, sps = [], [], []
    for sh in shards:
        k = torch.from_numpy(sh).to(gpu)
        sorter.sort(k)
        sorted_.append(k)
        sk, sp = shard_sample(k, k.numel(), S)
        sks.append(sk)
        sps.append(sp)
    gk, gp = torch.cat(sks), torch.cat(sps)
    sends, sizes = [], []
    for r, k in enumerate(sorted_):
        send, sz = shard_encode(sorter, k, k.numel(), gk, gp, G, r)
        sends.append(send)
        sizes.append(sz.cpu().numpy().astype(np.int64))
    mat = np.stack(sizes)                     # row p: (keys, words) of each bucket of rank p
    outs = []
    for r in range(G):
        parts, offs, lens, off = [], [], [], 0
        for p in range(G):
            words = mat[p, 1::2]
            start = int(words[:r].sum())
            w = int(words[r])
            parts.append(sends[p][start:start + w])
            offs.append(off)
            lens.append(int(mat[p, 2 * r]))
            off += w
        recv = torch.cat(parts) if off else torch.zeros(1, dtype=torch.uint32, device=gpu)
        out = torch.empty(max(sum(lens), 1), dtype=torch.uint32, device=gpu)
        m = shard_decode_merge(sorter, recv, offs, lens, out)
        sorter.check_error()
        outs.append(out[:m].cpu().numpy())
    sorter.close()
    return outs, mat


@pytest.mark.parametrize("merge", ["kway", "rounds"])
@pytest.mark.parametrize("G", [1, 2, 3, 4, 5, 8, 16])
@pytest.mark.parametrize("name", ["uniform", "all_equal", "few_unique", "skewed"])
def test_presorted_sim_matches_sort(gpu, G, name, merge):
    rng = np.random.default_rng(G * 31 + len(name))
    n_local = 200_003
    shards = [_dist(name, n_local + 1000 * r, rng) for r in range(G)]
    outs, mat = sim_presorted(shards, gpu, merge=merge)
    allk = np.concatenate(shards)
    got = np.concatenate(outs)
    assert np.array_equal(got, np.sort(allk))
    # every rank's bucket keys sum to its shard; ties split by global index keep the ranks even
    assert [int(mat[p, 0::2].sum()) for p in range(G)] == [len(s) for s in shards]
    sizes = np.array([len(o) for o in outs])
    if G > 1:
        assert sizes.max() / sizes.mean() <= 1.1, sizes


@pytest.mark.parametrize("merge", ["kway", "rounds"])
@pytest.mark.parametrize("name", ["max_gaps", "sorted_desc", "uniform"])
def test_presorted_sim_edges(gpu, name, merge):
    """32-bit delta widths, ragged last blocks, empty shards, tiny shards, one-key shards."""
    rng = np.random.default_rng(5)
    for lens in ([0, 0, 0], [1, 0, 5, 255], [256, 257, 1, 4095, 4097], [0, 100_000], [70_001] * 5):
        shards = [_dist(name, n, rng) for n in lens]
        outs, _ = sim_presorted(shards, gpu, merge=merge)
        assert np.array_equal(np.concatenate(outs), np.sort(np.concatenate(shards))), lens


def test_presorted_encoding_size(gpu):
    """Uniform keys at 8 ranks: a run of n_local / 8 keys from one source spans 2^32 / 8 values,
    so its deltas average 2^32 / n_local and a 256-key block's widest delta is about ln(256)
    times that: 16 bits at n_local = 2^20 (2 bytes a key); at C4's 2^27 per rank, 8 bits."""
    rng = np.random.default_rng(11)
    G, n_local = 8, 1 << 20
    shards = [rng.integers(0, 2**32, n_local, dtype=np.uint64).astype(np.uint32) for _ in range(G)]
    outs, mat = sim_presorted(shards, gpu)
    words = int(mat[:, 1::2].sum())
    assert np.array_equal(np.concatenate(outs), np.sort(np.concatenate(shards)))
    bytes_per_key = 4 * words / (G * n_local)
    assert 1.8 < bytes_per_key < 2.1, bytes_per_key


def test_presorted_steps_reject_short_buffers(gpu):
    import ctypes

    import gpuradixsort_amd as grs
    from gpuradixsort_amd import _lib

    L = _lib.lib()
    s = grs.RadixSorter(1000, key_bits=32, device=gpu.index)
    k = torch.zeros(1000, dtype=torch.uint32, device=gpu)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    # send buffer below grs_shard_encode_words_max
    rc = L.grs_shard_encode(s._h, P(k), 1000, P(k), P(k), 2, 0, P(k), 100, P(k), None)
    assert rc == _lib.GRS_ECAPACITY
    # received keys above the sorter's capacity
    wo = (ctypes.c_uint64 * 2)(0, 0)
    ln = (ctypes.c_uint32 * 2)(800, 800)
    assert L.grs_shard_decode_merge(s._h, P(k), 2, wo, ln, P(k), 1000, None) == _lib.GRS_ECAPACITY
    s.close()


def test_presorted_world1_empty_and_tiny(gpu, monkeypatch):
    """grs_sort_sharded's presorted path on a one-rank RCCL communicator: empty, one-key and
    one-block shards (the RCCL transport at G > 1 needs more GPUs than a box has)."""
    import os
    import socket

    import torch.distributed as dist

    from gpuradixsort_amd.sharded import RcclComm, ShardedSorter

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        comm = RcclComm(device=gpu.index)
        s = ShardedSorter(5000, key_bits=32, device=gpu, comm=comm,
                          options={"sharded_path": "general"})
        rng = np.random.default_rng(2)
        for n in (0, 1, 255, 256, 257, 4999):
            keys = rng.integers(0, 2**32, 5000, dtype=np.uint64).astype(np.uint32)
            ko, _ = s.sort(torch.from_numpy(keys).to(gpu), n=n)
            assert s.last_n_out == n
            assert np.array_equal(ko.cpu().numpy(), np.sort(keys[:n]))
        s.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("merge", ["kway", "rounds"])
@pytest.mark.parametrize("k", [2, 3, 7, 8, 13, 16])
def test_merge_at_run_and_tie_boundaries(gpu, k, merge):
    """The k-way merge on its own (grs_shard_decode_merge of encoded sorted runs): runs of very
    different lengths, long runs of one key crossing the sample spacing and the tile boundaries
    in several runs at once, and keys whose only difference is the run they come from."""
    import gpuradixsort_amd as grs
    from gpuradixsort_amd import _lib
    from gpuradixsort_amd.sharded import shard_decode_merge, shard_encode, shard_sample

    S = int(_lib.lib().grs_shard_samples_per_rank(1))
    rng = np.random.default_rng(100 + k)
    runs = []
    for q in range(k):
        n = int(rng.choice([0, 1, 255, 256, 257, 4096 * 3 + 17, 60_000 + 1000 * q]))
        base = rng.integers(0, 50, n, dtype=np.uint64).astype(np.uint32) * np.uint32(1 << 26)
        noise = rng.integers(0, 3, n, dtype=np.uint64).astype(np.uint32)
        runs.append(np.sort(base + noise))
    total = sum(len(r) for r in runs)
    sorter = grs.RadixSorter(max(total, 1), key_bits=32, device=gpu.index, options={"merge": merge})
    # each run becomes the single bucket of a one-rank encode (G = 1: the whole shard)
    parts, offs, lens, off = [], [], [], 0
    for r in runs:
        t = torch.from_numpy(r).to(gpu) if len(r) else torch.zeros(1, dtype=torch.uint32, device=gpu)
        sk, sp = shard_sample(t, len(r), S)
        send, sz = shard_encode(sorter, t, len(r), sk, sp, 1, 0)
        w = int(sz.cpu().numpy()[1])
        parts.append(send[:w])
        offs.append(off)
        lens.append(len(r))
        off += w
    recv = torch.cat(parts) if off else torch.zeros(1, dtype=torch.uint32, device=gpu)
    out = torch.empty(max(total, 1), dtype=torch.uint32, device=gpu)
    m = shard_decode_merge(sorter, recv, offs, lens, out)
    sorter.check_error()
    assert m == total
    assert np.array_equal(out[:m].cpu().numpy(), np.sort(np.concatenate(runs)))
    sorter.close()
