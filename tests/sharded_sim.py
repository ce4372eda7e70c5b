"""Host simulation of grs_sort_sharded for the CPU (gloo) tests — TEST INFRASTRUCTURE.

It follows the device steps of gpuradixsort_amd/csrc/grs_capi.hip (run_sharded_n) one by one,
with gloo collectives in place of RCCL and numpy restatements of the three device kernels:

  grs_shard_samples      (grs_shard.hpp)   -> _samples
  grs_shard_splitters    (grs_shard.hpp)   -> np.lexsort by (key, gathered index), then
                                              libgrs's host twin grs_shard_splitters_host
  partition pass         (grs_pass.hpp with grs::SplitterIdxDigit) -> _buckets + stable argsort
  count exchange + plan  -> gloo all_gather + libgrs's host twin grs_shard_plan_host
  exchange               -> gloo all_to_all_single, source-rank order
  local sort             -> stable argsort

The splitter and plan arithmetic are the product's own (libgrs host twins, the same inline
functions the device code uses); nothing here is imported by gpuradixsort_amd.

sim_presorted_sort follows the presorted exchange (run_sharded_presorted, grs_codec.hpp) for
u32 keys without payload: local sort, samples of the SORTED shard, the same splitters, bucket
bounds = clamp(threshold, lower_bound, upper_bound) of each splitter key (libgrs's host twin
grs_shard_bounds_host of the device step grs_shard_bounds, checked against numpy),
exchange of the bucket runs in source-rank order, merge.  The encoding of the runs is exercised
on the GPU (tests/test_gpu_presorted.py); here the runs travel as plain keys.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist


def _lib():
    from gpuradixsort_amd._lib import check, lib

    return lib(), check


def _samples(keys: np.ndarray, s: int):
    n = keys.size
    if n == 0:
        return np.full(s, np.iinfo(keys.dtype).max, keys.dtype), np.full(s, 0xFFFFFFFF, np.uint32)
    pos = (np.arange(s, dtype=np.uint64) * np.uint64(n)) // np.uint64(s)
    return keys[pos.astype(np.int64)], pos.astype(np.uint32)


def _buckets(keys: np.ndarray, sk: np.ndarray, th: np.ndarray) -> np.ndarray:
    """grs::SplitterIdxDigit: #{b : sk[b] < k || (sk[b] == k && th[b] <= i)}."""
    i = np.arange(keys.size, dtype=np.uint64)
    b = np.zeros(keys.size, np.int64)
    for kb, tb in zip(sk, th):
        b += (kb < keys) | ((kb == keys) & (np.uint64(tb) <= i))
    return b


def _all_gather_np(a: np.ndarray, world: int, group=None) -> np.ndarray:
    t = torch.from_numpy(np.ascontiguousarray(a).view(np.int64 if a.itemsize == 8 else np.int32))
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    return np.concatenate([o.numpy() for o in out]).view(a.dtype)


def sim_sharded_sort(keys: np.ndarray, vals, group=None):
    """Returns (keys_out, vals_out, count_matrix) of this rank."""
    L, check = _lib()
    G, me = dist.get_world_size(group), dist.get_rank(group)
    S = int(L.grs_shard_samples_per_rank(G))
    kb = keys.dtype.itemsize
    sk, sp = _samples(keys, S)
    ak = _all_gather_np(sk, G, group)                 # rank-major: j = rank * S + i
    ap = _all_gather_np(sp, G, group)
    order = np.lexsort((np.arange(G * S), ak))        # by (key, j)
    sorted_k = np.ascontiguousarray(ak[order])
    sorted_j = np.ascontiguousarray(order.astype(np.uint32))
    spl = np.zeros(max(G - 1, 1), keys.dtype)
    th = np.zeros(max(G - 1, 1), np.uint32)
    check(L.grs_shard_splitters_host(sorted_k.ctypes.data, sorted_j.ctypes.data, ap.ctypes.data,
                                     kb, G, S, me, spl.ctypes.data, th.ctypes.data),
          "grs_shard_splitters_host")
    spl, th = spl[:G - 1], th[:G - 1]
    b = _buckets(keys, spl, th)
    perm = np.argsort(b, kind="stable")
    send_k = keys[perm]
    send_v = vals[perm] if vals is not None else None
    cnt = np.bincount(b, minlength=G).astype(np.uint32)
    mat = np.ascontiguousarray(_all_gather_np(cnt, G, group))
    soff = (ctypes.c_uint64 * G)()
    roff = (ctypes.c_uint64 * G)()
    n_out = ctypes.c_uint64()
    check(L.grs_shard_plan_host(mat.ctypes.data, G, me, soff, roff, ctypes.byref(n_out)),
          "grs_shard_plan_host")
    sc = [int(x) for x in mat.reshape(G, G)[me]]
    rc = [int(x) for x in mat.reshape(G, G)[:, me]]
    assert [int(roff[p]) for p in range(G)] == list(np.concatenate([[0], np.cumsum(rc)[:-1]]))
    assert [int(soff[p]) for p in range(G)] == list(np.concatenate([[0], np.cumsum(sc)[:-1]]))
    wide = np.int64 if kb == 8 else np.int32
    rk = torch.empty(int(n_out.value), dtype=torch.int64 if kb == 8 else torch.int32)
    dist.all_to_all_single(rk, torch.from_numpy(send_k.view(wide).copy()), output_split_sizes=rc,
                           input_split_sizes=sc, group=group)
    out_k = rk.numpy().view(keys.dtype)
    out_v = None
    if vals is not None:
        rv = torch.empty(int(n_out.value), dtype=torch.int32)
        dist.all_to_all_single(rv, torch.from_numpy(send_v.view(np.int32).copy()),
                               output_split_sizes=rc, input_split_sizes=sc, group=group)
        out_v = rv.numpy().view(np.uint32)
    p2 = np.argsort(out_k, kind="stable")
    return out_k[p2], (out_v[p2] if out_v is not None else None), mat.reshape(G, G)


def _splitters(sk, sp, G, me, S, kb, dtype, group=None):
    L, check = _lib()
    ak = _all_gather_np(sk, G, group)
    ap = _all_gather_np(sp, G, group)
    order = np.lexsort((np.arange(G * S), ak))
    sorted_k = np.ascontiguousarray(ak[order])
    sorted_j = np.ascontiguousarray(order.astype(np.uint32))
    spl = np.zeros(max(G - 1, 1), dtype)
    th = np.zeros(max(G - 1, 1), np.uint32)
    check(L.grs_shard_splitters_host(sorted_k.ctypes.data, sorted_j.ctypes.data, ap.ctypes.data,
                                     kb, G, S, me, spl.ctypes.data, th.ctypes.data),
          "grs_shard_splitters_host")
    return spl[:G - 1], th[:G - 1]


def sim_presorted_sort(keys: np.ndarray, group=None):
    """Returns (keys_out, bucket-size matrix) of this rank (u32 keys, presorted exchange)."""
    L, _ = _lib()
    G, me = dist.get_world_size(group), dist.get_rank(group)
    S = int(L.grs_shard_samples_per_rank(G))
    srt = np.sort(keys, kind="stable")
    sk, sp = _samples(srt, S)
    spl, th = _splitters(sk, sp, G, me, S, 4, keys.dtype, group)
    L, check = _lib()
    b = (ctypes.c_uint64 * (G + 1))()
    spl = np.ascontiguousarray(spl)
    th = np.ascontiguousarray(th)
    check(L.grs_shard_bounds_host(srt.ctypes.data, srt.size, 4, spl.ctypes.data, th.ctypes.data,
                                  G, b), "grs_shard_bounds_host")     # the product's arithmetic
    bounds = np.array(list(b), np.int64)
    lb = np.searchsorted(srt, spl, side="left")                        # ... and its restatement
    ub = np.searchsorted(srt, spl, side="right")
    assert np.array_equal(bounds[1:G], np.clip(th.astype(np.int64), lb, ub))
    assert np.all(np.diff(bounds) >= 0)
    cnt = np.diff(bounds).astype(np.uint32)
    mat = np.ascontiguousarray(_all_gather_np(cnt, G, group)).reshape(G, G)
    rc = [int(x) for x in mat[:, me]]
    rk = torch.empty(sum(rc), dtype=torch.int32)
    dist.all_to_all_single(rk, torch.from_numpy(srt.view(np.int32).copy()), output_split_sizes=rc,
                           input_split_sizes=[int(x) for x in cnt], group=group)
    runs = np.split(rk.numpy().view(np.uint32), np.cumsum(rc)[:-1])
    assert all(np.all(r[1:] >= r[:-1]) for r in runs)   # every received run is sorted
    return np.sort(np.concatenate(runs), kind="stable"), mat


def _chunk_thresholds(th: np.ndarray, base: int) -> np.ndarray:
    """grs_shard_chunk_digits: the thresholds of the chunk that starts at shard position base."""
    th = th.astype(np.uint64)
    out = np.where(th == 0xFFFFFFFF, th, np.where(th <= base, 0, th - np.uint64(base)))
    return out.astype(np.uint32)


def sim_chunked_sort(keys: np.ndarray, chunks: int, group=None):
    """The chunked partition-first exchange (run_sharded_chunked, keys only): the same splitters;
    per chunk c of ceil(n / chunks) keys the partition digit with chunk-local thresholds, the
    chunk's count matrix all-gathered, the plan from libgrs's host twin
    grs_shard_chunk_plan_host (chunk-major receive), the chunk's exchange into its planned
    place; then the local sort.  Returns (keys_out, [count matrix per chunk], receive buffer)."""
    L, check = _lib()
    G, me = dist.get_world_size(group), dist.get_rank(group)
    S = int(L.grs_shard_samples_per_rank(G))
    kb = keys.dtype.itemsize
    n = keys.size
    sk, sp = _samples(keys, S)
    spl, th = _splitters(sk, sp, G, me, S, kb, keys.dtype, group)
    every = _buckets(keys, spl, th)
    chunk = (n + chunks - 1) // chunks
    mats, sends = [], []
    for c in range(chunks):
        c0 = min(n, c * chunk)
        part = keys[c0:min(n, c0 + chunk)]
        b = _buckets(part, spl, _chunk_thresholds(th, c0))
        assert np.array_equal(b, every[c0:c0 + part.size])   # same buckets as the whole shard's
        sends.append(part[np.argsort(b, kind="stable")])
        cnt = np.bincount(b, minlength=G).astype(np.uint32)
        mats.append(np.ascontiguousarray(_all_gather_np(cnt, G, group)).reshape(G, G))
    allm = np.ascontiguousarray(np.stack(mats))
    soff = (ctypes.c_uint64 * (chunks * G))()
    roff = (ctypes.c_uint64 * (chunks * G))()
    n_out = ctypes.c_uint64()
    check(L.grs_shard_chunk_plan_host(allm.ctypes.data, chunks, G, me, chunk, soff, roff, ctypes.byref(n_out)),
          "grs_shard_chunk_plan_host")
    wide = np.int64 if kb == 8 else np.int32
    recv = np.zeros(int(n_out.value), keys.dtype)
    base = 0
    for c in range(chunks):
        m = mats[c]
        sc = [int(x) for x in m[me]]
        rc = [int(x) for x in m[:, me]]
        c0 = min(n, c * chunk)
        assert [int(soff[c * G + p]) for p in range(G)] == list(c0 + np.concatenate([[0], np.cumsum(sc)[:-1]]))
        assert [int(roff[c * G + p]) for p in range(G)] == list(base + np.concatenate([[0], np.cumsum(rc)[:-1]]))
        rk = torch.empty(sum(rc), dtype=torch.int64 if kb == 8 else torch.int32)
        dist.all_to_all_single(rk, torch.from_numpy(sends[c].view(wide).copy()), output_split_sizes=rc,
                               input_split_sizes=sc, group=group)
        recv[base:base + sum(rc)] = rk.numpy().view(keys.dtype)
        base += sum(rc)
    assert base == int(n_out.value)
    return np.sort(recv), mats, recv
