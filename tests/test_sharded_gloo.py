"""Multi-process CPU tests (gloo, world_size 2-4) of the multi-GPU orchestration in
gpuradixsort_amd/sharded.py: splitter selection, count exchange, all-to-all-v, and the
source-rank-order concatenation that keeps the global sort stable.

The device steps (partition, local sort) are swapped for numpy stand-ins HERE ONLY; the
collective calls and bookkeeping are the production code.  The concatenated outputs of all
ranks must equal the oracle's stable sort of the whole input (keys and global indices)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class NumpyOps:
    """CPU stand-in for HipOps (tests only)."""

    def __init__(self, key_bits, pairs):
        self.key_bits, self.pairs = key_bits, pairs

    def partition(self, keys, vals, keys_out, vals_out, splitters, counts):
        n = keys.numel()
        k = keys.numpy()
        b = np.searchsorted(np.asarray(splitters, k.dtype), k, side="right")
        perm = np.argsort(b, kind="stable")
        keys_out[:n] = torch.from_numpy(k[perm])
        if vals is not None:
            vals_out[:n] = torch.from_numpy(vals.numpy()[perm])
        counts.copy_(torch.from_numpy(np.bincount(b, minlength=counts.numel()).astype(np.uint32)))

    def local_sort(self, keys, vals, n):
        k = keys[:n].numpy()
        perm = np.argsort(k, kind="stable")
        keys[:n] = torch.from_numpy(k[perm].copy())
        if vals is not None:
            vals[:n] = torch.from_numpy(vals[:n].numpy()[perm].copy())

    def set_profiling(self, ring):
        pass


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_local, key_bits, pairs, dist_name, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gpuradixsort_amd.sharded import ShardedSorter

    dt = np.uint32 if key_bits == 32 else np.uint64
    rng = np.random.default_rng(1234)   # same global input on every rank
    total = n_local * world
    if dist_name == "uniform":
        allk = rng.integers(0, np.iinfo(dt).max, total, dtype=dt, endpoint=True)
    elif dist_name == "few_unique":
        allk = rng.integers(0, 5, total).astype(dt) * dt(1 << (key_bits - 4))
    elif dist_name == "all_equal":
        allk = np.full(total, 42, dt)
    else:   # skewed: 90 % of the keys in one narrow range
        allk = np.where(rng.random(total) < 0.9, rng.integers(0, 1000, total),
                        rng.integers(0, np.iinfo(dt).max, total, dtype=dt)).astype(dt)
    shard = allk[rank * n_local:(rank + 1) * n_local].copy()
    keys = torch.from_numpy(shard)
    vals = torch.arange(rank * n_local, (rank + 1) * n_local, dtype=torch.int64).to(torch.uint32) \
        if pairs else None
    s = ShardedSorter(n_local, key_bits=key_bits, pairs=pairs, device=torch.device("cpu"),
                      oversample=64, ops=NumpyOps(key_bits, pairs))
    ko, vo = s.sort(keys, vals)
    np.save(os.path.join(out_dir, f"k{rank}.npy"), ko.numpy())
    if pairs:
        np.save(os.path.join(out_dir, f"v{rank}.npy"), vo.numpy())
    np.save(os.path.join(out_dir, "all.npy"), allk) if rank == 0 else None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_local,key_bits,pairs,dist_name", [
    (2, 5000, 32, True, "uniform"),
    (2, 4096, 64, True, "few_unique"),
    (3, 3001, 32, True, "skewed"),
    (4, 2500, 32, False, "uniform"),
    (4, 1000, 32, True, "all_equal"),
    (2, 0, 32, True, "uniform"),
])
def test_sharded_sort_equals_global_stable_sort(tmp_path, world, n_local, key_bits, pairs,
                                                 dist_name):
    import oracle

    port = _free_port()
    mp.spawn(_worker, args=(world, port, n_local, key_bits, pairs, dist_name, str(tmp_path)),
             nprocs=world, join=True)
    allk = np.load(tmp_path / "all.npy")
    keys = np.concatenate([np.load(tmp_path / f"k{r}.npy") for r in range(world)])
    perm = oracle.stable_argsort(allk)
    assert np.array_equal(keys, allk[perm])
    if pairs:
        vals = np.concatenate([np.load(tmp_path / f"v{r}.npy") for r in range(world)])
        assert np.array_equal(vals, perm)
