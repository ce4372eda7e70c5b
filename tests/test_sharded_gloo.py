"""Multi-process CPU tests (gloo, world_size 2-4) of the multi-GPU sort's orchestration
(grs_sort_sharded): sampling, on-device splitter choice with ties broken by global index,
count exchange and plan, all-to-all, source-rank-order concatenation, local stable sort.

tests/sharded_sim.py replays the device steps on the host with gloo collectives and libgrs's
host twins of the splitter and plan arithmetic.  The concatenated outputs of all ranks must
equal the oracle's stable sort of the whole input (keys and global indices), and the ranks'
loads must stay balanced even when the input is all one key."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _input(dist_name, total, key_bits):
    dt = np.uint32 if key_bits == 32 else np.uint64
    rng = np.random.default_rng(1234)   # same global input on every rank
    if dist_name == "uniform":
        return rng.integers(0, np.iinfo(dt).max, total, dtype=dt, endpoint=True)
    if dist_name == "few_unique":
        return rng.integers(0, 5, total).astype(dt) * dt(1 << (key_bits - 4))
    if dist_name == "all_equal":
        return np.full(total, 42, dt)
    # skewed: 90 % of the keys in one narrow range
    return np.where(rng.random(total) < 0.9, rng.integers(0, 1000, total),
                    rng.integers(0, np.iinfo(dt).max, total, dtype=dt)).astype(dt)


def _worker(rank, world, port, n_local, key_bits, pairs, dist_name, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sharded_sim

    allk = _input(dist_name, n_local * world, key_bits)
    shard = allk[rank * n_local:(rank + 1) * n_local].copy()
    vals = np.arange(rank * n_local, (rank + 1) * n_local, dtype=np.uint32) if pairs else None
    ko, vo, mat = sharded_sim.sim_sharded_sort(shard, vals)
    np.save(os.path.join(out_dir, f"k{rank}.npy"), ko)
    if pairs:
        np.save(os.path.join(out_dir, f"v{rank}.npy"), vo)
    if rank == 0:
        np.save(os.path.join(out_dir, "all.npy"), allk)
        np.save(os.path.join(out_dir, "mat.npy"), mat)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_local,key_bits,pairs,dist_name", [
    (2, 5000, 32, True, "uniform"),
    (2, 4096, 64, True, "few_unique"),
    (3, 3001, 32, True, "skewed"),
    (4, 2500, 32, False, "uniform"),
    (4, 1000, 32, True, "all_equal"),
    (4, 20000, 32, True, "few_unique"),
    (3, 7000, 64, False, "all_equal"),
    (2, 0, 32, True, "uniform"),
    (8, 2000, 32, True, "skewed"),          # C4's rank count (G in {1, 2, 4, 8})
])
def test_sharded_sort_equals_global_stable_sort(tmp_path, world, n_local, key_bits, pairs,
                                                 dist_name):
    import oracle

    port = _free_port()
    mp.spawn(_worker, args=(world, port, n_local, key_bits, pairs, dist_name, str(tmp_path)),
             nprocs=world, join=True)
    allk = np.load(tmp_path / "all.npy")
    outs = [np.load(tmp_path / f"k{r}.npy") for r in range(world)]
    keys = np.concatenate(outs)
    perm = oracle.stable_argsort(allk)
    assert np.array_equal(keys, allk[perm])
    if pairs:
        vals = np.concatenate([np.load(tmp_path / f"v{r}.npy") for r in range(world)])
        assert np.array_equal(vals, perm)
    # balance: ties are split by global index, so duplicate-heavy inputs stay balanced
    if n_local and dist_name in ("all_equal", "few_unique"):
        sizes = np.array([o.size for o in outs], np.float64)
        assert sizes.max() / sizes.mean() <= 1.1, sizes
    mat = np.load(tmp_path / "mat.npy")
    assert mat.sum() == n_local * world


def _worker_presorted(rank, world, port, n_local, dist_name, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sharded_sim

    allk = _input(dist_name, n_local * world, 32)
    ko, mat = sharded_sim.sim_presorted_sort(allk[rank * n_local:(rank + 1) * n_local].copy())
    np.save(os.path.join(out_dir, f"k{rank}.npy"), ko)
    if rank == 0:
        np.save(os.path.join(out_dir, "all.npy"), allk)
        np.save(os.path.join(out_dir, "mat.npy"), mat)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_local,dist_name", [
    (2, 5000, "uniform"), (3, 3001, "skewed"), (4, 2500, "all_equal"), (4, 20000, "few_unique"),
    (2, 0, "uniform"), (8, 3000, "few_unique"),
])
def test_presorted_exchange_equals_sort(tmp_path, world, n_local, dist_name):
    """The presorted exchange's orchestration (u32 keys): sorted-shard samples, the product's
    splitters, clamp bounds, source-order runs; sorted and balanced."""
    port = _free_port()
    mp.spawn(_worker_presorted, args=(world, port, n_local, dist_name, str(tmp_path)),
             nprocs=world, join=True)
    allk = np.load(tmp_path / "all.npy")
    outs = [np.load(tmp_path / f"k{r}.npy") for r in range(world)]
    assert np.array_equal(np.concatenate(outs), np.sort(allk))
    if n_local and dist_name in ("all_equal", "few_unique"):
        sizes = np.array([o.size for o in outs], np.float64)
        assert sizes.max() / sizes.mean() <= 1.1, sizes
    assert np.load(tmp_path / "mat.npy").sum() == n_local * world


def _worker_chunked(rank, world, port, n_local, key_bits, chunks, dist_name, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sharded_sim

    allk = _input(dist_name, n_local * world, key_bits)
    ko, mats, _ = sharded_sim.sim_chunked_sort(allk[rank * n_local:(rank + 1) * n_local].copy(), chunks)
    np.save(os.path.join(out_dir, f"k{rank}.npy"), ko)
    if rank == 0:
        np.save(os.path.join(out_dir, "all.npy"), allk)
        np.save(os.path.join(out_dir, "mats.npy"), np.stack(mats))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_local,key_bits,chunks,dist_name", [
    (2, 5000, 32, 4, "uniform"), (3, 3001, 64, 3, "skewed"), (4, 2500, 32, 1, "all_equal"),
    (4, 20000, 32, 7, "few_unique"), (2, 3, 32, 4, "uniform"), (2, 0, 32, 4, "uniform"),
    (8, 3000, 32, 4, "skewed"), (8, 2001, 64, 16, "few_unique"),
])
def test_chunked_exchange_equals_sort(tmp_path, world, n_local, key_bits, chunks, dist_name):
    """The chunked partition-first exchange's orchestration (keys only; GRS_OPT_EXCHANGE = 3):
    chunk-local thresholds give every key the bucket of the whole shard, the chunk-major plan of
    libgrs's host twin places every chunk's runs, and the ranks' outputs concatenate to the
    sorted input, balanced on duplicate-heavy inputs."""
    port = _free_port()
    mp.spawn(_worker_chunked, args=(world, port, n_local, key_bits, chunks, dist_name, str(tmp_path)),
             nprocs=world, join=True)
    allk = np.load(tmp_path / "all.npy")
    outs = [np.load(tmp_path / f"k{r}.npy") for r in range(world)]
    assert np.array_equal(np.concatenate(outs), np.sort(allk))
    if n_local and dist_name in ("all_equal", "few_unique"):
        sizes = np.array([o.size for o in outs], np.float64)
        assert sizes.max() / sizes.mean() <= 1.1, sizes
    assert np.load(tmp_path / "mats.npy").sum() == n_local * world


def test_host_twins_validate_arguments():
    import ctypes

    from gpuradixsort_amd import _lib

    L = _lib.lib()
    assert L.grs_shard_samples_per_rank(8) == 1024 and L.grs_shard_samples_per_rank(16) == 512
    out = (ctypes.c_uint64 * 4)()
    assert L.grs_shard_plan_host(None, 2, 0, out, out, ctypes.byref(ctypes.c_uint64())) == _lib.GRS_EINVAL
    mat = np.array([[3, 1], [2, 5]], np.uint32)
    so, ro, n = (ctypes.c_uint64 * 2)(), (ctypes.c_uint64 * 2)(), ctypes.c_uint64()
    assert L.grs_shard_plan_host(mat.ctypes.data, 2, 1, so, ro, ctypes.byref(n)) == 0
    assert list(so) == [0, 2] and list(ro) == [0, 1] and n.value == 6
    # two chunks of 10: chunk 1's sends start at 10, its receives after chunk 0's 6
    mats = np.array([[[3, 1], [2, 5]], [[4, 0], [1, 1]]], np.uint32)
    so4, ro4 = (ctypes.c_uint64 * 4)(), (ctypes.c_uint64 * 4)()
    assert L.grs_shard_chunk_plan_host(mats.ctypes.data, 2, 2, 1, 10, so4, ro4, ctypes.byref(n)) == 0
    assert list(so4) == [0, 2, 10, 11] and list(ro4) == [0, 1, 6, 6] and n.value == 7
    assert L.grs_shard_chunk_plan_host(None, 2, 2, 1, 10, so4, ro4, ctypes.byref(n)) == _lib.GRS_EINVAL
