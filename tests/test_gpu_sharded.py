"""GPU tests of the multi-GPU boundary grs_sort_sharded (include/grs.h) at world size 1, the
largest world a single-GPU box offers: a real RCCL communicator created by libgrs, the
sample all-gather, the on-device splitter step, the partition pass, the count all-gather and
host plan, the grouped send/recv (self copy at world 1) and the local sort all run through
the C-ABI; the result must equal the oracle's stable sort.  World sizes 2-4 of the same
orchestration run on CPU under gloo (tests/test_sharded_gloo.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def world1(gpu):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)   # only carries the RCCL id
    from gpuradixsort_amd.sharded import RcclComm

    comm = RcclComm(device=gpu.index)
    yield comm
    comm.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("path", ["general", "general_contig", "general_partition", "one_rank"])
@pytest.mark.parametrize("key_bits,pairs,dist_name", [(32, False, "uniform"), (32, True, "ties"),
                                                      (64, True, "uniform"), (64, False, "ties"),
                                                      (32, True, "all_equal")])
def test_sharded_sort_world1_rccl(gpu, world1, monkeypatch, path, key_bits, pairs, dist_name):
    """path "general": option sharded_path=general makes the one-rank call take the G-rank path
    (samples, all-gathers, device splitters, partition into per-bucket regions of the send
    buffer, bucket sizes from the look-back, count matrix, host sync, grouped send/recv with
    the self copy, local sort) -- u32 keys without payload take the presorted exchange there
    (local sort, encode, exchange of encoded words, decode + merge) unless "general_partition"
    forces the partition-first one; "general_contig": partition-first with the bucket histogram
    and contiguous send buckets (sharded_send=contig); "one_rank": the copy + local sort."""
    from gpuradixsort_amd.sharded import ShardedSorter

    opts = {}
    if path.startswith("general"):
        opts["sharded_path"] = "general"
    if path == "general_contig":
        opts["sharded_send"] = "contig"
    if path in ("general_contig", "general_partition"):
        opts["exchange"] = "partition"

    rng = np.random.default_rng(key_bits + pairs)
    dt = np.uint32 if key_bits == 32 else np.uint64
    n = 1_000_003
    keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
    if dist_name == "ties":
        keys[::11] = 5
    elif dist_name == "all_equal":
        keys[:] = 9
    perm = oracle.stable_argsort(keys)
    s = ShardedSorter(n, key_bits=key_bits, pairs=pairs, device=gpu, comm=world1, options=opts)
    k = torch.from_numpy(keys).to(gpu)
    v = torch.arange(n, dtype=torch.int64, device=gpu).to(torch.uint32) if pairs else None
    for _ in range(2):   # repeated calls reuse the sorter's scratch
        ko, vo = s.sort(k.clone(), v.clone() if pairs else None)
        assert s.last_n_out == n
        assert np.array_equal(ko.cpu().numpy(), keys[perm])
        if pairs:
            assert np.array_equal(vo.cpu().numpy(), perm)
    assert s.count_inversions() == 0
    if path.startswith("general"):     # exchange phases of the last call (profiling on)
        s.set_profiling(2)
        s.sort(k.clone(), v.clone() if pairs else None)
        xt = s.exchange_timing()
        assert xt["bytes_sent"] == 0 and xt["bytes_received"] == 0     # one rank: self copy only
        assert xt["total_ms"] >= xt["exchange_ms"] >= 0.0
        assert xt["exchange"] == ("presorted" if (key_bits == 32 and not pairs and path == "general")
                                  else "partition-first")
    s.sorter.close()


@pytest.mark.parametrize("key_bits,n,chunks,dist_name", [(32, 1_000_003, 4, "uniform"), (32, 300_001, 1, "ties"),
                                                         (64, 777_777, 7, "uniform"), (32, 5, 4, "uniform"),
                                                         (32, 60_000_013, 4, "uniform"), (64, 1_000_000, 16, "ties")])
def test_sharded_chunked_world1_rccl(gpu, world1, key_bits, n, chunks, dist_name):
    """The chunked partition-first exchange (exchange=chunked, keys only) on a one-rank RCCL
    communicator: chunk digits, one partition per chunk on the caller's stream, per chunk the
    count all-gather, host read, and send / recv (self copy) on the second stream, the local
    sort after it -- sorted, with more chunks than keys, and past 48M keys (MSD local sort)."""
    from gpuradixsort_amd.sharded import ShardedSorter

    rng = np.random.default_rng(n + chunks)
    dt = np.uint32 if key_bits == 32 else np.uint64
    keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
    if dist_name == "ties":
        keys[::7] = 3
    s = ShardedSorter(n, key_bits=key_bits, device=gpu, comm=world1,
                      options={"sharded_path": "general", "exchange": "chunked", "x_chunks": chunks})
    k = torch.from_numpy(keys).to(gpu)
    want = np.sort(keys)
    for _ in range(2):
        ko, _ = s.sort(k.clone())
        assert s.last_n_out == n
        assert np.array_equal(ko.cpu().numpy(), want)
    s.set_profiling(2)
    s.sort(k.clone())
    xt = s.exchange_timing()
    assert xt["bytes_sent"] == 0 and xt["total_ms"] >= xt["exchange_ms"] >= 0.0
    s.sorter.check_error()
    assert s.sorter.check_guards() == 0
    s.sorter.close()


@pytest.mark.parametrize("path", ["general", "one_rank"])
def test_sharded_prefix_n(gpu, world1, monkeypatch, path):
    """n < keys.numel(): only the first n items take part (samples, partition, exchange,
    sort), and the tail of the input tensor is left alone."""
    from gpuradixsort_amd.sharded import ShardedSorter

    opts = {"sharded_path": "general"} if path == "general" else {}
    rng = np.random.default_rng(9)
    total, n = 300_000, 123_457
    keys = rng.integers(0, 2**32, total, dtype=np.uint64).astype(np.uint32)
    s = ShardedSorter(total, key_bits=32, pairs=True, device=gpu, comm=world1, options=opts)
    k = torch.from_numpy(keys).to(gpu)
    v = torch.arange(total, dtype=torch.int64, device=gpu).to(torch.uint32)
    ko, vo = s.sort(k, v, n=n)
    perm = oracle.stable_argsort(keys[:n])
    assert s.last_n_out == n
    assert np.array_equal(ko.cpu().numpy(), keys[:n][perm])
    assert np.array_equal(vo.cpu().numpy(), perm)
    assert np.array_equal(k[n:].cpu().numpy(), keys[n:])
    s.sorter.close()


def test_records_then_sharded_scratch(gpu, world1, monkeypatch):
    """A record sort, then sharded sorts on the same sorter (their scratch buffers are
    allocated on first use and must not free each other's), then the record sort again."""
    import gpuradixsort_amd as grs
    from gpuradixsort_amd.sharded import ShardedSorter

    n = 200_003
    s = ShardedSorter(n, key_bits=32, pairs=True, device=gpu, comm=world1,
                      options={"sharded_path": "general"})
    rs = grs.RecordSort(n, key_bits=32)
    rs._sorter.close()
    rs._sorter = s.sorter                      # one libgrs sorter for both entry points
    rng = np.random.default_rng(3)
    rec = rng.integers(0, 2**32, (n, 3), dtype=np.uint64).astype(np.uint32)
    for _ in range(2):
        r = torch.from_numpy(rec.copy()).to(gpu)
        rs.sort(r, field=4)
        perm = oracle.stable_argsort(rec[:, 1].copy())
        assert np.array_equal(r.cpu().numpy(), rec[perm])
        keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        ko, vo = s.sort(torch.from_numpy(keys).to(gpu),
                        torch.arange(n, dtype=torch.int64, device=gpu).to(torch.uint32))
        assert np.array_equal(ko.cpu().numpy(), np.sort(keys, kind="stable"))
    s.sorter.close()


def test_sharded_capacity_errors(gpu, world1):
    import gpuradixsort_amd as grs
    from gpuradixsort_amd.sharded import ShardedSorter

    s = ShardedSorter(1000, key_bits=32, device=gpu, comm=world1)
    k = torch.zeros(2000, dtype=torch.uint32, device=gpu)
    with pytest.raises(ValueError):
        s.sort(k)                       # shard larger than capacity_local
    ko, _ = s.sort(k, n=0)              # empty shard
    assert ko.numel() == 0
    import ctypes

    from gpuradixsort_amd import _lib

    n_out = ctypes.c_size_t()
    rc = _lib.lib().grs_sort_sharded(s.sorter._h, None, None, 0, None, None, 0,
                                     ctypes.byref(n_out), None, None)
    assert rc == _lib.GRS_EINVAL        # NULL communicator / output
    s.sorter.close()


@pytest.mark.parametrize("key_bits,pairs", [(32, True), (64, False), (64, True), (32, False)])
def test_region_spill_redo(gpu, world1, key_bits, pairs):
    """The partition-first exchange's region send buffer (include/grs.h GRS_OPT_SHARDED_SEND):
    a bucket larger than its region spills into the next one, the count matrix shows it at
    the host synchronisation and the partition is redone into contiguous buckets.  The test
    hook sharded_send=shrunk (regions of n / 2G) makes every full bucket spill, so the redo
    runs on one rank too: u32 pairs (the joint key + payload scratch), u64 keys and u64 pairs,
    2^20 + 3 items; the output must be the exact stable sort and the redo counted."""
    from gpuradixsort_amd.sharded import ShardedSorter

    rng = np.random.default_rng(31 + key_bits + pairs)
    dt = np.uint32 if key_bits == 32 else np.uint64
    n = (1 << 20) + 3
    keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
    keys[::5] = 77                                   # ties: stability across the redo
    perm = oracle.stable_argsort(keys)
    s = ShardedSorter(n, key_bits=key_bits, pairs=pairs, device=gpu, comm=world1,
                      options={"sharded_path": "general", "exchange": "partition",
                               "sharded_send": "shrunk"})
    k = torch.from_numpy(keys).to(gpu)
    v = torch.arange(n, dtype=torch.int64, device=gpu).to(torch.uint32) if pairs else None
    before = s.redo_count()
    for i in range(2):
        ko, vo = s.sort(k.clone(), v.clone() if pairs else None)
        assert s.redo_count() == before + i + 1
        assert s.last_n_out == n
        assert np.array_equal(ko.cpu().numpy(), keys[perm])
        if pairs:
            assert np.array_equal(vo.cpu().numpy(), perm)
    # the default regions (even share + 25 % + 64K) hold a one-rank bucket: no redo
    s.sorter.set_option("sharded_send", "regions")
    ko, _ = s.sort(k.clone(), v.clone() if pairs else None)
    assert s.redo_count() == before + 2
    assert np.array_equal(ko.cpu().numpy(), keys[perm])
    s.sorter.close()


@pytest.mark.parametrize("n", [300_007, 1 << 20])
@pytest.mark.parametrize("dist_name", ["uniform", "ties", "span_redo"])
def test_presorted_out_of_place_msd(gpu, world1, n, dist_name):
    """The presorted exchange sorts its shard OUT OF PLACE (input -> the output tensor): with
    option msd=always that is the MSD schedule's src_in path (the sample, P1 and P1's redo read
    the caller's input; the result lands in the output).  span_redo: keys below 2^20 with a few
    top-bit keys where the span guess does not look, so P1's exact span redoes it.  Output ==
    the stable sort; the input tensor is left as it was."""
    from gpuradixsort_amd.sharded import ShardedSorter

    rng = np.random.default_rng(n + len(dist_name))
    keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    if dist_name == "ties":
        keys[::3] = keys[1]
    elif dist_name == "span_redo":
        keys = rng.integers(0, 1 << 20, n, dtype=np.uint64).astype(np.uint32)
        keys[[100, 101, n // 2 + 100, n - 100]] |= np.uint32(1 << 31)   # off the 64 guess chunks
    s = ShardedSorter(n, key_bits=32, device=gpu, comm=world1,
                      options={"sharded_path": "general", "msd": "always"})
    k = torch.from_numpy(keys).to(gpu)
    ko, _ = s.sort(k)
    assert s.last_n_out == n
    assert np.array_equal(ko.cpu().numpy(), np.sort(keys, kind="stable"))
    assert np.array_equal(k.cpu().numpy(), keys)
    assert s.sorter.check_guards() == 0
    s.sorter.close()
