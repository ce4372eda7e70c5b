"""GPU test of the multi-GPU path's production code (HipOps + RCCL collectives) at world
size 1, the largest world a single-GPU box offers: one real `nccl` (RCCL) process group, the
splitter all_gather, the counts all_to_all and the all_to_all_single exchange all run, and
the result must equal the oracle's stable sort.  World sizes 2-4 of the same orchestration
run on CPU under gloo (tests/test_sharded_gloo.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl_group(gpu):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=gpu)
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("key_bits,pairs", [(32, False), (32, True), (64, True)])
def test_sharded_sort_world1_rccl(gpu, nccl_group, key_bits, pairs):
    from gpuradixsort_amd.sharded import ShardedSorter

    rng = np.random.default_rng(key_bits + pairs)
    dt = np.uint32 if key_bits == 32 else np.uint64
    n = 1_000_003
    keys = rng.integers(0, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
    keys[::11] = 5
    perm = oracle.stable_argsort(keys)
    s = ShardedSorter(n, key_bits=key_bits, pairs=pairs, device=gpu)
    k = torch.from_numpy(keys).to(gpu)
    v = torch.arange(n, dtype=torch.int64, device=gpu).to(torch.uint32) if pairs else None
    ko, vo = s.sort(k, v)
    torch.cuda.synchronize()
    assert s.last_local_n == n
    assert np.array_equal(ko.cpu().numpy(), keys[perm])
    if pairs:
        assert np.array_equal(vo.cpu().numpy(), perm)
    assert s.count_inversions() == 0
