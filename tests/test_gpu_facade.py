"""GPU tests of the reference-shaped host surfaces: the C++ facade (include/
grs_parallel_sort.hpp, driven by the grs_demo binary exactly like main.cpp:117-160) and the
Python mirror (OriginalDataSsbo / ParallelSort / RecordSort)."""
import os
import subprocess

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(REPO, "gpuradixsort_amd", "grs_demo")


@pytest.mark.parametrize("n", [0, 1, 16, 1025, 1_000_000, 3_000_001])
def test_cpp_facade_demo(gpu, n):
    """OriginalDataSsbo + ParallelSort + Sort() twice on a shuffled 0..N-1 (the reference's
    demo input, main.cpp:120-125) -> exactly 0..N-1.  N = 1,000,000 is MAX_DATA_COUNT
    (main.cpp:61); 3,000,001 is beyond the reference's 1,048,576 capacity."""
    r = subprocess.run([DEMO, str(n), "7"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sorted=yes" in r.stdout


def test_python_mirror_parallel_sort(gpu):
    import gpuradixsort_amd as grs

    kat = [12, 1, 9, 2, 0, 11, 7, 3, 4, 15, 8, 5, 14, 13, 10, 6]   # main.cpp:128-143
    ssbo = grs.OriginalDataSsbo(len(kat))
    ssbo.Upload(kat)
    ps = grs.ParallelSort(ssbo)
    ps.Sort()
    torch.cuda.synchronize()
    assert ssbo.Download().numpy().tolist() == list(range(16))

    rng = np.random.default_rng(5)
    keys = rng.integers(0, 2**32, 777_777, dtype=np.uint64).astype(np.uint32)
    keys[::7] = 0xFFFFFFFF
    ssbo = grs.OriginalDataSsbo(keys.size)
    ssbo.Upload(keys)
    ps = grs.ParallelSort(ssbo)
    ps.Sort()
    ps.Sort()   # sorting sorted data again is a no-op
    torch.cuda.synchronize()
    assert np.array_equal(ssbo.Download().numpy(), np.sort(keys))


def test_record_sort_gathers_whole_records(gpu):
    """The reference's intended use (ParallelSort.h:13-31): sort structs (here 24-byte
    particles) by a 32-bit key (a Morton code), via (key, index) pairs + K5 gather."""
    import gpuradixsort_amd as grs

    rng = np.random.default_rng(9)
    n = 200_003
    rec = rng.integers(0, 256, (n, 24), dtype=np.uint8)
    keys = rng.integers(0, 1 << 12, n).astype(np.uint32)           # many ties: stability
    perm = oracle.stable_argsort(keys)
    d_rec = torch.from_numpy(rec).to(gpu)
    d_keys = torch.from_numpy(keys).to(gpu)
    rs = grs.RecordSort(n)
    rs.sort(d_rec, d_keys)
    torch.cuda.synchronize()
    assert np.array_equal(d_rec.cpu().numpy(), rec[perm])
    assert np.array_equal(d_keys.cpu().numpy(), keys[perm])
    # odd record size (byte path of the gather)
    rec7 = rng.integers(0, 256, (n, 7), dtype=np.uint8)
    d7 = torch.from_numpy(rec7).to(gpu)
    d_keys = torch.from_numpy(keys).to(gpu)
    rs.sort(d7, d_keys)
    torch.cuda.synchronize()
    assert np.array_equal(d7.cpu().numpy(), rec7[perm])
