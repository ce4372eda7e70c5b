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


def test_record_key_buffers_at_capacity_then_smaller_n(gpu):
    """grs_records_key_buffers hands out the sorter's key / index buffers once (at capacity);
    a later grs_sort_records_by_keys of FEWER records must not lay its record copy over those
    buffers (they are their own capacity-sized allocation; the record copy is sized per call),
    and a larger record size grows only the per-call copy: the handed-out buffers stay where
    they are and stay valid."""
    import ctypes

    import gpuradixsort_amd as grs
    from gpuradixsort_amd._lib import lib

    L = lib()
    cap, rb = 1 << 20, 16
    s = grs.RadixSorter(cap, key_bits=32, pairs=True)
    keys_p, idx_p = ctypes.c_void_p(), ctypes.c_void_p()
    assert L.grs_records_key_buffers(s._h, cap, rb, ctypes.byref(keys_p), ctypes.byref(idx_p)) == 0
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(21)
    for n in (cap, cap // 2, 4097, 1):
        rec = rng.integers(0, 256, (n, rb), dtype=np.uint8)
        keys = rng.integers(0, 1 << 10, n).astype(np.uint32)   # ties: the sort must be stable
        d_rec = torch.from_numpy(rec).to(gpu)
        d_keys = torch.from_numpy(keys).to(gpu)
        # the caller's "key kernel": key and index into the sorter-owned buffers
        assert L.grs_copy_u32(ctypes.c_void_p(d_keys.data_ptr()), keys_p, n, stream) == 0
        assert L.grs_iota_u32(idx_p, n, 0, stream) == 0
        assert L.grs_sort_records_by_keys(s._h, ctypes.c_void_p(d_rec.data_ptr()), n, rb, keys_p,
                                          idx_p, stream) == 0
        torch.cuda.synchronize()
        assert np.array_equal(d_rec.cpu().numpy(), rec[oracle.stable_argsort(keys)]), n
    # a larger record size grows only the per-call record copy; the key buffers do not move
    n = 3001
    big = rng.integers(0, 256, (n, 64), dtype=np.uint8)
    keys = rng.integers(0, 1 << 8, n).astype(np.uint32)
    d_big = torch.from_numpy(big).to(gpu)
    d_keys = torch.from_numpy(keys).to(gpu)
    assert L.grs_copy_u32(ctypes.c_void_p(d_keys.data_ptr()), keys_p, n, stream) == 0
    assert L.grs_iota_u32(idx_p, n, 0, stream) == 0
    assert L.grs_sort_records_by_keys(s._h, ctypes.c_void_p(d_big.data_ptr()), n, 64, keys_p,
                                      idx_p, stream) == 0
    torch.cuda.synchronize()
    assert np.array_equal(d_big.cpu().numpy(), big[oracle.stable_argsort(keys)])
    k2, i2 = ctypes.c_void_p(), ctypes.c_void_p()
    assert L.grs_records_key_buffers(s._h, cap, 64, ctypes.byref(k2), ctypes.byref(i2)) == 0
    assert (k2.value, i2.value) == (keys_p.value, idx_p.value)


@pytest.mark.parametrize("kb", [32, 64])
def test_record_sort_key_extraction_hook(gpu, kb):
    """grs_sort_records (the K1 hook in the C-ABI): 28-byte particles sorted by the Morton
    code of their position, and 24-byte records by a signed / float / unsigned field, against
    the oracle's extraction + stable argsort (parity unpinned: the reference names Morton
    codes, ParallelSort.h:13-31, but defines none)."""
    import gpuradixsort_amd as grs

    rng = np.random.default_rng(kb + 3)
    n = 250_007
    # particles: pos (3 f32) | vel (3 f32) | id
    pos = (rng.random((n, 3), dtype=np.float32) * 2.4 - 1.2).astype(np.float32)
    pos[::101] = np.nan
    pos[::53, 1] = pos[7, 1]          # ties in one axis
    rec = np.zeros((n, 28), np.uint8)
    rec[:, :12] = pos.view(np.uint8).reshape(n, 12)
    rec[:, 24:28] = np.arange(n, dtype=np.uint32).view(np.uint8).reshape(n, 4)
    lo, hi = (-1.0, -1.0, -1.0), (1.0, 1.0, 1.0)
    code = oracle.morton3_np(pos, lo, hi, kb)
    perm = oracle.stable_argsort(code)
    rs = grs.RecordSort(n, key_bits=kb)
    d = torch.from_numpy(rec).to(gpu)
    rs.sort(d, morton=(0, lo, hi))
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), rec[perm])
    # fields: u32 / i32 / f32 (kb 32) or u64 / i64 / f64 (kb 64) at byte offset 8
    rec24 = rng.integers(0, 256, (n, 24), dtype=np.uint8)
    for transform in (0, 1, 2):
        if transform == 2:
            f = rng.standard_normal(n).astype(np.float32 if kb == 32 else np.float64)
            f[::77] = 0.0
            rec24[:, 8:8 + kb // 8] = f.view(np.uint8).reshape(n, kb // 8)
        keys = oracle.extract_keys_np(rec24, 8, kb, transform)
        perm = oracle.stable_argsort(keys)
        d = torch.from_numpy(rec24).to(gpu)
        rs.sort(d, field=8, transform=transform)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), rec24[perm]), transform
    # unaligned field (byte offset 3 of 13-byte records)
    rec13 = rng.integers(0, 256, (n, 13), dtype=np.uint8)
    keys = oracle.extract_keys_np(rec13, 3, kb, 0)
    perm = oracle.stable_argsort(keys)
    d = torch.from_numpy(rec13).to(gpu)
    rs.sort(d, field=3)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), rec13[perm])


def test_cpp_facade_particles_by_morton(gpu):
    """C++ ParallelSort(RecordSsbo<Particle>, MortonKey(...)) — grs_demo particles mode,
    checked in the demo against a host std::stable_sort by the same Morton code."""
    r = subprocess.run([DEMO, "particles", "300001", "5"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sorted=yes" in r.stdout


@pytest.mark.parametrize("n", [1, 4097, 300_001])
def test_cpp_key_functor(gpu, n):
    """A user-defined key functor (the reference's K1 hook, OriginalDataToIntermediateData
    .comp:12-19): C++ ParallelSortBy<Particle, DistanceKey> sorts 28-byte particles by their
    float distance from a point (grs::OrderedBits), the extraction kernel instantiated by the
    demo's own hipcc; checked in the demo against a host std::stable_sort by the same functor,
    after a second Sort() of the sorted records (stability under heavy ties)."""
    r = subprocess.run([DEMO, "distance", str(n), "3"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sorted=yes" in r.stdout
