"""Throughput of the §8f extensions on one MI355X (hipEvents on torch's current stream).

python tools/bench_extras.py [--n N] [--reps R]
Prints one JSON line per operation with its algorithmic bytes per item, GB/s and the fraction
of the 8 TB/s HBM peak:
  scan            grs_exclusive_scan_u32, 2^28 items: 8 B/item (read + write)
  key_transform   grs_key_transform f32, 2^28 items: 8 B/item
  segmented_sort  grs_sort_segmented u32 key + u32 payload, 2^26 items in 2^16, 2^12 and 2^6
                  segments (Gkeys/s; the first two sorted in LDS, the last by the general path)
"""
import argparse
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import gpuradixsort_amd as grs  # noqa: E402

PEAK = 8000.0


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 28)
    ap.add_argument("--reps", type=int, default=10)
    a, _ = ap.parse_known_args()
    dev = torch.device("cuda", 0)
    n = a.n
    L = grs.lib()

    x = torch.empty(n, dtype=torch.int32, device=dev)
    grs.fill_splitmix(x, 1)
    y = torch.empty_like(x)
    scratch = torch.empty((L.grs_scan_scratch_bytes(n) + 3) // 4, dtype=torch.int32, device=dev)
    tot = torch.empty(1, dtype=torch.int32, device=dev)
    import ctypes
    vp = ctypes.c_void_p
    sp = vp(torch.cuda.current_stream().cuda_stream)

    def scan():
        assert L.grs_exclusive_scan_u32(vp(x.data_ptr()), vp(y.data_ptr()), n, vp(tot.data_ptr()),
                                        vp(scratch.data_ptr()), scratch.numel() * 4, sp) == 0
    ms = timed(scan, a.reps)
    gbs = n * 8 / ms / 1e6
    print(json.dumps({"op": "exclusive_scan_u32", "n": n, "ms": round(ms, 4),
                      "GB/s": round(gbs, 1), "frac": round(gbs / PEAK, 4),
                      "bytes_per_item": 8}), flush=True)

    f = x.view(torch.float32)
    ms = timed(lambda: grs.key_transform(f), a.reps)
    gbs = n * 8 / ms / 1e6
    print(json.dumps({"op": "key_transform_f32", "n": n, "ms": round(ms, 4),
                      "GB/s": round(gbs, 1), "frac": round(gbs / PEAK, 4),
                      "bytes_per_item": 8}), flush=True)
    del x, y, f

    m = 1 << 26
    s = grs.RadixSorter(m, key_bits=32, pairs=True)
    k0 = torch.empty(m, dtype=torch.int32, device=dev)
    grs.fill_splitmix(k0, 2)
    k = torch.empty_like(k0)
    v = torch.empty_like(k0)
    ms_copy = timed(lambda: k.copy_(k0), a.reps)
    # 1K-item segments (256-thread LDS sort), 16K-item segments (1024-thread LDS sort); 128K,
    # 1M and 16M-item segments and 64 ragged ones (the segmented LSD: one planner block, one
    # histogram, 4 segmented onesweep passes)
    import numpy as np
    rng = np.random.default_rng(3)
    cuts = np.sort(rng.integers(0, m + 1, 63))
    ragged = torch.from_numpy(np.concatenate([[0], cuts, [m]]).astype(np.int32)).to(dev)
    for segs in (1 << 16, 1 << 12, 1 << 9, 1 << 6, 4, "ragged64"):
        off = ragged if segs == "ragged64" else torch.arange(0, m + 1, m // segs, dtype=torch.int32, device=dev)

        def seg():
            k.copy_(k0)
            s.sort_segmented(k, off, v)
        ms = timed(seg, a.reps) - ms_copy
        print(json.dumps({"op": "sort_segmented_u32_pairs", "n": m, "segments": segs,
                          "ms": round(ms, 4), "Gkeys/s": round(m / ms / 1e6, 2),
                          "note": "restore copy of the keys subtracted"}), flush=True)


def record_sort(n=1 << 24, rb=28):
    """grs_sort_records (the reference's intended use, ParallelSort.h:13-31):
    n 28-byte particles (position float3 at offset 0) sorted by the 30-bit Morton code of their
    position: key extraction, stable (key, index) sort, record gather, copy-back."""
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    rec0 = torch.empty((n, rb), dtype=torch.uint8, device=dev)
    pos = torch.rand((n, 3), generator=g, device=dev) * 2 - 1
    rec0[:, :12] = pos.view(torch.uint8).view(n, 12)
    rec0[:, 12:] = 0
    rec = torch.empty_like(rec0)
    rs = grs.RecordSort(n)
    ms_copy = timed(lambda: rec.copy_(rec0), 10)

    def go():
        rec.copy_(rec0)
        rs.sort(rec, morton=(0, (-1.0, -1.0, -1.0), (1.0, 1.0, 1.0)))
    ms = timed(go, 10) - ms_copy
    print(json.dumps({"op": f"sort_records_morton_{rb}B", "n": n, "ms": round(ms, 4),
                      "Mrecords/s": round(n / ms / 1e3, 1),
                      "record_GB/s": round(n * rb * 2 / ms / 1e6, 1),
                      "note": "extraction + (key, index) sort + gather + copy-back; restore copy subtracted"}),
          flush=True)


def partition(n, g=8, options=None):
    """grs_partition (the multi-GPU exchange's local step): 2^27 u32 keys into g buckets by
    g - 1 splitters at uniform quantiles; 8 B/key algorithmic (read + write)."""
    dev = torch.device("cuda", 0)
    s = grs.RadixSorter(n, key_bits=32, options=options or {})
    k = torch.empty(n, dtype=torch.int32, device=dev)
    grs.fill_splitmix(k, 4)
    out = torch.empty_like(k)
    counts = torch.zeros(16, dtype=torch.int32, device=dev)
    sp = [(i * (1 << 32)) // g for i in range(1, g)]
    ms = timed(lambda: s.partition(k, out, sp, counts), 10)
    print(json.dumps({"op": f"partition_u32_{g}_buckets", "options": options or {}, "n": n, "ms": round(ms, 4),
                      "GB/s": round(n * 8 / ms / 1e6, 1), "frac": round(n * 8 / ms / 1e6 / PEAK, 4),
                      "note": "histogram + one onesweep pass with a splitter digit"}), flush=True)


def host_sort(n):
    """grs_sort_host on 2^27 u32 keys in pageable host memory: the PCIe-inclusive rate."""
    import numpy as np

    s = grs.RadixSorter(n, key_bits=32)
    keys = np.random.default_rng(1).integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    k = keys.copy()
    s.sort_host(k)
    import time
    ts = []
    for _ in range(3):
        k[:] = keys
        t = time.perf_counter()
        s.sort_host(k)
        ts.append(time.perf_counter() - t)
    ms = sorted(ts)[1] * 1e3
    print(json.dumps({"op": "sort_host_u32 (PCIe both ways, pageable)", "n": n, "ms": round(ms, 3),
                      "Gkeys/s": round(n / ms / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
    record_sort()
    partition(1 << 27)
    if "--partition-ab" in sys.argv:
        partition(1 << 27, options={"rank": "match"})
        partition(1 << 27, g=4)
        partition(1 << 27, g=4, options={"rank": "match"})
    host_sort(1 << 27)
