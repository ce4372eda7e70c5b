"""Histogram laboratory driver (tools/histlab.hip): interleaved timing of upfront-histogram
variants on 2^27 uniform u32 keys, with a correctness check against torch.bincount.

python tools/histlab.py [--n N] [--rounds R] [--variants id:grid,...]
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import gpuradixsort_amd as grs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 27)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--variants", default="0:2048,0:1280,1:2048,2:2048,3:2048")
    a = ap.parse_args()
    L = ctypes.CDLL(os.path.join(HERE, "libhistlab.so"))
    vp = ctypes.c_void_p
    dev = torch.device("cuda", 0)
    sp = vp(torch.cuda.current_stream().cuda_stream)
    keys = torch.empty(a.n, dtype=torch.uint32, device=dev)
    grs.fill_splitmix(keys, 0x6A09E667F3BCC908 + 4)
    hist = torch.zeros(8192, dtype=torch.uint32, device=dev)
    k64 = keys.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    want = torch.cat([torch.bincount((k64 >> (8 * p)) & 255, minlength=256) for p in range(4)])
    del k64
    variants = [tuple(int(x) for x in v.split(":")) for v in a.variants.split(",")]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {v: [] for v in variants}
    ok = {}
    for r in range(a.rounds):
        for v in variants:
            hist.zero_()
            torch.cuda.synchronize()
            e0.record()
            rc = L.histlab_run(v[0], v[1], vp(keys.data_ptr()), ctypes.c_uint32(a.n),
                               vp(hist.data_ptr()), sp)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, (v, rc)
            times[v].append(e0.elapsed_time(e1))
            if r == 0:
                ok[v] = torch.equal(hist[:1024].to(torch.int64), want)
    for v in variants:
        med = statistics.median(times[v])
        print(f"variant {v[0]:2d} grid {v[1]:5d}: median {med:8.4f} ms  min {min(times[v]):8.4f}"
              f"  {a.n * 4 / med / 1e6:8.1f} GB/s  hist {'OK' if ok[v] else 'differs'}", flush=True)


if __name__ == "__main__":
    main()
