"""Round-5 lab driver (tools/lab5.hip): the MSD-first pieces, timed in one process.

python tools/lab5.py [--n N] [--rounds R] [--p3 block:items:c16,...]
Prints median ms and the fraction of 8 TB/s each piece's algorithmic bytes reach; checks each
piece's output against torch.
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
    ap.add_argument("--n", type=int, default=1 << 28)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--p3", default="256:20:0,256:20:1,512:10:0,256:24:0")
    ap.add_argument("--h2chunk", default="65536,262144")
    a = ap.parse_args()
    L = ctypes.CDLL(os.path.join(HERE, "liblab5.so"))
    vp = ctypes.c_void_p
    P = lambda t: vp(t.data_ptr())  # noqa: E731
    n = a.n
    dev = torch.device("cuda", 0)
    sp = vp(torch.cuda.current_stream().cuda_stream)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    keys = torch.empty(n, dtype=torch.uint32, device=dev)
    grs.fill_splitmix(keys, 0x6A09E667F3BCC908 + 4)
    k64 = keys.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn, pre=None):
        ts = []
        for _ in range(a.rounds):
            if pre:
                pre()
            torch.cuda.synchronize()
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts), min(ts)

    def line(name, med, mn, nbytes):
        print(f"{name:36s} median {med:8.4f} ms  min {mn:8.4f}  {nbytes / med / 1e6:8.1f} GB/s "
              f"({nbytes / med / 8e9:.3f} of 8 TB/s)", flush=True)

    out = torch.empty_like(keys)
    for grid in (2048, 4096, 8192):
        med, mn = timed(lambda: L.lab5_copy(P(keys), P(out), n, grid, sp))
        line(f"copy grid={grid}", med, mn, n * 8)

    hist = torch.zeros(16 * 256, dtype=torch.uint32, device=dev)
    for qn in (4, 1):
        med, mn = timed(lambda: L.lab5_h1(P(keys), n, P(hist), cus, qn, sp), lambda: hist.zero_())
        line(f"hist {qn} digit(s) (lab5_h1)", med, mn, n * 4)
    ref = torch.bincount(k64 >> 24, minlength=256)
    print("   top-byte histogram", "OK" if torch.equal(hist[:256].to(torch.int64), ref) else "WRONG", flush=True)

    # P1's output: stable by top byte
    p1 = keys.view(torch.int32)[torch.sort(k64 >> 24, stable=True)[1]].view(torch.uint32).contiguous()
    h2 = torch.zeros(65536, dtype=torch.uint32, device=dev)
    ref2 = torch.bincount(k64 >> 16, minlength=65536)
    for ch in (int(x) for x in a.h2chunk.split(",")):
        for blk in (512, 1024):
            med, mn = timed(lambda: L.lab5_h2(P(p1), n, ch, P(h2), blk, sp), lambda: h2.zero_())
            ok = torch.equal(h2.to(torch.int64), ref2)
            line(f"h2 chunk={ch} block={blk}", med, mn, n * 4)
            print("   per-bucket byte-2 histogram", "OK" if ok else "WRONG", flush=True)
    del p1

    # P2's output: stable by the top 16 bits; segments = the 65536 prefixes
    p64 = k64 >> 16
    p2 = keys.view(torch.int32)[torch.sort(p64, stable=True)[1]].view(torch.uint32).contiguous()
    off = torch.zeros(65537, dtype=torch.int64, device=dev)
    off[1:] = torch.cumsum(ref2, 0)
    off32 = off.to(torch.int32).view(torch.uint32).contiguous()
    print(f"segments: mean {n / 65536:.0f}, max {int(ref2.max())}", flush=True)
    expect = torch.sort(k64)[0]
    err = torch.zeros(4, dtype=torch.uint32, device=dev)
    for spec in a.p3.split(","):
        b, it, c16 = (int(x) for x in spec.split(":"))
        if b * it < int(ref2.max()):
            print(f"p3 {spec}: segment too long for {b * it}", flush=True)
            continue
        out.zero_()
        err.zero_()
        rc = L.lab5_p3(b, it, c16, P(p2), P(out), P(off32), 65536, P(err), sp)
        assert rc == 0, (spec, rc)
        torch.cuda.synchronize()
        ok = torch.equal(out.view(torch.int32).to(torch.int64) & 0xFFFFFFFF, expect)
        med, mn = timed(lambda: L.lab5_p3(b, it, c16, P(p2), P(out), P(off32), 65536, P(err), sp))
        line(f"p3 {spec}", med, mn, n * 8)
        print(f"   sorted: {'OK' if ok else 'WRONG'} err={int(err[0])}", flush=True)


if __name__ == "__main__":
    main()
