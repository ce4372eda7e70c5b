"""Driver of tools/lab7.hip: the LDS segment sort of the MSD schedule (P3) with 0 / 1 / 2 rounds.
Input: 2^28 (or --n) u32 keys already grouped by their top 16 bits into equal segments (P3's
input after the two scatters); output checked against a sort for 2 rounds.
python tools/lab7.py [--n N] [--shapes 256:20:0,768:24:1]"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import gpuradixsort_amd as grs  # noqa: E402

L = ctypes.CDLL(os.path.join(HERE, "liblab7.so"))
vp = ctypes.c_void_p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 28)
    ap.add_argument("--shapes", default="256:20:0,768:24:1")
    ap.add_argument("--pshapes", default="", help="persistent pipelined: block:items:c16:per_cu,...")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, nseg = a.n, 65536
    seg = n // nseg
    low = torch.empty(n, dtype=torch.int32, device=dev)
    grs.fill_splitmix(low, 9)
    keys = ((torch.arange(n, device=dev, dtype=torch.int64) // seg) << 16) | (low.to(torch.int64) & 0xFFFF)
    keys = keys.to(torch.int64).to(torch.int32)   # wraps to the u32 bit pattern
    off = torch.arange(0, n + 1, seg, dtype=torch.int32, device=dev)
    want = torch.sort(keys.to(torch.int64) & 0xFFFFFFFF)[0]
    out = torch.empty_like(keys)
    stream = vp(torch.cuda.current_stream().cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for spec in a.pshapes.split(",") if a.pshapes else []:
        b, it, c16, per_cu = (int(x) for x in spec.split(":"))
        if b * it < seg:
            continue
        ts = []
        for _ in range(7):
            out.zero_()
            e0.record()
            rc = L.lab7_p3p(b, it, c16, per_cu, cus, vp(keys.data_ptr()), vp(out.data_ptr()), vp(off.data_ptr()),
                            nseg, stream)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, (spec, rc)
            ts.append(e0.elapsed_time(e1))
        ms = statistics.median(ts)
        ok = bool(torch.equal(out.to(torch.int64) & 0xFFFFFFFF, want))
        print(f"p3 persistent {spec}: {ms * 1e3:8.1f} us  {n * 8 / ms / 1e6:7.1f} GB/s "
              f"({n * 8 / ms / 1e6 / 8000:.3f} of 8 TB/s) sorted={ok}", flush=True)
    for spec in a.shapes.split(","):
        b, it, c16 = (int(x) for x in spec.split(":"))
        if b * it < seg:
            print(f"{spec}: segment of {seg} too long", flush=True)
            continue
        for rounds in (0, 1, 2):
            ts = []
            for _ in range(7):
                e0.record()
                rc = L.lab7_p3(b, it, c16, rounds, vp(keys.data_ptr()), vp(out.data_ptr()), vp(off.data_ptr()),
                               nseg, stream)
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0, rc
                ts.append(e0.elapsed_time(e1))
            ms = statistics.median(ts)
            ok = ""
            if rounds == 2:
                ok = f" sorted={bool(torch.equal(out.to(torch.int64) & 0xFFFFFFFF, want))}"
            print(f"p3 {spec} rounds={rounds}: {ms * 1e3:8.1f} us  {n * 8 / ms / 1e6:7.1f} GB/s "
                  f"({n * 8 / ms / 1e6 / 8000:.3f} of 8 TB/s){ok}", flush=True)


if __name__ == "__main__":
    main()
