"""Kernel laboratory: interleaved timing of onesweep-pass variants (tools/lab.hip).

python tools/lab.py [--n N] [--rounds R] [--variants 16:0,16:1,...]
Prints one line per variant: median / min ms and algorithmic GB/s (8 B per key per pass).
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
    ap.add_argument("--lib", default="liblab.so")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--variants", default="256:16:0,256:16:4,256:16:1,256:16:2,256:16:3,256:16:7,"
                    "256:24:0,256:32:0,256:32:4,256:32:1,256:32:2,256:32:3,512:8:0,512:12:0,"
                    "512:16:0,512:16:4,512:16:1,512:16:3,1024:8:0,1024:16:0")
    a = ap.parse_args()
    L = ctypes.CDLL(os.path.join(HERE, a.lib))
    vp = ctypes.c_void_p
    n = a.n
    dev = torch.device("cuda", 0)
    keys = torch.empty(n, dtype=torch.uint32, device=dev)
    grs.fill_splitmix(keys, 0x6A09E667F3BCC908 + 4)
    out = torch.empty_like(keys)
    hist = torch.zeros(4 * 256, dtype=torch.uint32, device=dev)
    ticket = torch.zeros(4, dtype=torch.uint32, device=dev)
    err = torch.zeros(4, dtype=torch.uint32, device=dev)
    max_tiles = (n + 1023) // 1024
    st = torch.zeros(max_tiles * 256, dtype=torch.uint32, device=dev)
    st2 = torch.zeros_like(st)
    s = torch.cuda.current_stream()
    sp = vp(s.cuda_stream)
    P = lambda t: vp(t.data_ptr())  # noqa: E731
    assert L.lab_hist(P(keys), ctypes.c_uint32(n), P(hist), P(st), ctypes.c_uint32(0), sp) == 0
    torch.cuda.synchronize()

    variants = []
    for v in a.variants.split(","):
        parts = v.split(":")
        b, it, dbg = parts[:3]
        grid = int(parts[3]) if len(parts) > 3 else 0   # persistent grid (0 = one tile per WG)
        variants.append((int(b), int(it), int(dbg), grid))
    times = {v: [] for v in variants}
    copy_t = {0: [], 1: []}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        for v in variants:
            st.zero_()
            ticket.zero_()
            L.lab_set_persistent(v[3])
            e0.record()
            rc = L.lab_pass(v[0] * 10000 + v[1] * 16 + v[2], P(keys), P(out), ctypes.c_uint32(n), P(hist), P(ticket),
                            P(st), P(st2), P(err), 0, sp)
            e1.record()
            assert rc == 0, (v, rc)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
        for w in (0, 1):
            e0.record()
            L.lab_copy(w, P(keys), P(out), ctypes.c_uint32(n), sp)
            e1.record()
            torch.cuda.synchronize()
            copy_t[w].append(e0.elapsed_time(e1))
    alg = n * 8
    print(f"n={n}  error word={int(err[0].item())}")
    for w in (0, 1):
        med = statistics.median(copy_t[w])
        print(f"copy {'x4   ' if w else 'dword'}          median {med:8.4f} ms  {alg / med / 1e6:8.1f} GB/s")
    for v in variants:
        med, mn = statistics.median(times[v]), min(times[v])
        print(f"block={v[0]:4d} items={v[1]:2d} dbg={v[2]} grid={v[3]:4d}  median {med:8.4f} ms  min {mn:8.4f}  {alg / med / 1e6:8.1f} GB/s")


if __name__ == "__main__":
    main()
