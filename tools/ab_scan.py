"""A/B of the device-wide exclusive scan: the library's grs_exclusive_scan_u32 against the
single-pass decoupled look-back kernel (grs_scan_onepass<rows>) built into tools/liblab2.so, same process,
interleaved; both checked against torch's cumsum (mod 2^32).

python tools/ab_scan.py [--n N] [--reps R]
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
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = grs.lib()
    lab = ctypes.CDLL(os.path.join(HERE, "liblab2.so"))
    vp = ctypes.c_void_p
    sp = vp(torch.cuda.current_stream().cuda_stream)
    for n in sorted({a.n, (1 << 24) + 5, 1 << 20, 100_003}):
        x = torch.empty(n, dtype=torch.int32, device=dev)
        grs.fill_splitmix(x, 3)
        want = torch.cumsum(x.to(torch.int64) & 0xFFFFFFFF, 0)
        want = ((want - (x.to(torch.int64) & 0xFFFFFFFF)) & 0xFFFFFFFF)
        y = torch.empty_like(x)
        tot = torch.zeros(1, dtype=torch.int32, device=dev)
        scratch = torch.empty((L.grs_scan_scratch_bytes(n) + 3) // 4, dtype=torch.int32, device=dev)
        ctl = torch.empty(4 + 2 * (n // 8192 + 2), dtype=torch.int32, device=dev)

        def lib_scan():
            assert L.grs_exclusive_scan_u32(vp(x.data_ptr()), vp(y.data_ptr()), n, vp(tot.data_ptr()),
                                            vp(scratch.data_ptr()), scratch.numel() * 4, sp) == 0

        def one_pass2(rows):
            def f():
                assert lab.lab2_scan2(rows, vp(x.data_ptr()), vp(y.data_ptr()), ctypes.c_uint32(n),
                                      vp(ctl.data_ptr()), vp(tot.data_ptr()), sp) == 0
            return f

        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        res = {}
        for name, fn in (("reduce-then-scan (library)", lib_scan), ("wave rows x8", one_pass2(8)), ("wave rows x16", one_pass2(16)),
                         ("wave rows x32", one_pass2(32))):
            y.zero_()
            fn()
            torch.cuda.synchronize()
            ok = torch.equal(y.to(torch.int64) & 0xFFFFFFFF, want)
            okt = (int(tot.item()) & 0xFFFFFFFF) == (int(want[-1].item()) + (int(x[-1].item()) & 0xFFFFFFFF)) & 0xFFFFFFFF
            res[name] = [ok and okt, []]
        for _ in range(a.reps):
            for name, fn in (("reduce-then-scan (library)", lib_scan), ("wave rows x8", one_pass2(8)), ("wave rows x16", one_pass2(16)),
                         ("wave rows x32", one_pass2(32))):
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                res[name][1].append(e0.elapsed_time(e1))
        err = int(ctl[0].item())
        for name, (ok, ts) in res.items():
            med = statistics.median(ts)
            print(f"n={n:>10d} {name:28s} median {med:8.4f} ms  min {min(ts):8.4f}  "
                  f"{n * 8 / med / 1e6:8.1f} GB/s ({n * 8 / med / 8e9:.3f} of 8 TB/s)  "
                  f"{'exact' if ok else 'WRONG'}{'' if err == 0 else '  error word set'}", flush=True)


if __name__ == "__main__":
    main()
