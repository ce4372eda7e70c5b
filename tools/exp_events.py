"""Whole-sort time with and without libgrs's per-phase hipEvent ring (grs_set_profiling), and
with the same sorts under a kernel trace: do the events between launches cost time?

python tools/exp_events.py [--configs c2,ns,c4] [--steps 20]"""
import argparse
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import gpuradixsort_amd as grs  # noqa: E402

CFG = {"c2": (1 << 24, 4), "ns": (1 << 28, 8), "c4": (1 << 30, 8)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,ns,c4")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for c in a.configs.split(","):
        n, rb = CFG[c]
        pool = [torch.empty(n, dtype=torch.uint32, device=dev) for _ in range(2)]
        for i, k in enumerate(pool):
            grs.fill_splitmix(k, 99, first_index=i * n)
        s = grs.RadixSorter(n, key_bits=32, radix_bits=rb)
        res = {}
        for mode in ("events", "plain", "events", "plain"):
            s.set_profiling(a.steps if mode == "events" else 0)
            for i in range(3):
                s.sort(pool[i % 2])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                grs.fill_splitmix(pool[i % 2], 7, first_index=i * n) if False else None
                s.sort(pool[i % 2])
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.steps
            res.setdefault(mode, []).append(ms)
        s.check_error()
        print(f"{c}: n={n} rb={rb}  ms/sort with per-phase events {res['events']}  without {res['plain']}  "
              f"Gkeys/s {n / min(res['events']) / 1e6:.1f} vs {n / min(res['plain']) / 1e6:.1f}", flush=True)
        s.close()
        del pool
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
