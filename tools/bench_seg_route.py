"""grs_sort_segmented's two routes for segments past LDS size: the segmented passes
(a workgroup per segment at least: a segment shorter than a tile is a solo tile) against one
composite (segment, key) sort, on many short segments beside one long one.
python tools/bench_seg_route.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpuradixsort_amd as grs  # noqa: E402


def offsets(short_len, n_short, long_len, dev):
    lens = torch.full((n_short + 1,), short_len, dtype=torch.int64)
    lens[n_short // 2] = long_len   # the long segment in the middle
    off = torch.zeros(n_short + 2, dtype=torch.int64)
    off[1:] = torch.cumsum(lens, 0)
    return off.to(torch.int32).to(dev), int(off[-1])


def main():
    dev = torch.device("cuda", 0)
    cases = [(4, 1 << 20, 1 << 24), (64, 1 << 18, 1 << 24), (256, 1 << 16, 1 << 24), (1024, 1 << 14, 1 << 24),
             (2048, 1 << 13, 1 << 24), (4096, 1 << 12, 1 << 24), (20000, 1 << 10, 1 << 24)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for short_len, n_short, long_len in cases:
        off, n = offsets(short_len, n_short, long_len, dev)
        keys0 = torch.empty(n, dtype=torch.uint32, device=dev)
        grs.fill_splitmix(keys0, 5)
        s = grs.RadixSorter(n, key_bits=32, pairs=True)
        res = {}
        outs = {}
        for route in ("passes", "composite"):
            s.set_option("seg_route", route)
            ts = []
            for _ in range(5):
                k = keys0.clone()
                v = torch.arange(n, dtype=torch.int32, device=dev).view(torch.uint32)
                torch.cuda.synchronize()
                e0.record()
                s.sort_segmented(k, off, v)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            s.check_error()
            res[route] = statistics.median(ts)
            outs[route] = (k, v)
        same = torch.equal(outs["passes"][0], outs["composite"][0]) and torch.equal(outs["passes"][1], outs["composite"][1])
        print(f"{n_short} x {short_len} + 1 x {long_len} keys (n {n}): passes {res['passes']:.3f} ms, "
              f"composite {res['composite']:.3f} ms, same output {same}", flush=True)
        s.close()


if __name__ == "__main__":
    main()
