"""Local steps of the multi-GPU sort (grs_sort_sharded) measured on one MI355X, for the
DESIGN.md §6 scaling estimate of BASELINE config C4 at N ranks (strong scaling, 2^30 / N keys
per rank).

python tools/bench_sharded_steps.py [--ranks 8] [--reps 10]
Prints one JSON line per step:
  partition      grs_partition_ranges of one rank's shard into N buckets with tie-breaking
  partition_regions  the same into the exchange's region send buffer (grs_partition_regions:
                 no bucket histogram; what grs_sort_sharded runs)
                 splitters (the splitters of rank 0, from the host twin over all ranks' samples)
  local_sort     grs_sort of the received run (2^30 / N keys), full-range keys and (the
                 realistic case) keys of one of the N key ranges
  sharded_world1 grs_sort_sharded on a one-rank RCCL communicator (samples, device splitters,
                 partition into one bucket, count all-gather, the one host sync, the self copy,
                 local sort): its difference to local_sort is the fixed orchestration cost
"""
import argparse
import ctypes
import json
import os
import socket
import statistics
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import gpuradixsort_amd as grs  # noqa: E402
from gpuradixsort_amd._lib import check, lib  # noqa: E402


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
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--total", type=int, default=1 << 30)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--chunks", type=int, default=4, help="chunks of the chunked exchange")
    ap.add_argument("--link-gbs", type=float, default=64.0, help="xGMI GB/s per direction per link")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = lib()
    G, n = a.ranks, a.total // a.ranks
    seed = 0x6A09E667F3BCC908 + 4
    S = L.grs_shard_samples_per_rank(G)
    shard = torch.empty(n, dtype=torch.uint32, device=dev)
    pos = (torch.arange(S, dtype=torch.int64) * n) // S
    ak, ap_ = [], []
    for r in range(G):
        grs.fill_splitmix(shard, seed, first_index=r * n)
        ak.append(shard.index_select(0, pos.to(dev)).cpu().numpy())
        ap_.append(pos.numpy().astype(np.uint32))
    ak, ap_ = np.concatenate(ak), np.ascontiguousarray(np.concatenate(ap_))
    order = np.lexsort((np.arange(G * S), ak))
    sk = np.ascontiguousarray(ak[order])
    sj = np.ascontiguousarray(order.astype(np.uint32))
    spl = np.zeros(max(G - 1, 1), np.uint32)
    th = np.zeros(max(G - 1, 1), np.uint32)
    check(L.grs_shard_splitters_host(sk.ctypes.data, sj.ctypes.data, ap_.ctypes.data, 4, G, S, 0,
                                     spl.ctypes.data, th.ctypes.data), "splitters")
    grs.fill_splitmix(shard, seed, first_index=0)
    s = grs.RadixSorter(n, key_bits=32)
    out = torch.empty_like(shard)
    cnt = torch.zeros(16, dtype=torch.uint32, device=dev)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def part():
        check(L.grs_partition_ranges(s._h, ctypes.c_void_p(shard.data_ptr()), None,
                                     ctypes.c_void_p(out.data_ptr()), None, n, spl.ctypes.data,
                                     th.ctypes.data, G - 1, ctypes.c_void_p(cnt.data_ptr()), sp),
              "partition")
    ms = timed(part, a.reps)
    s.check_error()
    print(json.dumps({"step": "partition", "ranks": G, "n_local": n, "ms": round(ms, 4),
                      "GB/s": round(n * 8 / ms / 1e6, 1)}), flush=True)
    # what grs_sort_sharded runs: the region send buffer (no bucket histogram), the region being
    # the even share + 25 % + 64K items
    region = min(n, n * 5 // 4 // G + 65536)
    xout = torch.empty((G - 1) * region + n, dtype=shard.dtype, device=dev)

    def part_regions():
        check(L.grs_partition_regions(s._h, ctypes.c_void_p(shard.data_ptr()), None,
                                      ctypes.c_void_p(xout.data_ptr()), None, n, spl.ctypes.data,
                                      th.ctypes.data, G - 1, region, ctypes.c_void_p(cnt.data_ptr()), sp),
              "partition_regions")
    ms = timed(part_regions, a.reps)
    ms_part_regions = ms
    s.check_error()
    print(json.dumps({"step": "partition_regions", "ranks": G, "n_local": n, "ms": round(ms, 4),
                      "GB/s": round(n * 8 / ms / 1e6, 1)}), flush=True)
    del xout

    bufs = [torch.empty_like(shard) for _ in range(a.reps + 1)]
    for b in bufs:
        grs.fill_splitmix(b, seed)
    it = iter(bufs)
    ms = timed(lambda: s.sort(next(it)), a.reps)
    ms_sort = ms
    s.check_error()
    print(json.dumps({"step": "local_sort", "n": n, "ms": round(ms, 4),
                      "Gkeys/s": round(n / ms / 1e6, 2)}), flush=True)
    # what a rank really receives: the keys of one of G key ranges (uniform keys: the top
    # log2(G) bits fixed), i.e. a narrower key for the local sort's MSD schedule
    lg = max(0, G.bit_length() - 1)
    for b in bufs:
        grs.fill_splitmix(b, seed)
        if lg:
            b.view(torch.int32).bitwise_and_((1 << (32 - lg)) - 1)
    it = iter(bufs)
    ms = timed(lambda: s.sort(next(it)), a.reps)
    ms_sort_range = ms
    s.check_error()
    print(json.dumps({"step": "local_sort_one_range", "n": n, "key_range_bits": 32 - lg,
                      "ms": round(ms, 4), "Gkeys/s": round(n / ms / 1e6, 2)}), flush=True)
    del bufs

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    from gpuradixsort_amd.sharded import ShardedSorter

    world1 = {}
    for name, opts in [("sharded_world1", {}),
                       ("sharded_world1_partition", {"sharded_path": "general", "exchange": "partition"}),
                       ("sharded_world1_chunked", {"sharded_path": "general", "exchange": "chunked",
                                                   "x_chunks": a.chunks})]:
        sh = ShardedSorter(n, key_bits=32, device=dev, options=opts)
        bufs = [torch.empty_like(shard) for _ in range(a.reps + 1)]
        for b in bufs:
            grs.fill_splitmix(b, seed)
        it = iter(bufs)
        ms = timed(lambda: sh.sort(next(it), check_error=False), a.reps)
        sh.sorter.check_error()
        assert sh.count_inversions() == 0
        line = {"step": name, "n": n, "ms": round(ms, 4), "Gkeys/s": round(n / ms / 1e6, 2)}
        if opts:
            sh.set_profiling(2)
            grs.fill_splitmix(bufs[0], seed)
            sh.sort(bufs[0])
            line["phases_ms"] = {k: round(v, 4) for k, v in sh.exchange_timing().items()
                                 if k.endswith("_ms")}
        world1[name] = ms
        if opts:
            world1[name + "_before"] = line["phases_ms"]["before_ms"]
        print(json.dumps(line), flush=True)
        sh.close()
        del bufs
    dist.destroy_process_group()

    # one chunk's partition, and the step's critical path at G ranks from the measured parts:
    # the exchange moves n / G keys over each of the G - 1 links (one link per peer)
    cn = (n + a.chunks - 1) // a.chunks
    ms_chunk = timed(lambda: check(L.grs_partition_ranges(
        s._h, ctypes.c_void_p(shard.data_ptr()), None, ctypes.c_void_p(out.data_ptr()), None, cn,
        spl.ctypes.data, th.ctypes.data, G - 1, ctypes.c_void_p(cnt.data_ptr()), sp), "partition"), a.reps)
    link_ms = (n / G) * 4 / (a.link_gbs * 1e9) * 1e3
    # fixed orchestration (samples, splitters, the count all-gather, the host sync): the one-rank
    # partition-first run's phase before its exchange less its partition (its exchange phase is
    # the self copy of the whole shard, 1/G of it at G ranks, overlapping the links); the
    # chunked run's extra per chunk on top of that
    fixed = max(0.0, world1["sharded_world1_partition_before"] - ms_part_regions)
    per_chunk = max(0.0, (world1["sharded_world1_chunked"] - world1["sharded_world1_partition"]) / a.chunks)
    pf = ms_part_regions + link_ms + ms_sort_range + fixed
    ch = ms_chunk + max((a.chunks - 1) * ms_chunk, link_ms + a.chunks * per_chunk) + ms_sort_range + fixed
    print(json.dumps({"step": "projection", "ranks": G, "n_local": n, "chunks": a.chunks,
                      "link_GBps": a.link_gbs, "link_ms": round(link_ms, 4),
                      "partition_chunk_ms": round(ms_chunk, 4), "fixed_ms": round(fixed, 4),
                      "chunk_overhead_ms": round(per_chunk, 4),
                      "step_partition_first_ms": round(pf, 4), "step_chunked_ms": round(ch, 4),
                      "speedup_vs_1gpu_partition_first": round(G * ms_sort / pf, 2),
                      "speedup_vs_1gpu_chunked": round(G * ms_sort / ch, 2),
                      "note": "unmeasured across GPUs: one-GPU parts plus link arithmetic"}), flush=True)


if __name__ == "__main__":
    main()
