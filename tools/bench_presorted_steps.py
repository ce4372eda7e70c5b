"""Local steps of the PRESORTED multi-GPU exchange (grs_sort_sharded, u32 keys; grs_codec.hpp)
measured on one MI355X for BASELINE config C4 at N ranks (strong scaling, 2^30 / N keys per
rank).  All N shards are generated and sorted on this one device so that the splitters, bucket
sizes and encoded sizes are the real ones; rank 0's encode and receiver 0's decode + merge are
timed.

python tools/bench_presorted_steps.py [--ranks 8] [--total 2^30] [--reps 10] [--link-gbs 64]
Prints one JSON line per step and an estimate of the step at N ranks:
  local_sort       grs_sort of one shard
  encode           grs_shard_encode of rank 0 (splitters, bounds, block widths, scan, pack)
  decode_merge     grs_shard_decode_merge of receiver 0: decode + ceil(log2 N) 2-way merge
                   rounds (the default), and decode + the one-pass k-way merge (option)
  exchange_words   encoded bytes per key; the busiest link's bytes / link-gbs gives the exchange
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import gpuradixsort_amd as grs  # noqa: E402
from gpuradixsort_amd._lib import lib  # noqa: E402
from gpuradixsort_amd.sharded import shard_decode_merge, shard_encode, shard_sample  # noqa: E402


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
    ap.add_argument("--link-gbs", type=float, default=64.0)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    G, n = a.ranks, a.total // a.ranks
    seed = 0x6A09E667F3BCC908 + 4
    S = int(lib().grs_shard_samples_per_rank(G))
    s = grs.RadixSorter(max(n * 2, a.total // G * 2), key_bits=32)
    shards, sks, sps = [], [], []
    for r in range(G):
        k = torch.empty(n, dtype=torch.uint32, device=dev)
        grs.fill_splitmix(k, seed, first_index=r * n)
        s.sort(k)
        shards.append(k)
        sk, sp = shard_sample(k, n, S)
        sks.append(sk)
        sps.append(sp)
    s.check_error()
    gk, gp = torch.cat(sks), torch.cat(sps)

    src = torch.empty(n, dtype=torch.uint32, device=dev)
    grs.fill_splitmix(src, seed)
    tmp = torch.empty_like(src)

    def sort_once():
        tmp.copy_(src)
        s.sort(tmp)
    copy_ms = timed(lambda: tmp.copy_(src), a.reps)
    ms_sort = timed(sort_once, a.reps) - copy_ms
    print(json.dumps({"step": "local_sort", "n": n, "ms": round(ms_sort, 4)}), flush=True)

    sends, sizes = [], []
    for r in range(G):
        send, sz = shard_encode(s, shards[r], n, gk, gp, G, r)
        sends.append(send)
        sizes.append(sz.cpu().numpy().astype(np.int64))
    mat = np.stack(sizes)
    ms_enc = timed(lambda: shard_encode(s, shards[0], n, gk, gp, G, 0), a.reps)
    words = mat[:, 1::2]
    keys = mat[:, 0::2]
    print(json.dumps({"step": "encode", "n": n, "ms": round(ms_enc, 4),
                      "bytes_per_key": round(4 * words.sum() / keys.sum(), 3)}), flush=True)

    parts, offs, lens, off = [], [], [], 0
    for p in range(G):
        start = int(words[p, :0].sum())
        w = int(words[p, 0])
        parts.append(sends[p][start:start + w])
        offs.append(off)
        lens.append(int(keys[p, 0]))
        off += w
    recv = torch.cat(parts)
    m = sum(lens)
    out = torch.empty(m, dtype=torch.uint32, device=dev)
    ms_modes = {}
    for mode in ("rounds", "kway"):   # the receive side's two merges (GRS_OPT_MERGE)
        s.set_option("merge", mode)
        ms_modes[mode] = timed(lambda: shard_decode_merge(s, recv, offs, lens, out), a.reps)
        s.check_error()
        o64 = out.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        ok = bool(torch.all(o64[1:] >= o64[:-1]).item())
        print(json.dumps({"step": "decode_merge", "merge": mode, "n": m, "ms": round(ms_modes[mode], 4),
                          "sorted": ok}), flush=True)
    ms_dm = ms_modes["rounds"]
    s.set_option("merge", "rounds")

    # busiest link: the largest off-diagonal bucket (one xGMI link per rank pair)
    off_diag = [int(words[p, q]) for p in range(G) for q in range(G) if p != q]
    link_bytes = 4 * max(off_diag) if off_diag else 0
    ms_x = link_bytes / (a.link_gbs * 1e9) * 1e3
    step = ms_sort + ms_enc + ms_x + ms_dm
    print(json.dumps({"step": "estimate", "ranks": G, "link_GBps": a.link_gbs,
                      "exchange_ms": round(ms_x, 4), "step_ms_without_sync": round(step, 4),
                      "Gkeys_per_s": round(a.total / step / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
