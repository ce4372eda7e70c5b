"""bench.py — Gkeys/s of the MI355X radix sort (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c2|c3|c5|ns] [--dist uniform|perm]
  (N > 1: torchrun --nproc-per-node N ... bench.py --gpus N ...; one rank per GPU, RCCL)

A step = one complete sort of one batch of synthetic keys already resident in HBM
(key[i] = splitmix64(seed ^ global_i)).  Every step sorts its OWN unsorted
buffer (generated before the timed region), so nothing is restored or skipped inside it.

Default workload: BASELINE config C4 itself, 2^30 uniform uint32 keys in total, 8-bit digits
(from 48M keys the MSD-first schedule: two stable scatters by the keys' top two varying bytes,
then every 16-bit segment sorted in LDS; below, and for 4-bit digits, the LSD passes),
STRONG scaling: at N = 1 one MI355X sorts all 2^30 keys in one call; at N > 1 rank r holds
2^30 / N keys and the sort is grs_sort_sharded (gpuradixsort_amd/sharded.py): up to 4 ranks
the presorted exchange (local sort, bit-packed delta encoding of the buckets, one RCCL send /
recv per peer over xGMI, decode, merge), beyond that the partition-first one (range partition,
one RCCL all-to-all, local sort).  `value` = 2^30 keys x steps / wall time.

At N = 1 the default line also carries `north_star` (2^28 uniform u32 keys, BASELINE's
north-star target) and `reference_input` (the reference's own input, 0..N-1 shuffled,
main.cpp:119-125, at 2^28 and 2^30: the MSD digits adapt to its 28 / 30-bit span).

Rank 0 prints ONE JSON line with the driver contract plus:
  roofline      dominant kernel (the LSD schedule's pass: grs_onesweep_v4, or v6 on small
                grids; the MSD schedule's slowest of its two scatters and its LDS sort, each of
                which reads and writes every key once): algorithmic bytes per launch
                (n_local x 2 x (key + value bytes)) / its mean duration from
                hipEvents recorded on the sort's stream during the timed steps; `traffic` is
                the HBM bytes per launch that rocprofv3's FETCH_SIZE / WRITE_SIZE counters
                measure in two child runs of this script (--pmc-probe: one sort of the same
                workload + a known-byte calibration copy with the pass's access width, which
                gives the counters' correction factors), after the timed region (rank 0, N = 1;
                --no-traffic skips them, null on any failure)
  moved_roofline  the bytes the schedule that ran actually moves per step (LSD: a histogram
                read + 2 x per pass; MSD: 3 read+write sweeps + H2's sampled read), over the step
                time, next to `sort_roofline`'s credited SURVEY §8d bytes (key bits / digit bits
                passes, whatever schedule ran: an MSD sort can exceed 1 there)
  cpu_baseline  the oracle's host std::sort on a bounded sample (rank 0, N = 1 only)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "Gkeys/s (uint32) at 1/2/4/8 MI355X; achieved HBM GB/s vs peak"
HBM_PEAK_GBPS = 8000.0     # MI355X_MICROARCH.md chip table (spec)

CONFIGS = {
    # name: (config_id, total keys (c4: strong scaling) or keys per GPU, key_bits, pairs,
    #        radix_bits, description)
    "c4": (4, 1 << 30, 32, False, 8, "C4: 2^30 uint32 keys in total (strong scaling: 2^30 / N per "
                                     "GPU), 8-bit digits (MSD schedule at N = 1); N > 1: one RCCL "
                                     "exchange over xGMI (config.exchange)"),
    "c2": (2, 1 << 24, 32, False, 4, "C2: 16M uint32 keys, 4-bit-digit LSD"),
    "c3": (3, 1 << 28, 32, True, 8, "C3: 256M uint32 key + uint32 payload, stable, 8-bit digits "
                                    "(MSD schedule)"),
    "c5": (5, 1 << 28, 64, False, 8, "C5: 256M uint64 keys, 8-bit digits (MSD schedule: 2 scatters + "
                                     "LDS rounds; 8 passes credited)"),
    # BASELINE.json north_star's own 1-GPU target: >= 60 % of the HBM roofline on 256 M
    # uniform-random uint32 keys (keys only)
    "ns": (6, 1 << 28, 32, False, 8, "north star: 256M uniform uint32 keys, keys only, 8-bit digits "
                                     "(MSD schedule)"),
}
DISTS = ("uniform", "perm")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--dist", default="uniform", choices=DISTS,
                    help="uniform: splitmix64 keys; perm: the reference's input, 0..N-1 shuffled "
                         "(main.cpp:119-125; grs_fill_permutation)")
    ap.add_argument("--no-reference-input", action="store_true",
                    help="skip the reference-input legs (0..N-1 shuffled at 2^28 and 2^30)")
    ap.add_argument("--n", type=int, default=0, help="override the total (c4) / per-GPU key count")
    ap.add_argument("--traffic-json", default="", help="tools/bench_pmc.py output of this workload")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC child runs")
    ap.add_argument("--pmc-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-north-star", action="store_true",
                    help="skip the second leg (north star: 2^28 u32 keys) after the c4 headline")
    ap.add_argument("--cpu-sample", type=int, default=1 << 26)
    ap.add_argument("--sharded", action="store_true",
                    help="N = 1 through grs_sort_sharded's multi-rank code path (option "
                         "sharded_path=general, a one-rank RCCL communicator): a one-GPU "
                         "rehearsal of N > 1")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="sorter option (grs_set_option, gpuradixsort_amd._lib.OPTIONS) for A/B "
                         "runs; repeatable")
    ap.add_argument("--pool-gib", type=float, default=160.0,
                    help="HBM budget for the distinct per-step input buffers (the default holds "
                         "warmup + steps C4 inputs of 4 GiB at the default 3 + 20 and 5 + 20)")
    return ap.parse_args()


def usable_cores():
    """(threads to use, what the host reports): the affinity mask's CPUs, capped by the
    cgroup v2 CPU quota (cpu.max) when one is set."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    cores = max(1, min(aff, quota) if quota else aff)
    return cores, {"os_cpu_count": os.cpu_count(), "affinity_cpus": aff, "cgroup_quota_cpus": quota,
                   "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(n_sample: int, key_bits: int, pairs: bool, seed: int) -> dict:
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np

    import oracle

    keys = oracle.splitmix_keys(n_sample, key_bits, seed)
    t = time.perf_counter()
    if pairs:
        vals = np.arange(n_sample, dtype=np.uint32)
        oracle.cpu_stable_sort_pairs(keys, vals, 1)
        what = "std::sort of (key, index) words = stable pair sort"
    else:
        oracle.cpu_sort(keys, 1)
        what = "std::sort"
    dt = time.perf_counter() - t
    out = {"value": round(n_sample / dt / 1e9, 5), "unit": "Gkeys/s", "cores": 1, "kind": "port",
           "sample": f"{n_sample} keys of the same splitmix64 uniform workload, {what}, "
                     f"1 thread, {dt:.2f} s (oracle/cpu_sort.cpp)"}
    # __gnu_parallel::sort on ALL of the host cores this process may use: the
    # CPUs of its affinity mask, capped by the cgroup's CPU quota where one is set (a GPU box
    # shares a larger machine; os.cpu_count() counts the whole machine there)
    cores, host = usable_cores()
    host["hardware_concurrency"] = oracle.hardware_concurrency()
    keys = oracle.splitmix_keys(n_sample, key_bits, seed)
    t = time.perf_counter()
    if pairs:
        oracle.cpu_stable_sort_pairs(keys, np.arange(n_sample, dtype=np.uint32), cores)
    else:
        oracle.cpu_sort(keys, cores)
    dt = time.perf_counter() - t
    out["parallel"] = {"value": round(n_sample / dt / 1e9, 5), "cores": cores,
                       "what": f"__gnu_parallel::sort, {cores} threads, {dt:.2f} s",
                       "host": host}
    return out


CAL_WORDS = 1 << 27   # calibration copy: 512 MiB read + 512 MiB written


def config_seed(cid):
    """SURVEY.md §8(d)'s seed, 0x6A09E667F3BCC908 + config id; the north-star leg (id 6, C3's n
    and key width) also differs in bit 48 so that its keys are not C3's multiset (the same rule
    as oracle.config_seed, restated: bench.py's timed legs do not import the oracle)."""
    s = 0x6A09E667F3BCC908 + cid + ((1 << 48) if cid == 6 else 0)
    return s & ((1 << 64) - 1)


def pmc_probe(a, options):
    """Child run under rocprofv3 --pmc (see measure_traffic): one warm sort, one measured sort
    of the same workload, two calibration copies of known bytes."""
    import gpuradixsort_amd as grs

    cid, n_cfg, kb, pairs, rb, _ = CONFIGS[a.config]
    n = a.n or n_cfg
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    seed = config_seed(cid)
    k = torch.empty(n, dtype=torch.uint32 if kb == 32 else torch.uint64, device=dev)
    v = torch.empty(n, dtype=torch.uint32, device=dev) if pairs else None
    s = grs.RadixSorter(n, key_bits=kb, pairs=pairs, radix_bits=rb, options=options)
    for i in range(2):
        if a.dist == "perm":
            grs.fill_permutation(k, seed + i)
        else:
            grs.fill_splitmix(k, seed, first_index=i * n)
        if pairs:
            grs.iota_u32(v)
        s.sort(k, v)
    src = torch.ones(CAL_WORDS, dtype=torch.int32, device=dev)
    dst = torch.empty_like(src)
    from gpuradixsort_amd._lib import check, lib
    import ctypes
    for _ in range(2):
        check(lib().grs_copy_u32(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                                 CAL_WORDS, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
              "grs_copy_u32")
    torch.cuda.synchronize()
    s.check_error()


def measure_traffic(a, config, options, n_local, kernel="grs_onesweep_v", dist="uniform"):
    """HBM bytes per launch of the roofline kernel (the pass, or the MSD schedule's dominant
    kernel; names match by prefix) from rocprofv3 PMC counters (MI355X_MICROARCH.md, HBM):
    one counter per rocprofv3 run (FETCH_SIZE, then WRITE_SIZE) over a child --pmc-probe run;
    each counter is corrected by known bytes / counter bytes of the calibration copy, which
    issues the pass's own access width (one dword per lane).  Returns (dict, None) or
    (None, reason)."""
    import csv
    import glob
    import shutil
    import signal
    import statistics
    import subprocess
    import tempfile

    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rp):
        return None, "rocprofv3 not found"
    env = dict(os.environ, TMPDIR="/tmp")
    extra = [f"--opt={k}={v}" for k, v in options.items()]
    got = {}
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        chosen = None
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(d, ctr)
            cmd = [rp, "--pmc", ctr, "-d", out, "-o", "p", "--output-format", "csv", "--",
                   sys.executable, os.path.abspath(__file__), "--pmc-probe", "--config", config,
                   "--n", str(n_local), "--dist", dist] + extra
            p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env,
                                 start_new_session=True)
            try:
                _, err = p.communicate(timeout=150)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                return None, f"rocprofv3 --pmc {ctr} timed out"
            if p.returncode != 0:
                return None, f"rocprofv3 --pmc {ctr} rc={p.returncode}: {err.decode()[-300:]}"
            # rows of the roofline kernel by instantiation (its name followed by "<": the MSD
            # schedule launches other instantiations of the same template that usually leave at
            # once, e.g. the gated redo passes): the one reading the most is the roofline kernel
            vals = {"pass": {}, "cal": [], "all": 0.0}
            for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if r["Counter_Name"] != ctr:
                        continue
                    name = r["Kernel_Name"]
                    if (kernel + "<") in name:
                        vals["pass"].setdefault(name, []).append(float(r["Counter_Value"]) * 1024.0)   # KiB -> bytes
                    if "grs_copy_u32" in name:
                        vals["cal"].append(float(r["Counter_Value"]) * 1024.0)
                    elif not any(x in name for x in ("grs_fill_", "grs_iota_u32")):
                        vals["all"] += float(r["Counter_Value"]) * 1024.0   # every kernel of the 2 sorts
            if not vals["pass"] or not vals["cal"]:
                return None, f"no {ctr} rows for the pass or the calibration copy"
            if chosen is None:
                chosen = max(vals["pass"], key=lambda nm: statistics.mean(vals["pass"][nm]))
            rows = vals["pass"].get(chosen)
            if not rows:
                return None, f"no {ctr} rows for {chosen[:80]}"
            got[ctr] = (statistics.mean(rows), statistics.mean(vals["cal"]), len(rows), vals["all"] / 2)
    known = CAL_WORDS * 4
    fr, fw = known / got["FETCH_SIZE"][1], known / got["WRITE_SIZE"][1]
    rd, wr = fr * got["FETCH_SIZE"][0], fw * got["WRITE_SIZE"][0]
    sort_bytes = fr * got["FETCH_SIZE"][3] + fw * got["WRITE_SIZE"][3]
    return {"bytes_per_launch": round(rd + wr), "read_bytes": round(rd), "write_bytes": round(wr),
            "sort_bytes": round(sort_bytes),
            "read_factor": round(fr, 4), "write_factor": round(fw, 4),
            "launches": got["FETCH_SIZE"][2], "instantiation": chosen[:160],
            "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one counter per run, over "
                      "bench.py --pmc-probe (2 sorts of this workload) with a grs_copy_u32 "
                      "calibration of known bytes"}, None


def moved_bytes(n, kb, pairs, rb, schedule):
    """HBM bytes the schedule that ran moves per sort of n keys (its algorithmic traffic, rare
    redo / fallback passes excluded): LSD = the histogram read + a read and a write per pass (+ a
    copy-back for an odd pass count); MSD (grs_msd.hpp) = the top digit's scatter, the byte-2
    scatter and the LDS sort each read and write every element once, plus H2's read of a
    1 / 2^k sample of the keys (k as run_msd picks it) and the 4-MB sample."""
    e = kb // 8 + (4 if pairs else 0)
    if schedule == "msd":
        k = 0
        while k < 6 and (n >> (k + 1)) >= 65536 * 512:
            k += 1
        return 3 * 2 * n * e + (n * (kb // 8)) // (1 << k) + (4 << 20)
    passes = -(-kb // rb)
    return n * (kb // 8) + passes * 2 * n * e + (2 * n * e if passes % 2 else 0)


def run_config(a, config, world, rank, local, dev, sharded, steps, warmup, dist="uniform",
               traffic=True, cpu=True):
    """One workload of CONFIGS, timed per the driver contract; returns rank 0's JSON dict.
    dist: "uniform" (splitmix64) or "perm" (the reference's shuffled 0..N-1)."""
    import gpuradixsort_amd as grs

    cid, n_cfg, kb, pairs, rb, desc = CONFIGS[config]
    options = dict(o.split("=", 1) for o in a.opt)
    options = {k: (int(v) if v.lstrip("-").isdigit() else v) for k, v in options.items()}
    if sharded and world == 1:
        options.setdefault("sharded_path", "general")
    if a.n and config == a.config:
        n_cfg = a.n
    strong = config == "c4"
    n_local = n_cfg // world if strong else n_cfg
    seed = config_seed(cid)
    kdt = torch.uint32 if kb == 32 else torch.uint64
    step_bytes = n_local * (kb // 8 + (4 if pairs else 0))
    pool = max(1, min(warmup + steps, int(a.pool_gib * 2**30 // step_bytes)))

    # distinct unsorted inputs, one per step (step s uses global indices offset by s * N_total;
    # perm: step s is the seeded permutation seed + s of 0..N_total-1, rank r its slice r)
    n_total = n_local * world

    def fill(k, i):
        if dist == "perm":
            grs.fill_permutation(k, seed + i, total=n_total, first_index=rank * n_local)
        else:
            grs.fill_splitmix(k, seed, first_index=i * n_total + rank * n_local)

    keys_pool, vals_pool = [], []
    for i in range(pool):
        k = torch.empty(n_local, dtype=kdt, device=dev)
        fill(k, i)
        keys_pool.append(k)
        if pairs:
            v = torch.empty(n_local, dtype=torch.uint32, device=dev)
            grs.iota_u32(v, rank * n_local)
            vals_pool.append(v)

    if not sharded:
        sorter = grs.RadixSorter(n_local, key_bits=kb, pairs=pairs, radix_bits=rb, options=options)

        def step(i):
            k = keys_pool[i % pool]
            if i >= pool:   # pool exhausted: regenerate inside the step (counted, honest)
                fill(k, i)
            sorter.sort(k, vals_pool[i % pool] if pairs else None)
    else:
        from gpuradixsort_amd.sharded import ShardedSorter

        sorter = ShardedSorter(n_local, key_bits=kb, pairs=pairs, radix_bits=rb, device=dev,
                               options=options)

        def step(i):
            k = keys_pool[i % pool]
            if i >= pool:
                fill(k, i)
            # the exchange synchronises once per call (the counts); the timeout check of the
            # local sort happens after the timed region (bench.py reads the error word below)
            sorter.sort(k, vals_pool[i % pool] if pairs else None, check_error=False)

    def barrier():
        torch.cuda.synchronize()
        if sharded:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    for i in range(warmup):
        step(i)
    barrier()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        step(i)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # look-back timeouts of the timed steps surface here (error word; raises GrsError)
    (sorter.sorter if sharded else sorter).check_error()
    # correctness of the last timed step (cheap property: sortedness on device)
    last = (warmup + steps - 1) % pool
    inversions = sorter.count_inversions() if sharded else grs.count_inversions(keys_pool[last])

    # per-phase GPU times: the same steps again, untimed, with libgrs's per-phase hipEvent ring
    # on (events between the launches cost 2-5 us each, 13 % of a C2 sort; the timed steps above
    # run without them, as a caller's sorts do)
    nprof = min(steps, pool)
    sorter.set_profiling(nprof)
    barrier()
    for i in range(warmup, warmup + nprof):
        # the timed steps sorted these buffers: fresh unsorted inputs of the same workload
        fill(keys_pool[i % pool], i)
        if pairs:
            grs.iota_u32(vals_pool[i % pool], rank * n_local)
        step(i)
    barrier()
    (sorter.sorter if sharded else sorter).check_error()
    tims = [sorter.timing(k) for k in range(nprof)]
    hist_ms = sum(t["hist_ms"] for t in tims) / len(tims)
    sort_ms = sum(t["total_ms"] for t in tims) / len(tims)
    msd = tims[0].get("kind") == "msd"
    msd_phases = None
    if msd:
        # the MSD schedule (grs_msd.hpp): sample | P1 top-byte scatter into sampled regions,
        # its redo (a run outgrew its region; empty launches otherwise), H2, P2 byte-2 scatter,
        # P3 LDS sort of the 16-bit segments, fallback; each of P1 / P2 / P3 reads and writes
        # every key once, so the dominant one of them is the roofline kernel
        names = ["p1_scatter_top_byte", "p1_redo", "h2_hist_byte2", "p2_scatter_byte2",
                 "p3_local_sort", "fallback"]
        msd_phases = {nm: round(sum(t["pass_ms"][i] for t in tims) / len(tims), 5)
                      for i, nm in enumerate(names)}
        dom = max(("p1_scatter_top_byte", "p2_scatter_byte2", "p3_local_sort"), key=msd_phases.get)
        mean_pass_ms = msd_phases[dom]
    elif tims[0].get("kind") == "fused":
        # every pass in one launch (grs_onesweep_fused): pass_ms[0] is that launch
        mean_pass_ms = sum(t["pass_ms"][0] for t in tims) / len(tims)
    else:
        pass_ms = [p for t in tims for p in t["pass_ms"]]
        mean_pass_ms = sum(pass_ms) / len(pass_ms)
    fused = tims[0].get("kind") == "fused"
    # the exchange grs_sort_sharded took (include/grs.h): presorted = local sort of the shard
    # first, then the encoded exchange and a merge; partition-first = local sort of the received
    # run.  Its phases of the last step, with the xGMI bytes and rate of this rank
    exchange, xt = None, None
    if sharded:
        xt = sorter.exchange_timing()
        exchange = xt["exchange"]
    n_sorted_local = sorter.last_n_out if exchange == "partition-first" else n_local
    kernel_name = (sorter.sorter if sharded else sorter).pass_kernel_for(n_sorted_local)
    if msd:
        kernel_name = {"p1_scatter_top_byte": "grs_onesweep_region", "p2_scatter_byte2": "grs_onesweep_seg",
                       "p3_local_sort": "grs_msd_local"}[dom]
    alg_bytes = n_sorted_local * 2 * (kb // 8 + (4 if pairs else 0)) * (kb // rb if fused else 1)
    achieved = alg_bytes / (mean_pass_ms * 1e-3) / 1e9
    # SURVEY §8d credits P_cfg = key bits / digit bits passes, whatever schedule ran
    passes = kb // rb
    del keys_pool, vals_pool, sorter
    torch.cuda.empty_cache()

    cpu_b = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline and cpu:
        cpu_b = cpu_baseline(min(a.cpu_sample, n_local), kb, pairs, seed)

    # PMC bytes per launch: rocprofv3 child runs of this workload (after the timed region)
    want_traffic = traffic
    traffic, traffic_info = None, None
    if rank == 0 and world == 1 and not sharded and not a.no_traffic and want_traffic:
        traffic_info, why = measure_traffic(a, config, options, n_local, kernel_name, dist)
        if traffic_info:
            traffic = traffic_info["bytes_per_launch"]
        else:
            traffic_info = {"error": why}
    elif a.traffic_json and os.path.exists(a.traffic_json):
        rec = json.load(open(a.traffic_json))
        if rec.get("n") == n_sorted_local and rec.get("config") == config:
            traffic = rec.get("hbm_bytes_per_launch")

    sort_alg = n_local * 2 * passes * (kb // 8 + (4 if pairs else 0))
    schedule = "msd" if msd else "lsd-fused" if fused else "lsd"
    moved = moved_bytes(n_sorted_local, kb, pairs, rb, "msd" if msd else "lsd")
    if rank != 0:
        return None
    value = n_total * steps / elapsed / 1e9
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "Gkeys/s", "n_gpus": world,
        "steps": steps, "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u32" if kb == 32 else "u64",
        "data": ("synthetic: splitmix64(seed ^ global_index) uniform keys" if dist == "uniform" else
                 "synthetic: the reference's input, 0..N-1 shuffled by a seeded bijection "
                 "(grs_fill_permutation; main.cpp:119-125)")
                + ", a distinct unsorted buffer per step resident in HBM"
                + ("; payload = global index" if pairs else ""),
        "config": {"workload": desc, "dist": dist, "keys_per_gpu": n_local, "total_keys": n_total,
                   "key_bits": kb, "payload": "u32" if pairs else None, "radix_bits": rb,
                   "passes": passes, "parallelism": f"range-shard x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic, "kernel": kernel_name,
                     "kernel_mean_ms": round(mean_pass_ms, 5),
                     "alg_bytes_per_launch": alg_bytes,
                     "traffic_over_alg": round(traffic / alg_bytes, 4) if traffic else None},
        # whole-sort view of SURVEY.md §8d: B_alg = N x 2 x passes x (key + value bytes)
        # over the whole step (histogram and exchange included)
        "sort_roofline": {"achieved": round(sort_alg / (elapsed / steps) / 1e9, 1),
                          "frac": round(sort_alg / (elapsed / steps) / 1e9 / HBM_PEAK_GBPS, 4),
                          "alg_bytes_per_step": sort_alg, "unit": "GB/s",
                          "credited_passes": passes},
        # what the schedule that ran actually moves (moved_bytes), over the same step time
        "moved_roofline": {"bytes_per_step": moved,
                           "achieved": round(moved / (elapsed / steps) / 1e9, 1),
                           "frac": round(moved / (elapsed / steps) / 1e9 / HBM_PEAK_GBPS, 4),
                           "unit": "GB/s", "schedule": schedule},
        "cpu_baseline": cpu_b,
        "phases_ms": {"hist": round(hist_ms, 5), "pass_mean": round(mean_pass_ms, 5),
                      "sort_total_gpu": round(sort_ms, 5)},
        "schedule": schedule,
        "check": {"inversions_last_step": inversions},
    }
    if msd:
        out["phases_ms"]["msd"] = msd_phases
        out["config"]["passes"] = f"{passes} (credited, SURVEY §8d); MSD schedule: 2 scatters + LDS sort"
    if options:
        out["config"]["options"] = options
    if traffic_info:
        out["traffic_pmc"] = traffic_info
        if traffic_info.get("sort_bytes"):
            # every kernel of one sort, from the same PMC runs: the bytes HBM really moved
            out["moved_roofline"]["pmc_bytes_per_step"] = traffic_info["sort_bytes"]
            out["moved_roofline"]["pmc_over_moved"] = round(traffic_info["sort_bytes"] / moved, 4)
    if sharded:
        out["phases_ms"]["recv_keys_rank0"] = n_sorted_local
        out["config"]["exchange"] = exchange
        xms = max(xt["exchange_ms"], 1e-6)
        out["exchange_rank0"] = {
            "before_ms": round(xt["before_ms"], 4), "exchange_ms": round(xt["exchange_ms"], 4),
            "after_ms": round(xt["after_ms"], 4), "bytes_sent": xt["bytes_sent"],
            "bytes_received": xt["bytes_received"],
            "xgmi_GBps_sent": round(xt["bytes_sent"] / xms / 1e6, 1)}
    return out


def main():
    a = parse()
    if a.pmc_probe:
        opts = dict(o.split("=", 1) for o in a.opt)
        pmc_probe(a, {k: (int(v) if v.lstrip("-").isdigit() else v) for k, v in opts.items()})
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and not (world == 1 and a.gpus == 1):
        if world == 1:
            raise SystemExit("--gpus N > 1 must be launched with torchrun (one rank per GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    sharded = world > 1 or a.sharded
    if sharded and world == 1:
        import socket

        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)

    out = run_config(a, a.config, world, rank, local, dev, sharded, a.steps, a.warmup, a.dist)
    keep = ("value", "unit", "ms_per_step", "steps", "warmup", "roofline", "sort_roofline",
            "moved_roofline", "phases_ms", "check", "schedule", "config", "traffic_pmc")
    default_line = world == 1 and not sharded and a.config == "c4" and not a.n and a.dist == "uniform"
    # the north star's own 1-GPU target (BASELINE.json: >= 60 % of the HBM roofline on 256 M
    # uniform uint32 keys) as a second leg of the same driver-timed run, after the headline
    if default_line and not a.no_north_star:
        ns = run_config(a, "ns", world, rank, local, dev, sharded, a.steps, a.warmup)
        if out is not None and ns is not None:
            out["north_star"] = {k: ns[k] for k in keep if k in ns}
    # the reference's own input (0..N-1 shuffled, main.cpp:119-125) at the north star's 2^28 and
    # C4's 2^30 keys, through the default schedule (no PMC child runs, no CPU baseline)
    if default_line and not a.no_reference_input:
        legs = {}
        for cfg in ("ns", "c4"):
            r = run_config(a, cfg, world, rank, local, dev, sharded, a.steps, a.warmup, "perm",
                           traffic=False, cpu=False)
            if r is not None:
                legs[cfg] = {k: r[k] for k in keep if k in r}
        if out is not None:
            out["reference_input"] = legs
    if out is not None:
        print(json.dumps(out), flush=True)
    if sharded:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
