"""Driver of tools/lab8.hip: P3 (the MSD sort's LDS segment sort) with dword against 16-B HBM
accesses, on P3's real geometry: 65536 segments of n / 65536 +- 3 sqrt keys, each read from a
region that starts after a random gap (any alignment) and written packed (any alignment); keys
grouped by their top 16 bits.  rounds 0 = the load + store skeleton, 2 = the sort.
python tools/lab8.py [--n N] [--shapes 768:24:1] [--modes 0,1,2,3]"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import gpuradixsort_amd as grs  # noqa: E402

L = None   # the lab library (--lib)
vp = ctypes.c_void_p
NAMES = {0: "dword ld / dword st", 1: "dword ld / 16B st rot", 3: "dword ld / 16B st"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 30)
    ap.add_argument("--shapes", default="768:24:1")
    ap.add_argument("--modes", default="0,1,3")
    ap.add_argument("--u64-shapes", default="256:20,512:10,1024:5")
    ap.add_argument("--half-shapes", default="",
                    help="grs::LocalSort16 (low halves in LDS) shapes block:items:minw, e.g. 512:36:6")
    ap.add_argument("--persistent", default="",
                    help="persistent static-stride P3 block:items:minw:half:grid_per_cu, e.g. 256:20:6:0:6")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--exact", action="store_true",
                    help="segments of exactly n / 65536 keys, no gaps (every run 16-B... 64-KB aligned, as the "
                         "reference's shuffled 0..n-1 makes them)")
    ap.add_argument("--perm-keys", action="store_true",
                    help="the low bits of every segment a permutation of 0..m-1 (the reference's input)")
    ap.add_argument("--u64", action="store_true", help="u64 keys (C5), shape 256:20, modes 0 (6 rounds) / "
                                                       "1 (16-B, 2 rounds + run finish)")
    ap.add_argument("--lib", default="liblab8.so", help="liblab8_lds0/2.so: P3's LDS layout 0 / 2 (Makefile)")
    a = ap.parse_args()
    global L
    L = ctypes.CDLL(os.path.join(HERE, a.lib))
    dev = torch.device("cuda", 0)
    nseg = 65536
    g = torch.Generator(device="cpu").manual_seed(8)
    m = a.n // nseg
    sd = max(1, int(3 * m ** 0.5))
    lens = (m + torch.randint(-sd, sd + 1, (nseg,), generator=g)).clamp(min=1)
    # the total back to n, spread evenly (never into one segment: it must fit the LDS shape)
    diff = a.n - int(lens.sum())
    lens += diff // nseg
    lens[: abs(diff % nseg)] += 1 if diff % nseg > 0 else 0
    assert int(lens.sum()) == a.n and int(lens.max()) <= m + sd + 2, (int(lens.sum()), int(lens.max()))
    gaps = torch.randint(0, 257, (nseg,), generator=g)
    if a.exact:
        lens = torch.full((nseg,), m, dtype=torch.int64)
        gaps = torch.zeros(nseg, dtype=torch.int64)
    outoff = torch.cumsum(lens, 0) - lens
    inoff = torch.cumsum(lens + gaps, 0) - lens - gaps + (0 if a.exact else 3)   # +3: any alignment
    total_in = int(inoff[-1] + lens[-1]) + 64
    n = int(lens.sum())
    if a.u64:
        return run_u64(a, dev, nseg, m, sd, lens, inoff, outoff, total_in, n)
    # keys: segment b holds prefix b in the top 16 bits, random low halves
    low = torch.empty(total_in, dtype=torch.int32, device=dev)
    grs.fill_splitmix(low, 9)
    seg_of = torch.repeat_interleave(torch.arange(nseg, dtype=torch.int64, device=dev), lens.to(dev))
    pos_in = (torch.arange(n, dtype=torch.int64, device=dev) - outoff.to(dev)[seg_of] + inoff.to(dev)[seg_of])
    keys = low.clone()
    lowbits = low[pos_in].to(torch.int64) & 0xFFFF
    if a.perm_keys:   # segment b's low bits: a permutation of 0..m-1 (exact segments)
        assert a.exact
        r = torch.argsort(torch.rand(nseg, m, device=dev), dim=1).reshape(-1)
        lowbits = r.to(torch.int64)
        del r
    keys[pos_in] = ((seg_of << 16) | lowbits).to(torch.int32)
    want = torch.sort(keys[pos_in].to(torch.int64) & 0xFFFFFFFF)[0]
    out = torch.empty(n + 64, dtype=torch.int32, device=dev)
    i32 = lambda t: t.to(torch.int32).to(dev)   # noqa: E731
    d_in, d_out, d_len = i32(inoff), i32(outoff), i32(lens)
    stream = vp(torch.cuda.current_stream().cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    print(f"n {n}, segments {nseg} of {m} +- {sd}, regions at gaps 0..256 (+3); exact={a.exact} "
          f"perm_keys={a.perm_keys}", flush=True)
    if a.half_shapes:
        run_half(a, keys, out, d_in, d_out, d_len, nseg, n, m, sd, want, stream, e0, e1)
    if a.persistent:
        run_persistent(a, keys, out, d_in, d_out, d_len, nseg, n, m, sd, want, stream, e0, e1)
    for spec in filter(None, a.shapes.split(",")):
        b, it, c16 = (int(x) for x in spec.split(":"))
        if b * it < m + sd:
            print(f"{spec}: segments too long for the shape", flush=True)
            continue
        for mode in (int(x) for x in a.modes.split(",")):
            for rounds in (0, 2):
                ts = []
                for _ in range(a.reps):
                    e0.record()
                    rc = L.lab8_p3(b, it, c16, mode, rounds, vp(keys.data_ptr()), vp(out.data_ptr()),
                                   vp(d_in.data_ptr()), vp(d_out.data_ptr()), vp(d_len.data_ptr()), nseg,
                                   stream)
                    e1.record()
                    torch.cuda.synchronize()
                    assert rc == 0, (spec, mode, rc)
                    ts.append(e0.elapsed_time(e1))
                ms = statistics.median(ts)
                ok = ""
                if rounds == 2:
                    ok = f" sorted={bool(torch.equal(out[:n].to(torch.int64) & 0xFFFFFFFF, want))}"
                print(f"p3 {spec} mode {mode} ({NAMES[mode]:22s}) rounds={rounds}: {ms * 1e3:8.1f} us "
                      f"{n * 8 / ms / 1e6:7.1f} GB/s ({n * 8 / ms / 1e6 / 8000:.3f} of 8 TB/s){ok}", flush=True)


def run_half(a, keys, out, d_in, d_out, d_len, nseg, n, m, sd, want, stream, e0, e1):
    for spec in filter(None, a.half_shapes.split(",")):
        b, it, minw = (int(x) for x in spec.split(":"))
        if b * it < m + sd:
            print(f"half {spec}: segments too long for the shape", flush=True)
            continue
        for rounds in (0, 2):
            ts = []
            for _ in range(a.reps):
                e0.record()
                rc = L.lab8_p3h(b, it, minw, rounds, vp(keys.data_ptr()), vp(out.data_ptr()), vp(d_in.data_ptr()),
                                vp(d_out.data_ptr()), vp(d_len.data_ptr()), nseg, stream)
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0, (spec, rc)
                ts.append(e0.elapsed_time(e1))
            ms = statistics.median(ts)
            ok = f" sorted={bool(torch.equal(out[:n].to(torch.int64) & 0xFFFFFFFF, want))}" if rounds else ""
            print(f"p3 half {spec} (LocalSort16) rounds={rounds}: {ms * 1e3:8.1f} us "
                  f"{n * 8 / ms / 1e6:7.1f} GB/s ({n * 8 / ms / 1e6 / 8000:.3f} of 8 TB/s){ok}", flush=True)


def run_persistent(a, keys, out, d_in, d_out, d_len, nseg, n, m, sd, want, stream, e0, e1):
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for spec in filter(None, a.persistent.split(",")):
        b, it, minw, half, per_cu = (int(x) for x in spec.split(":"))
        if b * it < m + sd:
            print(f"persistent {spec}: segments too long for the shape", flush=True)
            continue
        for rounds in (2,):
            ts = []
            for _ in range(a.reps):
                e0.record()
                rc = L.lab8_p3s(b, it, minw, half, per_cu * cus, rounds, vp(keys.data_ptr()), vp(out.data_ptr()),
                                vp(d_in.data_ptr()), vp(d_out.data_ptr()), vp(d_len.data_ptr()), nseg, stream)
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0, (spec, rc)
                ts.append(e0.elapsed_time(e1))
            ms = statistics.median(ts)
            ok = f" sorted={bool(torch.equal(out[:n].to(torch.int64) & 0xFFFFFFFF, want))}"
            print(f"p3 persistent {spec} (grid {per_cu} x {cus}) rounds={rounds}: {ms * 1e3:8.1f} us "
                  f"{n * 8 / ms / 1e6:7.1f} GB/s ({n * 8 / ms / 1e6 / 8000:.3f} of 8 TB/s){ok}", flush=True)


def run_u64(a, dev, nseg, m, sd, lens, inoff, outoff, total_in, n):
    low = torch.empty(total_in, dtype=torch.int64, device=dev)
    grs.fill_splitmix(low, 10)
    seg_of = torch.repeat_interleave(torch.arange(nseg, dtype=torch.int64, device=dev), lens.to(dev))
    pos_in = (torch.arange(n, dtype=torch.int64, device=dev) - outoff.to(dev)[seg_of] + inoff.to(dev)[seg_of])
    keys = low.clone()
    keys[pos_in] = (seg_of << 47) | (low[pos_in] & ((1 << 47) - 1))   # prefix in bits 47..62: signed order = unsigned
    want = torch.sort(keys[pos_in])[0]
    out = torch.empty(n + 64, dtype=torch.int64, device=dev)
    i32 = lambda t: t.to(torch.int32).to(dev)   # noqa: E731
    d_in, d_out, d_len = i32(inoff), i32(outoff), i32(lens)
    stream = vp(torch.cuda.current_stream().cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    print(f"u64: n {n}, segments {nseg} of {m} +- {sd}", flush=True)
    for spec in a.u64_shapes.split(","):
        b, it = (int(x) for x in spec.split(":"))
        if b * it < m + sd:
            continue
        for mode in (0, 1):
            for rounds in (0, 6):
                ts = []
                for _ in range(a.reps):
                    e0.record()
                    rc = L.lab8_p3w(b, it, mode, rounds, vp(keys.data_ptr()), vp(out.data_ptr()),
                                    vp(d_in.data_ptr()), vp(d_out.data_ptr()), vp(d_len.data_ptr()), nseg, stream)
                    e1.record()
                    torch.cuda.synchronize()
                    assert rc == 0, rc
                    ts.append(e0.elapsed_time(e1))
                ms = statistics.median(ts)
                ok = f" sorted={bool(torch.equal(out[:n], want))}" if rounds else ""
                name = {0: "6 rounds, 8-B", 1: "8-B ld, 16-B st, 2 rounds + runs"}[mode]
                print(f"p3 u64 {spec} mode {mode} ({name}) rounds={rounds}: "
                      f"{ms * 1e3:8.1f} us {n * 16 / ms / 1e6:7.1f} GB/s ({n * 16 / ms / 1e6 / 8000:.3f} of 8 TB/s)"
                      f"{ok}", flush=True)


if __name__ == "__main__":
    main()
