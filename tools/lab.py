"""Kernel laboratory: interleaved timing of onesweep-pass variants (tools/lab.hip).

python tools/lab.py [--n N] [--rounds R] [--lib liblab.so] [--copy]
                    [--variants kb:pairs:block:items:dbg[:grid],...]
Prints one line per variant: median / min ms and algorithmic GB/s of one pass
(2 x (key + payload bytes) per key); DBG & 8 variants also print per-phase cycle stamps.
"""
import argparse
import ctypes
import os
import statistics
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import gpuradixsort_amd as grs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 27)
    ap.add_argument("--lib", default="liblab.so")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="32:0:512:24:0")
    ap.add_argument("--copy", action="store_true")
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    L = ctypes.CDLL(os.path.join(HERE, a.lib))
    vp = ctypes.c_void_p
    P = lambda t: vp(t.data_ptr())  # noqa: E731
    n = a.n
    dev = torch.device("cuda", 0)
    sp = vp(torch.cuda.current_stream().cuda_stream)

    variants = []
    for v in a.variants.split(","):
        # "a32:..." = atomic-rank kernel (lab_ar), grid 0 = one tile per WG; "b32:..." = ar2
        # "c32:..." = v3 (lab_v3, grid = persistent workgroups)
        ar = {"a": 1, "b": 2, "c": 3}.get(v[0], 0)
        parts = [int(x) for x in v.lstrip("abc").split(":")]
        variants.append(tuple(parts + [0] * (6 - len(parts))) + (int(ar),))
    bufs = {}
    for kb in sorted({v[0] for v in variants}):
        dt = torch.uint32 if kb == 32 else torch.uint64
        keys = torch.empty(n, dtype=dt, device=dev)
        grs.fill_splitmix(keys, 0x6A09E667F3BCC908 + 4)
        hist = torch.zeros(8 * 256, dtype=torch.uint32, device=dev)
        scratch = torch.zeros(1, dtype=torch.uint32, device=dev)
        assert L.lab_hist(kb, P(keys), ctypes.c_uint32(n), P(hist), P(scratch), ctypes.c_uint32(0), sp) == 0
        bufs[kb] = (keys, torch.empty_like(keys), hist)
    vin = torch.arange(n, dtype=torch.int64, device=dev).to(torch.uint32)
    vout = torch.empty_like(vin)
    ticket = torch.zeros(4, dtype=torch.uint32, device=dev)
    max_tiles = (n + 1023) // 1024
    err = torch.zeros(64 + 8 * max_tiles + 64, dtype=torch.uint32, device=dev)
    print("lib", a.lib)
    st = torch.zeros(max_tiles * 256, dtype=torch.uint32, device=dev)
    st2 = torch.zeros_like(st)
    torch.cuda.synchronize()

    def run(v):
        kb, pairs, block, items, dbg, grid, ar = v
        keys, out, hist = bufs[kb]
        if ar == 3:
            rc = L.lab_v3(kb, pairs, block, items, dbg, grid, P(keys), P(out), P(vin), P(vout),
                          ctypes.c_uint32(n), P(hist), P(ticket), P(st), P(st2), P(err), 0, sp)
        elif ar == 2:
            rc = L.lab_ar2(kb, pairs, block, items, dbg, P(keys), P(out), P(vin), P(vout),
                           ctypes.c_uint32(n), P(hist), P(ticket), P(st), P(st2), P(err), 0, sp)
        elif ar:
            rc = L.lab_ar(kb, pairs, block, items, dbg, grid, P(keys), P(out), P(vin), P(vout),
                          ctypes.c_uint32(n), P(hist), P(ticket), P(st), P(st2), P(err), 0, sp)
        else:
            L.lab_set_persistent(grid)
            rc = L.lab_pass2(kb, pairs, block, items, dbg, P(keys), P(out), P(vin), P(vout),
                             ctypes.c_uint32(n), P(hist), P(ticket), P(st), P(st2), P(err), 0, sp)
        assert rc == 0, (v, rc)

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {v: [] for v in variants}
    copy_t = []
    for _ in range(a.rounds):
        for v in variants:
            st.zero_()
            ticket.zero_()
            torch.cuda.synchronize()
            e0.record()
            run(v)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
        if a.copy:
            k32 = bufs[min(bufs)]
            e0.record()
            L.lab_copy(P(k32[0]), P(k32[1]), ctypes.c_uint32(n), sp)
            e1.record()
            torch.cuda.synchronize()
            copy_t.append(e0.elapsed_time(e1))
    print(f"n={n}  error word={int(err[0].item())}")
    if a.check:
        # one pass = stable partition by the low 8 bits: compare with torch's stable sort
        for v in variants:
            if v[4] & ~96:
                continue
            kb, pairs = v[0], v[1]
            keys, out, hist = bufs[kb]
            st.zero_()
            ticket.zero_()
            err.zero_()
            run(v)
            torch.cuda.synchronize()
            k64 = keys.view(torch.int32 if kb == 32 else torch.int64).to(torch.int64)
            dig = k64 & 255
            _, idx = torch.sort(dig, stable=True)
            ok = torch.equal(out.view(k64.dtype if kb == 64 else torch.int32).to(torch.int64)
                             if kb == 32 else out.view(torch.int64), k64[idx])
            okv = (not pairs) or torch.equal(vout.to(torch.int64) if False else
                                            vout.view(torch.int32).to(torch.int64) & 0xFFFFFFFF,
                                            idx)
            print(f"check {v}: keys {'OK' if ok else 'MISMATCH'} vals {'OK' if okv else 'MISMATCH'}"
                  f" err={int(err[0].item())}")
    if copy_t:
        med = statistics.median(copy_t)
        print(f"copy x4 of n u32: median {med:8.4f} ms  {n * 8 / med / 1e6:8.1f} GB/s")
    for v in variants:
        kb, pairs = v[0], v[1]
        alg = n * 2 * (kb // 8 + (4 if pairs else 0))
        med, mn = statistics.median(times[v]), min(times[v])
        print(f"{['  ', 'AR', 'A2', 'V3'][v[6]]} kb={kb} pairs={pairs} block={v[2]:4d} items={v[3]:2d} dbg={v[4]:2d} grid={v[5]:4d}"
              f"  median {med:8.4f} ms  min {mn:8.4f}  {alg / med / 1e6:8.1f} GB/s")
    names = ["ticket+issue", "load+hist", "p2", "p3", "p4", "reorder", "store"]
    for v in variants:
        if v[4] & 16:
            err.zero_()
            st.zero_()
            ticket.zero_()
            run(v)
            torch.cuda.synchronize()
            tiles = (n + v[2] * v[3] - 1) // (v[2] * v[3])
            a_ = err[64:64 + 8 * tiles].view(torch.int32).cpu().numpy().reshape(tiles, 8).astype("float64")
            if v[6] == 3:
                print(f"v3 look-back stats {v}: rounds mean {a_[:,0].mean():.2f} p90 {np.percentile(a_[:,0],90):.0f} max {a_[:,0].max():.0f}; spins mean {a_[:,1].mean():.2f} p90 {np.percentile(a_[:,1],90):.0f} max {a_[:,1].max():.0f}")
                continue
            if v[4] & 96:
                print(f"lookback2 stats {v}: tile rounds mean {a_[:,0].mean():.2f} p90 {np.percentile(a_[:,0],90):.0f} max {a_[:,0].max():.0f}; "
                      f"spins mean {a_[:,1].mean():.2f} p90 {np.percentile(a_[:,1],90):.0f}; group rounds mean {a_[:,2].mean():.2f} "
                      f"p90 {np.percentile(a_[:,2],90):.0f} max {a_[:,2].max():.0f}; fallbacks mean {a_[:,3].mean():.2f} p90 {np.percentile(a_[:,3],90):.0f}")
                continue
            print(f"lookback stats {v}: rounds mean {a_[:,0].mean():.2f} p90 {np.percentile(a_[:,0],90):.0f} "
                  f"max {a_[:,0].max():.0f}; spins mean {a_[:,1].mean():.2f} p90 {np.percentile(a_[:,1],90):.0f}; "
                  f"walk mean {a_[:,2].mean():.1f} p90 {np.percentile(a_[:,2],90):.0f}; "
                  f"first RT cycles mean {a_[1:,3].mean():.0f} p10 {np.percentile(a_[1:,3],10):.0f} p90 {np.percentile(a_[1:,3],90):.0f}")
        if not (v[4] & 8):
            continue
        err.zero_()
        st.zero_()
        ticket.zero_()
        run(v)
        torch.cuda.synchronize()
        tiles = (n + v[2] * v[3] - 1) // (v[2] * v[3])
        a_ = err[64:64 + 8 * tiles].view(torch.int32).cpu().numpy().reshape(tiles, 8).astype("float64")
        if v[6] == 3:
            m = a_[1:, :6].mean(0)   # cycles since the iteration start at each phase end
            d = np.diff(np.concatenate([[0.0], m]))
            print(f"v3 stamps {v}: L0-wait={d[0]:.0f} rank+B1={d[1]:.0f} digits+B2={d[2]:.0f} "
                  f"fold+B2.5={d[3]:.0f} reorder+lookback+B3={d[4]:.0f} store+drain={d[5]:.0f} "
                  f"total={m[5]:.0f}")
            continue
        if v[6]:
            m = a_[:, :7].mean(0)
            print(f"stamps {v}: ticket+load={m[6]:.0f} rank+B1={m[1]-m[0]:.0f} scan+B2={m[2]-m[1]:.0f} "
                  f"lookback+B3={m[3]-m[2]:.0f} reorder+B4={m[4]-m[3]:.0f} store+drain={m[5]-m[4]:.0f} "
                  f"total={m[5]:.0f}  (p90 lookback {np.percentile(a_[:, 3] - a_[:, 2], 90):.0f})")
            continue
        ph = a_[:, :7]
        d = np.diff(np.concatenate([np.zeros((tiles, 1)), ph], axis=1), axis=1)
        print(f"stamps {v}: mean cycles per phase "
              + ", ".join(f"{nm}={x:.0f}" for nm, x in zip(names, d.mean(0)))
              + f"  total={ph[:, 6].mean():.0f}")


if __name__ == "__main__":
    main()
