"""Round-2 kernel laboratory driver (tools/lab2.hip): interleaved timing of pass variants.

python tools/lab2.py [--n N] [--rounds R] [--check] [--copy]
       [--variants v4:kb:pairs:block:items:minw:opt,v6:kb:pairs:block:items:minw:opt:grid,...]
Prints median / min ms and algorithmic GB/s (2 x (key + payload) bytes per key) per variant;
variants with the stamp bit (opt & 8) also print mean cycles per phase.
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--variants", default="p4:32:0:1024:36:1:272")
    ap.add_argument("--copy", action="store_true")
    ap.add_argument("--lds-atomic", action="store_true", help="returning ds_add rate by address multiplicity")
    ap.add_argument("--rot", type=int, default=0, help="OPT 2048 store-sweep rotation per tile (keys)")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--xcc", action="store_true", help="print the XCC id of each block (placement)")
    ap.add_argument("--lib", default="", help="load tools/liblab2_LIB.so (a build with other knobs)")
    ap.add_argument("--lib4", default="", help="p4 variants from tools/liblab4_LIB4.so")
    ap.add_argument("--emu", default="", help="block:items:mode:lds,... pass memory-pattern emulation")
    ap.add_argument("--emu-handoff", default="", help="block:items:var:lds,... boundary-line hand-off emulation")
    ap.add_argument("--replay", default="", help="block:items:rb,... the pass's exact loads and stores, no ranking")
    ap.add_argument("--emu16", default="", help="block:items,... C2 memory pattern: 8 passes of 16 runs")
    ap.add_argument("--emu-pairs", default="", help="block:items:aos:lds,... pairs memory pattern (SoA vs AoS)")
    a = ap.parse_args()
    L = ctypes.CDLL(os.path.join(HERE, f"liblab2{'_' + a.lib if a.lib else ''}.so"))
    l4 = os.path.join(HERE, f"liblab4{'_' + a.lib4 if a.lib4 else ''}.so")
    L4 = ctypes.CDLL(l4) if os.path.exists(l4) else None
    vp = ctypes.c_void_p
    P = lambda t: vp(t.data_ptr())  # noqa: E731
    n = a.n
    dev = torch.device("cuda", 0)
    sp = vp(torch.cuda.current_stream().cuda_stream)
    variants = []
    for v in a.variants.split(","):
        f = v.split(":")
        variants.append((f[0],) + tuple(int(x) for x in f[1:]))
    bufs = {}
    hist4 = {}
    for kb in sorted({v[1] for v in variants}):
        dt = torch.uint32 if kb == 32 else torch.uint64
        keys = torch.empty(n, dtype=dt, device=dev)
        grs.fill_splitmix(keys, 0x6A09E667F3BCC908 + 4)
        k64 = keys.view(torch.int32 if kb == 32 else torch.int64).to(torch.int64)
        hist = torch.bincount(k64 & 255, minlength=256).to(torch.int32).view(torch.uint32)
        bufs[kb] = (keys, torch.empty_like(keys), hist.contiguous())
        hist4[kb] = torch.bincount(k64 & 15, minlength=16).to(torch.int32).view(torch.uint32).contiguous()
    vin = torch.arange(n, dtype=torch.int64, device=dev).to(torch.int32).view(torch.uint32)
    vout = torch.empty_like(vin)
    ticket = torch.zeros(64, dtype=torch.uint32, device=dev)   
    max_tiles = n // 4096 + 64
    err = torch.zeros(64 + 12 * max_tiles + 64, dtype=torch.uint32, device=dev)
    err[63] = a.rot
    st = torch.zeros(3 * max_tiles * 256, dtype=torch.uint32, device=dev)
    st2 = torch.zeros_like(st)
    torch.cuda.synchronize()

    xr_hist = {}

    def range_hist(kb, tile, radix=256):
        """per-XCD-range digit-0 histograms [8][radix] and the range size in tiles (OPT 1048576)"""
        if (kb, tile, radix) not in xr_hist:
            keys = bufs[kb][0]
            tiles = (n + tile - 1) // tile
            R = ((tiles + 7) // 8 + 7) // 8 * 8
            k64 = keys.view(torch.int32 if kb == 32 else torch.int64).to(torch.int64) & (radix - 1)
            hs = [torch.bincount(k64[min(n, c * R * tile):min(n, (c + 1) * R * tile)], minlength=radix)
                  for c in range(8)]
            xr_hist[(kb, tile, radix)] = (torch.stack(hs).to(torch.int32).view(torch.uint32).contiguous(), R)
        return xr_hist[(kb, tile, radix)]

    def run(v):
        kind, kb, pairs, block, items = v[:5]
        keys, out, hist = bufs[kb]
        stride, rtiles = 0, 0
        if kind in ("v4", "v6") and v[6] & 1048576:
            hist, rtiles = range_hist(kb, block * items)
            stride = 256
        args = (P(keys), P(out), P(vin), P(vout), ctypes.c_uint32(n), P(hist), P(ticket), P(st),
                P(st2), P(err), 0, sp, ctypes.c_uint32(stride), ctypes.c_uint32(rtiles))
        if kind in ("r4", "r6", "v4", "v6"):
            raise SystemExit(f"variant kind {kind}: the lab fork of the pass was removed in round 5 "
                             "(git show 729d494:tools/lab_pass.hpp); p4 = the shipped kernel")
        if kind == "r4":   # r4:32:0:block:items:minw:opt  (4-bit digits, low nibble)
            rc = L.lab2_v4rb4(block, items, v[5], v[6], P(keys), P(out), ctypes.c_uint32(n),
                              P(hist4[kb]), P(ticket), P(st), P(st2), P(err), sp)
        elif kind == "r6":   # r6:32:0:block:items:minw:opt:grid  (4-bit digits, persistent)
            h4, stride, rtiles = hist4[kb], 0, 0
            if v[6] & 1048576:
                h4, rtiles = range_hist(kb, block * items, 16)
                stride = 16
            rc = L.lab2_v6rb4(block, items, v[5], v[6], v[7], P(keys), P(out), ctypes.c_uint32(n),
                              P(h4), P(ticket), P(st), P(st2), P(err), sp, ctypes.c_uint32(stride),
                              ctypes.c_uint32(rtiles))
        elif kind == "v4":
            rc = L.lab2_v4(kb, pairs, block, items, v[5], v[6], *args)
        elif kind == "p4":   # the shipped kernel (tools/lab4.hip): p4:kb:pairs:block:items:minw:opt
            rc = L4.lab4_v4(kb, pairs, block, items, v[5], v[6], *args)
        elif kind == "v6":   # v6:kb:pairs:block:items:minw:opt:grid
            rc = L.lab2_v6(kb, pairs, block, items, v[5], v[6], v[7], *args)
        else:
            raise SystemExit(f"unknown variant kind {kind}")
        assert rc == 0, (v, rc)

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {v: [] for v in variants}
    for r in range(a.rounds):
        for v in variants:
            st.zero_()
            ticket.zero_()
            err.zero_()
            err[63] = a.rot
            torch.cuda.synchronize()
            if r == 0:
                print("run", v, flush=True)
            e0.record()
            run(v)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
            if r == 0:
                print(f"   {times[v][-1]:.4f} ms  err={int(err[0].item())}", flush=True)
    print(f"n={n}  error word={int(err[0].item())}", flush=True)
    if a.xcc:
        o = torch.zeros(4096, dtype=torch.uint32, device=dev)
        assert L.lab2_xcc(P(o), 4096, sp) == 0
        torch.cuda.synchronize()
        x = o.cpu().numpy()
        b = np.arange(4096)
        print("xcc ids of blocks 0..31:", x[:32].tolist())
        print("blocks whose xcc == (b - b0) % 8 + xcc0:", int(((b % 8 + x[0]) % 8 == x).sum()), "of 4096")
    if a.lds_atomic:
        o = torch.zeros(1024, dtype=torch.uint32, device=dev)
        for d in (64, 32, 16, 8, 1):
            for _ in range(2):
                assert L.lab2_lds_atomic(d, 4096, P(o), 256, sp) == 0
                torch.cuda.synchronize()
            cyc = o[:256].to(torch.float64).mean().item()
            # s_memtime ticks at 100 MHz on gfx9: convert with the shader clock estimate below
            print(f"lds_atomic distinct={d:2d}: {cyc / 4096:8.3f} memtime ticks per wave-iteration "
                  f"(16 waves per CU)", flush=True)
    if a.copy:
        src = torch.empty(n * 2, dtype=torch.uint32, device=dev)
        src.fill_(7)
        dst = torch.empty_like(src)
        nbytes = n * 4
        for kind in (0, 1):
            for unroll in (1, 4, 8):
                for grid in (1024, 2048, 4096, 8192):
                    ts = []
                    for _ in range(5):
                        e0.record()
                        assert L.lab2_stream(kind, unroll, grid, P(src), P(dst), ctypes.c_uint64(nbytes), sp) == 0
                        e1.record()
                        torch.cuda.synchronize()
                        ts.append(e0.elapsed_time(e1))
                    med = statistics.median(ts)
                    moved = nbytes * (2 if kind == 0 else 1)
                    print(f"{'copy' if kind == 0 else 'read'} unroll={unroll} grid={grid}: "
                          f"{med:.4f} ms  {moved / med / 1e6:.1f} GB/s", flush=True)
    if a.emu:
        keys, out, _ = bufs[32]
        for e in a.emu.split(","):
            b, it, mode, lds = (int(x) for x in e.split(":"))
            ts = []
            for _ in range(a.rounds):
                e0.record()
                assert L.lab2_emu(b, it, mode, lds, P(keys), P(out), ctypes.c_uint32(n), sp) == 0
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            med = statistics.median(ts)
            print(f"emu {e:20s} median {med:8.4f} ms  {n * 8 / med / 1e6:8.1f} GB/s", flush=True)
    if a.emu_handoff:
        keys, out, _ = bufs[32]
        ring = torch.zeros(2048 * 256 * 32, dtype=torch.uint32, device=dev)
        flags = torch.zeros(2048, dtype=torch.uint32, device=dev)
        herr = torch.zeros(4, dtype=torch.uint32, device=dev)
        epoch = 1
        for e in a.emu_handoff.split(","):
            b, it, var, lds = (int(x) for x in e.split(":"))
            ts = []
            for _ in range(a.rounds):
                epoch += 1
                e0.record()
                assert L.lab2_emu_handoff(b, it, var, lds, P(keys), P(out), ctypes.c_uint32(n), P(ring),
                                          P(flags), ctypes.c_uint32(epoch), P(herr), sp) == 0
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            med = statistics.median(ts)
            print(f"emu_handoff {e:16s} median {med:8.4f} ms  {n * 8 / med / 1e6:8.1f} GB/s "
                  f"err={int(herr[0].item())}", flush=True)
    if a.replay:
        keys, out, _ = bufs[32]
        k64 = keys.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        for e in a.replay.split(","):
            f = [int(x) for x in e.split(":")]
            b, it, rb = f[:3]
            x8 = f[3] if len(f) > 3 else 0
            R, T = 1 << rb, b * it
            tiles = (n + T - 1) // T
            pos = torch.arange(n, dtype=torch.int64, device=dev)
            comp = (pos // T) * R + (k64 & (R - 1))
            srt, perm = torch.sort(comp, stable=True)
            pre = keys.view(torch.int32)[perm].view(torch.uint32).contiguous()
            cnt = torch.bincount(comp, minlength=tiles * R).view(tiles, R)
            lstart = torch.cumsum(cnt, 1) - cnt                       # tile-local digit starts
            tpre = torch.cumsum(cnt, 0) - cnt                         # earlier tiles, per digit
            tot = cnt.sum(0)
            gbase = torch.cumsum(tot, 0) - tot
            table = (gbase[None, :] + tpre - lstart).to(torch.int32).view(torch.uint32).contiguous()
            del pos, comp, srt, perm, cnt, lstart, tpre
            ts = []
            for _ in range(a.rounds):
                ticket.zero_()
                torch.cuda.synchronize()
                e0.record()
                assert L.lab2_replay(b, it, rb, x8, P(pre), P(out), P(table), ctypes.c_uint32(n), 0,
                                     P(ticket), sp) == 0
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ref = torch.sort(k64 & (R - 1), stable=True)[1]
            ok = torch.equal(out.view(torch.int32).to(torch.int64) & 0xFFFFFFFF, k64[ref])
            med = statistics.median(ts)
            print(f"replay {e:12s} median {med:8.4f} ms  min {min(ts):8.4f}  {n * 8 / med / 1e6:8.1f} GB/s "
                  f"({n * 8 / med / 8e9:.3f} of 8 TB/s)  output {'= one stable digit pass' if ok else 'WRONG'}",
                  flush=True)
            del pre, table
    if a.emu16:
        keys, out, _ = bufs[32]
        for e in a.emu16.split(","):
            b, it = (int(x) for x in e.split(":"))
            ts = []
            for _ in range(a.rounds):
                e0.record()
                assert L.lab2_emu16(b, it, 8, P(keys), P(out), ctypes.c_uint32(n), sp) == 0
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            med = statistics.median(ts)
            print(f"emu16 {e:12s} 8 passes median {med:8.4f} ms = {med / 8 * 1e3:7.2f} us per pass  "
                  f"{n * 8 * 8 / med / 1e6:8.1f} GB/s", flush=True)
    if a.emu_pairs:
        # 2^28-pair C3 shape unless --n says otherwise: SoA (two arrays) vs AoS (one 8-B array)
        npair = n
        src = torch.empty(2 * npair, dtype=torch.uint32, device=dev)
        grs.fill_splitmix(src, 77)
        dst = torch.empty_like(src)
        for e in a.emu_pairs.split(","):
            b, it, aos, lds = (int(x) for x in e.split(":"))
            ts = []
            for _ in range(a.rounds):
                e0.record()
                assert L.lab2_emu_pairs(b, it, aos, lds, P(src), vp(src.data_ptr() + 4 * npair), P(dst),
                                        vp(dst.data_ptr() + 4 * npair), ctypes.c_uint32(npair), sp) == 0
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            med = statistics.median(ts)
            print(f"emu_pairs {e:20s} median {med:8.4f} ms  {npair * 16 / med / 1e6:8.1f} GB/s", flush=True)
    if a.check:
        for v in variants:
            kb, pairs = v[1], v[2]
            keys, out, hist = bufs[kb]
            st.zero_()
            ticket.zero_()
            err.zero_()
            err[63] = a.rot
            run(v)
            torch.cuda.synchronize()
            k64 = keys.view(torch.int32 if kb == 32 else torch.int64).to(torch.int64)
            _, idx = torch.sort(k64 & (15 if v[0] in ("r4", "r6") else 255), stable=True)
            o64 = out.view(torch.int32 if kb == 32 else torch.int64).to(torch.int64)
            ok = torch.equal(o64, k64[idx])
            okv = (not pairs) or torch.equal(vout.view(torch.int32).to(torch.int64) & 0xFFFFFFFF, idx)
            print(f"check {v}: keys {'OK' if ok else 'MISMATCH'} vals {'OK' if okv else 'MISMATCH'} "
                  f"err={int(err[0].item())}", flush=True)
    for v in variants:
        kb, pairs = v[1], v[2]
        alg = n * 2 * (kb // 8 + (4 if pairs else 0))
        med, mn = statistics.median(times[v]), min(times[v])
        print(f"{':'.join(str(x) for x in v):28s} median {med:8.4f} ms  min {mn:8.4f}  "
              f"{alg / med / 1e6:8.1f} GB/s", flush=True)
    for v in variants:
        stamped = v[0] in ("v4", "v6", "r4", "r6") and v[6] & 8
        if not stamped:
            continue
        err.zero_()
        err[63] = a.rot
        st.zero_()
        ticket.zero_()
        run(v)
        torch.cuda.synchronize()
        tiles = (n + v[3] * v[4] - 1) // (v[3] * v[4])
        a_ = err[64:64 + 12 * tiles].view(torch.int32).cpu().numpy().reshape(tiles, 12).astype("float64")
        m = a_[:, :6].mean(0)
        print(f"   ticket known at {a_[:, 6].mean():.0f} cycles (p90 {np.percentile(a_[:, 6], 90):.0f})", flush=True)
        d = np.diff(np.concatenate([[0.0], m]))
        names = ["ticket+load+rank", "zero+B1", "colscan+publish+scan+B2", "fold+issue+B3",
                 "reorder+lookback+B4", "store+drain"]
        print(f"stamps {v}: " + ", ".join(f"{nm}={x:.0f}" for nm, x in zip(names, d))
              + f"  total={m[5]:.0f}  (p90 reorder+lb {np.percentile(a_[:, 4] - a_[:, 3], 90):.0f})",
              flush=True)
        r_end, lb_end = a_[:, 8], a_[:, 9]
        print(f"   reorder ends at {r_end.mean():.0f}, look-back (thread 0) at {lb_end.mean():.0f} "
              f"cycles: look-back wait after the reorder {(lb_end - r_end).mean():.0f} "
              f"(p90 {np.percentile(lb_end - r_end, 90):.0f})", flush=True)
        # per CU: its tiles in start order, and the gap from one tile's drained stores (every
        # wave) to the next tile's first instruction on the same CU
        raw = err[64:64 + 12 * tiles].view(torch.int32).cpu().numpy().reshape(tiles, 12)
        # absolute (s_memtime >> 8) words: unwrap the 32-bit values around their median
        ref = int(np.median(raw[:, 7].astype(np.uint32)))
        unwrap = lambda x: ((x.astype(np.uint32).astype(np.int64) - ref + (1 << 31)) % (1 << 32)) - (1 << 31)  # noqa: E731
        st_ = unwrap(raw[:, 7])
        en_ = unwrap(raw[:, 10])
        cu = raw[:, 11].astype(np.uint32)
        gaps, busy, cus = [], [], 0
        for c in np.unique(cu):
            idx = np.where(cu == c)[0]
            o = idx[np.argsort(st_[idx])]
            s_, e_ = st_[o], en_[o]
            cus += 1
            if len(o) > 1:
                gaps.extend(((s_[1:] - e_[:-1]) * 256).tolist())
            busy.append(((e_ - s_).sum(), e_.max() - s_.min()))
        g = np.array(gaps, dtype=np.float64)
        b = np.array(busy, dtype=np.float64)
        print(f"   tiles={tiles} on {cus} CUs; per-CU gap between tiles mean {g.mean():.0f} "
              f"p50 {np.median(g):.0f} p90 {np.percentile(g, 90):.0f} cycles; CU busy "
              f"{b[:, 0].sum() / b[:, 1].sum():.3f} of its span; tile mean "
              f"{(en_ - st_).mean() * 256:.0f}", flush=True)
        if v[0] in ("v6", "r6"):   # persistent: every workgroup's entry and exit
            grid = min(tiles, v[7] if v[7] > 0 else 256)
            wg = err[64 + 12 * tiles:64 + 12 * tiles + 2 * grid].view(torch.int32).cpu().numpy()
            wg = unwrap(wg).reshape(grid, 2) * 256
            t0, t1 = wg[:, 0].min(), wg[:, 1].max()
            print(f"   workgroups: entry spread {wg[:, 0].max() - t0:.0f}, exit spread "
                  f"{t1 - wg[:, 1].min():.0f}, kernel span {t1 - t0:.0f} cycles; first tile "
                  f"starts {(st_ * 256).min() - t0:.0f} after the first entry, mean wg "
                  f"{(wg[:, 1] - wg[:, 0]).mean():.0f} (tiles {b[:, 0].sum() * 256 / cus:.0f} per CU)",
                  flush=True)


if __name__ == "__main__":
    main()
