"""Driver of tools/digit_probe.hip: time the partition's bucket histogram with the splitter digit
computed three ways (64-bit compares, 32-bit subtract/borrow, keys-only 32-bit compares) over
2^27 u32 keys, and check every mode's counts against mode 0's."""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "libdigit_probe.so"))
dev = torch.device("cuda", 0)
n = 1 << 27
g = torch.Generator(device=dev)
g.manual_seed(3)
keys = torch.randint(-(1 << 31), (1 << 31) - 1, (n,), dtype=torch.int32, device=dev, generator=g)
cus = torch.cuda.get_device_properties(0).multi_processor_count
vp = ctypes.c_void_p
sp = (ctypes.c_uint32 * 7)(*[(j * (1 << 32)) // 8 for j in range(1, 8)])
for th_name, thv in (("zero", [0] * 7), ("nonzero", [(j * 977) % 50000 for j in range(1, 8)])):
    th = (ctypes.c_uint32 * 7)(*thv)
    ref = None
    for mode in (0, 1, 2):
        if mode == 2 and th_name != "zero":
            continue
        hist = torch.zeros(16, dtype=torch.int32, device=dev)
        per_cu = L.digit_probe_run(mode, vp(keys.data_ptr()), n, sp, th, 7, vp(hist.data_ptr()), cus)
        assert per_cu > 0, per_cu
        torch.cuda.synchronize()
        h = hist.cpu()
        if ref is None:
            ref = h
        ok = bool(torch.equal(h, ref)) and int(h.sum()) == n
        ts = []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            L.digit_probe_run(mode, vp(keys.data_ptr()), n, sp, th, 7, vp(hist.data_ptr()), cus)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        ms = ts[len(ts) // 2]
        print(f"thresholds {th_name:8s} mode {mode}: {ms * 1e3:7.1f} us  {n * 4 / ms / 1e6:7.1f} GB/s  "
              f"blocks/CU {per_cu}  counts match mode 0: {ok}", flush=True)
