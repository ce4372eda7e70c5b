"""Driver of tools/smem_probe.hip: per mode, which reader blocks saw the other XCD's store
through scalar loads, after how many polls and how many microseconds."""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "libsmem_probe.so"))
flag = torch.zeros(64, dtype=torch.int32, device="cuda")
out = torch.zeros(4 * 64 + 64, dtype=torch.int32, device="cuda")
for mode, name in ((2, "vector sc1 loads"), (0, "scalar glc loads"), (1, "plain scalar load, then glc"),
                   (3, "64-word row, scalar x16 + writelane")):
    for rep in range(3):
        out.zero_()
        rc = L.smem_probe_run(ctypes.c_void_p(flag.data_ptr()), ctypes.c_void_p(out.data_ptr()), mode, 32,
                              ctypes.c_uint32(200000))
        assert rc == 0, rc
        o = out.view(-1, 4).cpu().numpy()
        wx = int(o[0, 0])
        r = o[1:32]
        seen = int((r[:, 1] == 1).sum())
        cross = r[r[:, 0] != wx]
        lat = cross[:, 3] / 100.0   # us since the block started (the store lands at ~20 us)
        print(f"{name:30s} rep {rep}: writer xcc {wx}; readers seeing the store {seen}/31; "
              f"other-XCC readers {len(cross)}: polls max {int(cross[:, 2].max()) if len(cross) else -1}, "
              f"done at {lat.min() if len(cross) else -1:.1f}-{lat.max() if len(cross) else -1:.1f} us"
              + (f"; cycles per row poll {int(out[4 * 64 + 1:4 * 64 + 32].float().median().item())}"
                 if mode == 3 else ""), flush=True)
