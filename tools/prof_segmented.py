"""Segmented sorts of 2^26 u32 pairs for a kernel trace: python tools/prof_segmented.py SEGS [REPS]
(SEGS: a number of equal segments, or "ragged64"); rocprofv3 --kernel-trace --stats -- python ..."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpuradixsort_amd as grs  # noqa: E402


def main():
    segs = sys.argv[1] if len(sys.argv) > 1 else "64"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    m = 1 << 26
    dev = torch.device("cuda", 0)
    s = grs.RadixSorter(m, key_bits=32, pairs=True)
    k0 = torch.empty(m, dtype=torch.int32, device=dev)
    grs.fill_splitmix(k0, 2)
    k = torch.empty_like(k0)
    v = torch.empty_like(k0)
    if segs.startswith("ragged"):
        g = int(segs[6:])
        cuts = np.sort(np.random.default_rng(3).integers(0, m + 1, g - 1))
        off = torch.from_numpy(np.concatenate([[0], cuts, [m]]).astype(np.int32)).to(dev)
    else:
        g = int(segs)
        off = torch.arange(0, m + 1, m // g, dtype=torch.int32, device=dev)
    for _ in range(reps):
        k.copy_(k0)
        s.sort_segmented(k, off, v)
    torch.cuda.synchronize()
    s.check_error()
    print("ok", segs, flush=True)


if __name__ == "__main__":
    main()
