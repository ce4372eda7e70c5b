"""How often the MSD sort's sampled P2 regions overflow on uniform input (grs_debug_msd_flags):
a spill sends P2 through the exact redo (correct, ~a P2 pass slower).  For each size and key
type, `--seeds` sorts of splitmix64 keys with different seeds; prints one JSON line per case
with the number of sorts that took the exact P2 and that redid P1.

python tools/msd_spill_rate.py [--seeds 8]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpuradixsort_amd as grs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cases = [((1 << 26) + 5, 32, False), (1 << 27, 32, False), (1 << 28, 32, False), (1 << 30, 32, False),
             (1 << 28, 32, True), (1 << 28, 64, False)]
    for n, kb, pairs in cases:
        k = torch.empty(n, dtype=torch.uint32 if kb == 32 else torch.uint64, device=dev)
        v = torch.empty(n, dtype=torch.uint32, device=dev) if pairs else None
        s = grs.RadixSorter(n, key_bits=kb, pairs=pairs)
        exact = redo = bad = 0
        for seed in range(a.seeds):
            grs.fill_splitmix(k, 0x5EED0000 + 131 * seed + n)
            if pairs:
                grs.iota_u32(v)
            s.sort(k, v)
            s.check_error()
            f = s.msd_flags()
            exact += f["p2_exact"]
            redo += f["p1_redo"]
            bad += grs.count_inversions(k) != 0
        print(json.dumps({"n": n, "key_bits": kb, "pairs": pairs, "sorts": a.seeds, "p2_exact": exact,
                          "p1_redo": redo, "unsorted": bad}), flush=True)
        s.close()
        del k, v
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
