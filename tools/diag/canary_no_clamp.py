"""The guard bands catch a region run written past the second buffer.

  GRS_DIAG_LIB=tools/diag/libgrs_noclamp.so python tools/diag/canary_no_clamp.py   # expect bad > 0
  python tools/diag/canary_no_clamp.py                                             # expect bad == 0

P1 (grs_onesweep_region) writes top-byte run d into a region of R_d = sampled share x 9/8 + 4096
keys; the regions fill the second buffer but for its last 1024 elements.  Here 7120 keys of top
byte 0xFF sit where the sample never looks, so digit 255's region is 4096 keys and its run
outgrows it by ~3000 keys: without the run clamp (libgrs_noclamp.so, -DGRS_TEST_NO_CLAMP) ~2000
keys land past the buffer's end -- inside its 16-KB guard band (and, for u32 pairs, the band
between alt's keys and payload), never further, so the scratch build faults nothing.  The
product build clamps the run and reports 0; both builds redo P1 exactly and sort correctly."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import gpuradixsort_amd as grs  # noqa: E402

if os.environ.get("GRS_DIAG_LIB"):
    grs._lib.LIB_PATH = os.environ["GRS_DIAG_LIB"]

SAMPLE_CHUNKS = 16384   # GRS_MSD_SAMPLE_CHUNKS


def p1_spill_keys(n, extra, rng):
    keys = rng.integers(0, 0xFF000000, n, dtype=np.uint64).astype(np.uint32)   # top bytes 0..254
    c = np.arange(SAMPLE_CHUNKS, dtype=np.uint64)
    starts = (c * np.uint64(n - 64) // np.uint64(SAMPLE_CHUNKS - 1)).astype(np.int64)
    seen = np.zeros(n, bool)
    seen[(starts[:, None] + np.arange(64)[None, :]).ravel()] = True
    hot = rng.choice(np.flatnonzero(~seen), 4096 + extra, replace=False)
    keys[hot] = np.uint32(0xFF000000) | rng.integers(0, 1 << 24, hot.size, dtype=np.uint32)
    return keys


def main():
    n = 1 << 22
    rng = np.random.default_rng(4243)
    spill = p1_spill_keys(n, 3024, rng)
    uniform = rng.integers(0, 1 << 32, n, dtype=np.uint32)
    dev = torch.device("cuda", 0)
    out = {"lib": grs._lib.LIB_PATH}
    for pairs in (False, True):
        s = grs.RadixSorter(n, key_bits=32, pairs=pairs, radix_bits=8)
        s.set_option("msd", "always")
        for name, keys in (("uniform", uniform), ("p1_spill", spill)):
            k = torch.from_numpy(keys).to(dev)
            v = torch.arange(n, dtype=torch.int32, device=dev).view(torch.uint32) if pairs else None
            s.sort(k, v)
            torch.cuda.synchronize()
            bad = s.check_guards()
            ok = bool(np.array_equal(k.cpu().numpy(), np.sort(keys)))
            out[f"{name}{'_pairs' if pairs else ''}"] = {"bad_guard_words": bad, "sorted_ok": ok}
            print(name, "pairs" if pairs else "keys", "bad guard words", bad, "sorted", ok, flush=True)
            del k, v
        s.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
