"""Generate the committed golden fixtures under tests/golden/ (run once, in the build
container where the reference is mounted at /root/reference; the GPU box never reads it).

Fixtures are DATA lifted from the reference's own files, plus digests computed by the
committed oracle:

  prefix_scan_xlsx.json   PrefixScan.xlsx sheet1 (reference repo root): the hand-traced
                          32-element Blelloch scan — input bits (row 3), up-sweep state after
                          "set last item to 0" (row 50), exclusive-scan result (row 102).
  main_cpp_16key.json     the commented debug input of main.cpp:128-143 (a permutation of
                          0..15) with its sorted output and stable permutation.
  digests.json            SHA-256 of the expected sorted keys (and stable permutation) of the
                          BASELINE.json configs at their seeds (SURVEY.md §8d generator).

usage: python tests/golden/make_golden.py [--large] [--only NAME]
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys
import zipfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402

REF = "/root/reference"


def xlsx_rows(path, wanted):
    z = zipfile.ZipFile(path)
    s = z.read("xl/worksheets/sheet1.xml").decode()
    rows = dict(re.findall(r'<row r="(\d+)"[^>]*>(.*?)</row>', s))
    out = {}
    for r in wanted:
        cells = re.findall(r'<c r="([A-Z]+)\d+"[^>]*>(?:<f[^>]*>[^<]*</f>|<f[^>]*/>)?<v>([^<]*)</v></c>',
                           rows[str(r)])
        # columns B..AG hold indices 0..31 (column A is a label)
        vals = {}
        for col, v in cells:
            if col == "A":
                continue
            ci = 0
            for ch in col:
                ci = ci * 26 + (ord(ch) - 64)
            vals[ci - 2] = int(float(v))
        out[r] = [vals[i] for i in range(32)]
    return out


def main_cpp_16key(path):
    src = open(path, encoding="latin-1").read()
    pairs = re.findall(r"//demoData\[(\d+)\]\._value = (\d+);", src)
    vals = [0] * len(pairs)
    for i, v in pairs:
        vals[int(i)] = int(v)
    return vals


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


CONFIGS = {
    # name: (config_id, n, key_bits, pairs)
    "c1_64k_u32": (1, 1 << 16, 32, False),
    "c1_64k_u32_pairs": (1, 1 << 16, 32, True),
    "c2_16m_u32": (2, 1 << 24, 32, False),
    "c3_256m_u32_pairs": (3, 1 << 28, 32, True),
    "c4_1b_u32": (4, 1 << 30, 32, False),
    "c5_256m_u64": (5, 1 << 28, 64, False),
    # the north star's own 1-GPU config (BASELINE.json north_star: 256 M uniform-random
    # uint32 keys, keys only); config id 6 = its own seed (oracle.config_seed: bit 48 set, so
    # its keys are not C3's multiset)
    "ns_256m_u32": (6, 1 << 28, 32, False),
}
SMALL = ("c1_64k_u32", "c1_64k_u32_pairs", "c2_16m_u32")


def digest(name):
    cid, n, kb, pairs = CONFIGS[name]
    seed = oracle.config_seed(cid)
    keys = oracle.splitmix_keys(n, kb, seed)
    rec = {"config_id": cid, "n": n, "key_bits": kb, "seed": seed, "pairs": pairs}
    if pairs:
        perm = oracle.stable_argsort(keys)
        rec["sha256_perm"] = sha(perm)
        keys = keys[perm]
        del perm
    else:
        keys.sort()
    rec["sha256_keys"] = sha(keys)
    rec["head"] = [int(x) for x in keys[:4]]
    rec["tail"] = [int(x) for x in keys[-4:]]
    return rec


def main():
    large = "--large" in sys.argv
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    rows = xlsx_rows(os.path.join(REF, "PrefixScan.xlsx"), [2, 3, 50, 102])
    assert rows[2] == list(range(32)), rows[2]
    scan = {"source": "PrefixScan.xlsx sheet1 rows 3 (input), 50 (after set-last-to-0), 102 (result)",
            "input": rows[3], "upsweep_after_zero": rows[50], "exclusive_scan": rows[102],
            "total": sum(rows[3])}
    json.dump(scan, open(os.path.join(HERE, "prefix_scan_xlsx.json"), "w"), indent=1)

    k16 = main_cpp_16key(os.path.join(REF, "main.cpp"))
    srt, perm = oracle.ref_parallel_sort(k16)
    json.dump({"source": "main.cpp:128-143 (commented debug input)", "input": k16,
               "sorted": srt.tolist(), "perm": perm.tolist()},
              open(os.path.join(HERE, "main_cpp_16key.json"), "w"), indent=1)

    path = os.path.join(HERE, "digests.json")
    digests = json.load(open(path)) if os.path.exists(path) else {}
    for name in CONFIGS:
        if (only is None and (name in SMALL or large)) or name == only:
            print("digest", name, flush=True)
            digests[name] = digest(name)
    json.dump(digests, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
