"""CPU checks of bench.py's host arithmetic: the workloads it measures are BASELINE.json's
configs, and the moved-bytes figure the bench line reports beside SURVEY §8d's credited
whole-sort fraction (DESIGN.md "Current state") is the schedule's algorithmic traffic.
No GPU, no libgrs: bench.py is imported only for its tables and pure functions."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_configs_match_baseline():
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert bench.METRIC == base["metric"]
    # configs[1..4] of BASELINE.json (configs[0] is the reference's host std::sort case, the
    # CPU baseline leg) and the north star's own 1-GPU workload
    want = {
        "c2": (2, 1 << 24, 32, False, 4),   # 16M u32, 4-bit-digit LSD
        "c3": (3, 1 << 28, 32, True, 8),    # 256M u32 key + u32 payload, stable
        "c4": (4, 1 << 30, 32, False, 8),   # 1B (2^30) u32 keys, sharded at N > 1
        "c5": (5, 1 << 28, 64, False, 8),   # 256M u64 keys, 8 x 8-bit digits
        "ns": (6, 1 << 28, 32, False, 8),   # north star: 256M uniform u32 keys
    }
    assert {k: v[:5] for k, v in bench.CONFIGS.items()} == want
    assert "16M" in base["configs"][1] and "4-bit" in base["configs"][1]
    assert "256M" in base["configs"][2] and "payload" in base["configs"][2]
    assert "1B" in base["configs"][3] and "8" in base["configs"][3]
    assert "256M" in base["configs"][4] and "uint64" in base["configs"][4]


def test_parse_defaults(monkeypatch):
    # the driver's no-flag run: N = 1, the C4 headline, a K / W that finish in minutes
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.gpus, a.config, a.dist, a.n) == (1, "c4", "uniform", 0)
    assert 1 <= a.steps <= 100 and 0 <= a.warmup <= 10


@pytest.mark.parametrize("n,kb,pairs,want", [
    # the values the round-6 bench lines carry (profiles/r06/final_s31/bench.txt):
    # C4 2^30 u32: 3 sweeps x (read + write) + H2's 1/32 sample + the 4-MB sample
    (1 << 30, 32, False, 3 * 2 * (1 << 30) * 4 + ((1 << 30) * 4 >> 5) + (4 << 20)),
    # ns 2^28 u32: H2 reads 1/8 of the keys
    (1 << 28, 32, False, 3 * 2 * (1 << 28) * 4 + ((1 << 28) * 4 >> 3) + (4 << 20)),
    # C3 2^28 pairs: 8-byte elements through the sweeps, H2 reads keys only
    (1 << 28, 32, True, 3 * 2 * (1 << 28) * 8 + ((1 << 28) * 4 >> 3) + (4 << 20)),
    # C5 2^28 u64
    (1 << 28, 64, False, 3 * 2 * (1 << 28) * 8 + ((1 << 28) * 8 >> 3) + (4 << 20)),
])
def test_moved_bytes_msd(n, kb, pairs, want):
    assert bench.moved_bytes(n, kb, pairs, 8, "msd") == want


def test_moved_bytes_pins_bench_line():
    assert bench.moved_bytes(1 << 30, 32, False, 8, "msd") == 25908215808
    assert bench.moved_bytes(1 << 28, 32, False, 8, "msd") == 6580862976


def test_moved_bytes_lsd():
    n = 1 << 24
    # C2: the up-front histogram's read + 8 passes of read + write, even count: no copy-back
    assert bench.moved_bytes(n, 32, False, 4, "lsd") == n * 4 + 8 * 2 * n * 4
    # 8-bit digits: 4 passes
    assert bench.moved_bytes(n, 32, False, 8, "lsd") == n * 4 + 4 * 2 * n * 4
    # an odd pass count (e.g. 11-bit digits over 32 bits: 3 passes) adds the copy-back
    assert bench.moved_bytes(n, 32, True, 11, "lsd") == n * 4 + 3 * 2 * n * 8 + 2 * n * 8


def test_moved_never_above_credited_for_msd():
    # the MSD schedule moves fewer bytes than SURVEY §8d credits (4 passes for u32, 8 for u64):
    # the credited fraction may pass 1, the moved one is the physical figure
    for n, kb in ((1 << 28, 32), (1 << 30, 32), (1 << 28, 64)):
        credited = n * 2 * (kb // 8) * (kb // 8)
        assert bench.moved_bytes(n, kb, False, 8, "msd") < credited
