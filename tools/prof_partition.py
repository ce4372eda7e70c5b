"""rocprofv3 target: grs_partition of 2^27 u32 keys into 8 buckets (tools/bench_extras.partition)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_extras  # noqa: E402

bench_extras.partition(1 << 27, 8)
