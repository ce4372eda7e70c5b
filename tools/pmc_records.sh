#!/bin/bash
# PMC write / fetch bytes of the C3 pass kernels with and without record passes (--opt records).
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 0 2; do
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmcrec_${r}_${c} -o p --output-format csv -- python3 bench.py --opt records=$r --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcrec_${r}_${c}.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import csv, glob, statistics
for r in (0, 2):
    for c in ("WRITE_SIZE", "FETCH_SIZE"):
        vals = []
        for path in glob.glob(f"gpurun_out/pmcrec_{r}_{c}/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(path)):
                if "grs_onesweep_v4" in row["Kernel_Name"] and row["Counter_Name"] == c:
                    vals.append(float(row["Counter_Value"]) * 1024)
        print(f"records={r} {c}: {len(vals)} launches, mean {statistics.mean(vals)/1e9:.4f} GB raw per launch"
              f" (algorithmic {2**28 * 8 / 1e9:.4f} GB each way)")
PY
