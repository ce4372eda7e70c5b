#!/bin/bash
# One GPU lab session = one plan file: every non-comment line is "NAME SECONDS COMMAND ...".
# Each step runs under its own time limit, its output goes to gpurun_out/NAME.txt, and the
# session stops at the first step that times out, crashes or faults the GPU (no retries).
#   gpurun --timeout T -- bash tools/run_steps.sh tools/plans/r5_s1.txt
# Builds the lab libraries a plan names with "make -C tools TARGET" steps of its own.
set -u
plan=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
while read -r name secs cmd; do
  [[ -z "$name" || "$name" == \#* ]] && continue
  echo "== $name ($secs s) $(date +%T)" >&2
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.txt" 2>&1
  rc=$?
  echo "== $name rc=$rc" >&2
  tail -4 "gpurun_out/$name.txt" | cut -c1-240 >&2
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  if grep -q "illegal memory access\|hipErrorIllegalAddress\|Memory access fault" "gpurun_out/$name.txt"; then
    echo "GPU fault in $name: stopping" >&2
    exit 99
  fi
  if [ $rc -ne 0 ]; then echo "step $name failed (rc=$rc): stopping" >&2; exit $rc; fi
done < "$plan"
exit 0
