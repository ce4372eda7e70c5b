# round 4, session 23: the tail of the ns pass -- per-key pass time at 2^28 (28.45 tiles per CU)
# against 28 x 256 tiles exactly (264,241,152 keys)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 268435456 264241152 268435456 264241152; do
  timeout -k 10 200 python -u bench.py --config ns --n $n --steps 20 --no-cpu-baseline --no-traffic > gpurun_out/r4s23_ns_$n.txt 2>&1 || exit $?
  python3 -c "
import json,sys
l=[x for x in open('gpurun_out/r4s23_ns_$n.txt') if x.startswith('{')][-1]; d=json.loads(l)
pm=d['phases_ms']['pass_mean']; print($n, 'pass_mean', pm, 'ns/key', pm*1e6/$n, 'value', d['value'])"
done
