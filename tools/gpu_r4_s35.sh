# round 4, session 35: the partition histogram with host splitters kept in SGPRs (FROM_DEV
# false): kernel stats, partition timing, then the GPU suite, smoke and the bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4s35_prof -o run --output-format csv -- python3 tools/prof_partition.py > gpurun_out/r4s35_prof.txt 2>&1 || exit $?
for r in 1 2 3; do timeout -k 10 120 python -u tools/prof_partition.py > gpurun_out/r4s35_part$r.txt 2>&1 || exit $?; done
bash tools/gpu_r4_final.sh r4i a
