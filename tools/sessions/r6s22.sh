cd $GRAFT_REPO_ROOT
bash tools/run_steps.sh tools/plans/r6_s22.txt
