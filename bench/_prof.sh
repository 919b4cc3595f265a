# rocprofv3 kernel trace + stats of the 1-GPU bench (kernel durations, launch gaps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_pk -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/prof_pk.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
find gpurun_out/prof_pk -name "*.csv" | head -20
exit $rc
