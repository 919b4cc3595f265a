set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bf16 -o run -- python3 $GRAFT_REPO_ROOT/bench/resnet50.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_bf16.log 2>&1 &&
DCA_FP8_MIN_CIN=1024 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fp8 -o run -- python3 $GRAFT_REPO_ROOT/bench/resnet50.py --steps 4 --warmup 2 --fp8 > $GRAFT_REPO_ROOT/gpurun_out/prof_fp8.log 2>&1
