# Full GPU tier + smoke + 1-GPU bench + 2-rank shared-GPU bench rehearsal + ResNet-50 paths
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 --path ops > gpurun_out/r50_ops.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 --path ops --fp8 > gpurun_out/r50_ops_fp8.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
grep -E "FAIL" gpurun_out/pytest_gpu.log | head
tail -1 gpurun_out/smoke.log
tail -1 gpurun_out/bench.log | cut -c1-200
for f in r50_ops r50_ops_fp8; do tail -1 gpurun_out/$f.log | cut -c1-160; done
exit $rc
