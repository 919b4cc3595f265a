# ops layer: kernel tests + ResNet-50 ops-path throughput (bf16 / fp8, two batch sizes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 --path ops --batch 64 > gpurun_out/r50_b64.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 6 --warmup 2 --path ops --batch 256 > gpurun_out/r50_b256.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 6 --warmup 2 --path ops --batch 256 --fp8 > gpurun_out/r50_b256_fp8.log 2>&1
rc=$?
grep -E "passed|failed|Error|error" gpurun_out/pytest_ops.log | tail -5
for f in r50_b64 r50_b256 r50_b256_fp8; do tail -1 gpurun_out/$f.log | cut -c1-170; done
exit $rc
