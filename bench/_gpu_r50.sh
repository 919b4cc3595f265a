# ResNet-50 synthetic 224x224 DDP throughput on 1 MI355X: stock path vs ops path (bf16, fp8) + ops tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_torch.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 --path ops > gpurun_out/r50_ops.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 --path ops --fp8 > gpurun_out/r50_ops_fp8.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_ops.log
for f in r50_torch r50_ops r50_ops_fp8; do tail -1 gpurun_out/$f.log | cut -c1-200; done
exit $rc
