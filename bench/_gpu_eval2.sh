# PPE ROI ops numerics + ResNet-50 inference throughput (ops vs stock)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ppe.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_ppe.log 2>&1 &&
timeout -k 10 200 python bench/resnet50.py --infer --steps 30 --warmup 5 > gpurun_out/r50_infer_ops.log 2>&1 &&
timeout -k 10 200 python bench/resnet50.py --infer --path torch --steps 30 --warmup 5 > gpurun_out/r50_infer_torch.log 2>&1 &&
timeout -k 10 200 python bench/resnet50.py --infer --fp8 --steps 30 --warmup 5 > gpurun_out/r50_infer_fp8.log 2>&1
rc=$?
grep -E "passed|failed|Error" gpurun_out/pytest_ppe.log | tail -5
for f in r50_infer_ops r50_infer_torch r50_infer_fp8; do echo "== $f"; grep metric gpurun_out/$f.log | cut -c1-260; done
exit $rc
