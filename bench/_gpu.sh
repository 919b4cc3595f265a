# One gpurun call: persistent-engine numerics, phase stamps, bench.  Every GPU step is time-boxed and chained
# with && so nothing else starts on the GPU after a failure.
set -o pipefail
timeout -k 10 300 python bench/engine_diag.py --batches 32,16 --persistent 1 > gpurun_out/diag_pk.log 2>&1 &&
DCA_ENGINE_VARIANT=stamps timeout -k 10 200 python bench/stamps.py bf16 persistent > gpurun_out/stamps_pk.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 500 --warmup 50 > gpurun_out/bench_pk.log 2>&1
rc=$?
grep -E "summary|FAILED" gpurun_out/diag_pk.log
grep -v amdgpu gpurun_out/stamps_pk.log | tr '\n' ' '
tail -1 gpurun_out/bench_pk.log | cut -c1-200
exit $rc
