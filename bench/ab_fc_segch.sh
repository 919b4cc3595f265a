set -e
for cfg in "1 64" "0 64" "1 256" "0 256"; do
  set -- $cfg
  DCA_PKS_FC_IN_STEP=$1 DCA_PKS_SEG_CH=$2 timeout -k 10 100 python -u bench.py --steps 600 --warmup 60 --no-fp32 > gpurun_out/ab_$1_$2.log 2>&1
done
