set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/r50_gemm_census.py --batch 256 > gpurun_out/census_a.log 2>&1 &&
DCA_OPS_REG_SINGLE_NK=9 timeout -k 10 300 python bench/r50_gemm_census.py --batch 256 > gpurun_out/census_b.log 2>&1 &&
DCA_OPS_REG_SINGLE_NK=100 timeout -k 10 300 python bench/r50_gemm_census.py --batch 256 > gpurun_out/census_c.log 2>&1
rc=$?
python3 - <<'PY'
import json
def load(p):
    d={}
    for l in open(p):
        if l.startswith('{"kind"'):
            r=json.loads(l); d[(r["kind"],r["M"],r["N"],r["K"])]=r["us"]
        elif l.startswith('{"total'): d["total"]=json.loads(l)["total_gemm_us"]
    return d
a=load('gpurun_out/census_a.log'); b=load('gpurun_out/census_b.log'); c=load('gpurun_out/census_c.log')
for k in sorted(a, key=lambda k: -a[k] if k!="total" else 0):
    if k!="total" and (abs(b.get(k,0)/a[k]-1) > 0.05 or abs(c.get(k,0)/a[k]-1) > 0.05): print(k, a[k], round(b.get(k,0)/a[k],2), round(c.get(k,0)/a[k],2))
print("total", a["total"], b["total"], c["total"])
PY
exit $rc
