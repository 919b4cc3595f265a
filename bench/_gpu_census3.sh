set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/r50_gemm_census.py --batch 256 > gpurun_out/census256.log 2>&1 &&
DCA_OPS_GLDS_NARROW=1 timeout -k 10 300 python bench/r50_gemm_census.py --batch 256 > gpurun_out/census256_gn.log 2>&1
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
a=load('gpurun_out/census256.log'); b=load('gpurun_out/census256_gn.log')
for k in sorted(a, key=lambda k: -a[k] if k!="total" else 0):
    if k!="total" and abs(b.get(k,0)/a[k]-1) > 0.04: print(k, a[k], b.get(k), round(b.get(k,0)/a[k],2))
print("total", a["total"], b["total"])
PY
exit $rc
