# Round 6: Phi-3 IT (micro-batch 16) with the SwiGLU backward also writing dgu^T for a TN gate_up weight gradient (LLMT_SWIGLU_DY_T=1) vs not (default at I = 8192),
# alternating runs on one box
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r6_swiglu_dyt_it_ab.jsonl
for i in 1 2 3; do
  for v in 0 1; do
    LLMT_SWIGLU_DY_T=$v timeout -k 10 400 python bench.py --workload it --steps 8 --warmup 3 > gpurun_out/dyt_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/dyt_$v.log | sed "s/^{/{\"arm\": \"it swiglu_dy_t=$v\", /" >> gpurun_out/r6_swiglu_dyt_it_ab.jsonl
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r6_swiglu_dyt_it_ab.jsonl"):
    d = json.loads(l); print(d["arm"], d["value"], d["ms_per_step"], d["peak_mem_gib"])
PY
