# Round 6: Phi-3 IT (micro-batch 16) with 8192- vs 16384-row loss chunks (lm_head GEMM + CE per chunk),
# alternating runs on one box
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r6_losschunk_it_ab.jsonl
for i in 1 2 3; do
  for v in 8192 16384; do
    timeout -k 10 400 python bench.py --workload it --loss-chunk $v --steps 8 --warmup 3 > gpurun_out/lc_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/lc_$v.log | sed "s/^{/{\"arm\": \"it loss_chunk=$v\", /" >> gpurun_out/r6_losschunk_it_ab.jsonl
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r6_losschunk_it_ab.jsonl"):
    d = json.loads(l); print(d["arm"], d["value"], d["ms_per_step"], d["peak_mem_gib"])
PY
