# Round 6: Llama PT with AdamW on its own stream overlapping the next forward (LLMT_OVERLAP_STEP=1, default) vs on the compute stream (0),
# alternating runs on one box
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r6_overlap_step_ab.jsonl
for i in 1 2 3; do
  for v in 1 0; do
    LLMT_OVERLAP_STEP=$v timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/ovl_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/ovl_$v.log | sed "s/^{/{\"arm\": \"pt overlap_step=$v\", /" >> gpurun_out/r6_overlap_step_ab.jsonl
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r6_overlap_step_ab.jsonl"):
    d = json.loads(l); print(d["arm"], d["value"], d["ms_per_step"], d["peak_mem_gib"])
PY
