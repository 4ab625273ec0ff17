# Round 6 (Phi-3 IT): a layout table timed under longer interleaved rounds (LLMT_GEMM_LAYOUT_ROUNDS=10, after a
# heating run), then in-step A/B of that table against the shipped one, alternating runs on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload it --steps 3 --warmup 2 > gpurun_out/sus_heat.log 2>&1 || exit $?
LLMT_GEMM_LAYOUTS=timed LLMT_GEMM_LAYOUT_ROUNDS=10 LLMT_GEMM_LAYOUT_DUMP=gpurun_out/r6_layouts_it_sustained.json \
  timeout -k 10 400 python bench.py --workload it --steps 3 --warmup 2 > gpurun_out/sus_make.log 2>&1 || exit $?
python - <<'PY' || exit 1
import json
t = json.load(open("llm_training_amd/tuning/gemm_layouts_gfx950.json"))
t["layouts"].update(json.load(open("gpurun_out/r6_layouts_it_sustained.json"))["layouts"])
json.dump(t, open("gpurun_out/r6_layouts_it_merged.json", "w"), indent=1)
PY
: > gpurun_out/r6_sustained_it_ab.jsonl
for i in 1 2 3; do
  for v in shipped sustained; do
    if [ $v = sustained ]; then export LLMT_GEMM_LAYOUT_TABLE=gpurun_out/r6_layouts_it_merged.json; else unset LLMT_GEMM_LAYOUT_TABLE; fi
    timeout -k 10 400 python bench.py --workload it --steps 8 --warmup 3 > gpurun_out/sus_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/sus_$v.log | sed "s/^{/{\"arm\": \"it table=$v\", /" >> gpurun_out/r6_sustained_it_ab.jsonl
  done
done
cut -c1-200 gpurun_out/r6_sustained_it_ab.jsonl
