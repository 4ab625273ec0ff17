# Round 6: for one workload (NAME, then its bench.py arguments), a layout table timed under longer interleaved
# rounds (LLMT_GEMM_LAYOUT_ROUNDS=10, after a heating run), merged over the shipped table, then an in-step A/B
# against the shipped table, alternating runs on one box.   bash scripts/gpu/r6_sustained_table_wl.sh it8 --workload it --micro-batch 8
set -o pipefail
mkdir -p gpurun_out
NAME=$1; shift
timeout -k 10 300 python bench.py "$@" --steps 3 --warmup 2 > gpurun_out/sus_${NAME}_heat.log 2>&1 || exit $?
LLMT_GEMM_LAYOUTS=timed LLMT_GEMM_LAYOUT_ROUNDS=10 LLMT_GEMM_LAYOUT_DUMP=gpurun_out/r6_layouts_${NAME}_sustained.json \
  timeout -k 10 400 python bench.py "$@" --steps 3 --warmup 2 > gpurun_out/sus_${NAME}_make.log 2>&1 || exit $?
python - "$NAME" <<'PY' || exit 1
import json, sys
name = sys.argv[1]
t = json.load(open("llm_training_amd/tuning/gemm_layouts_gfx950.json"))
t["layouts"].update(json.load(open(f"gpurun_out/r6_layouts_{name}_sustained.json"))["layouts"])
json.dump(t, open(f"gpurun_out/r6_layouts_{name}_merged.json", "w"), indent=1)
PY
: > gpurun_out/r6_sustained_${NAME}_ab.jsonl
for i in 1 2 3; do
  for v in shipped sustained; do
    if [ $v = sustained ]; then export LLMT_GEMM_LAYOUT_TABLE=gpurun_out/r6_layouts_${NAME}_merged.json; else unset LLMT_GEMM_LAYOUT_TABLE; fi
    timeout -k 10 400 python bench.py "$@" --steps 8 --warmup 3 > gpurun_out/sus_${NAME}_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/sus_${NAME}_$v.log | sed "s/^{/{\"arm\": \"$NAME table=$v\", /" >> gpurun_out/r6_sustained_${NAME}_ab.jsonl
  done
done
cut -c1-170 gpurun_out/r6_sustained_${NAME}_ab.jsonl
