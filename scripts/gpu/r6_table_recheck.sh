# Round 6: the re-timed layout table against the round-5 table on another box, alternating PT / IT runs
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r6_table_recheck.jsonl
for wl in pt it; do
  for i in 1 2 3; do
    for v in r5 r6; do
      if [ $v = r5 ]; then export LLMT_GEMM_LAYOUT_TABLE=profiles/r5_gemm_layouts_gfx950.json; else unset LLMT_GEMM_LAYOUT_TABLE; fi
      timeout -k 10 400 python bench.py --workload $wl --steps 8 --warmup 3 > gpurun_out/trc_$v.log 2>&1 || exit $?
      grep '^{"metric"' gpurun_out/trc_$v.log | sed "s/^{/{\"arm\": \"$wl table=$v\", /" >> gpurun_out/r6_table_recheck.jsonl
    done
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r6_table_recheck.jsonl"):
    d = json.loads(l); print(d["arm"], d["value"], d["ms_per_step"])
PY
