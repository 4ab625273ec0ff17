# Round 6: a layout table timed under longer interleaved rounds (LLMT_GEMM_LAYOUT_ROUNDS=10, after a
# heating run), then in-step A/B of that table against the shipped one, alternating runs on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 3 --warmup 2 > gpurun_out/sus_heat.log 2>&1 || exit $?
LLMT_GEMM_LAYOUTS=timed LLMT_GEMM_LAYOUT_ROUNDS=10 LLMT_GEMM_LAYOUT_DUMP=gpurun_out/r6_layouts_sustained.json \
  timeout -k 10 400 python bench.py --steps 3 --warmup 2 > gpurun_out/sus_make.log 2>&1 || exit $?
: > gpurun_out/r6_sustained_ab.jsonl
for i in 1 2 3; do
  for v in shipped sustained; do
    if [ $v = sustained ]; then export LLMT_GEMM_LAYOUT_TABLE=gpurun_out/r6_layouts_sustained.json; else unset LLMT_GEMM_LAYOUT_TABLE; fi
    timeout -k 10 400 python bench.py --steps 12 --warmup 3 > gpurun_out/sus_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/sus_$v.log | sed "s/^{/{\"arm\": \"pt table=$v\", /" >> gpurun_out/r6_sustained_ab.jsonl
  done
done
cut -c1-200 gpurun_out/r6_sustained_ab.jsonl
