# Round 6: in-step A/B of the shipped GEMM layout table against first-sight timed layouts
# (LLMT_GEMM_LAYOUTS=timed), alternating runs on one box, Llama-3-8B PT; each timed run dumps its choices.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r6_layout_ab.jsonl
for i in 1 2 3; do
  for v in table timed; do
    LLMT_GEMM_LAYOUTS=$v LLMT_GEMM_LAYOUT_DUMP=gpurun_out/r6_layouts_${v}_$i.json \
      timeout -k 10 300 python bench.py --gpus 1 --steps 12 --warmup 3 > gpurun_out/lab_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/lab_$v.log | sed "s/^{/{\"arm\": \"pt layouts=$v\", /" >> gpurun_out/r6_layout_ab.jsonl
  done
done
cut -c1-200 gpurun_out/r6_layout_ab.jsonl
