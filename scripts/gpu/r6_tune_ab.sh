# Round 6: in-step A/B of timing hipBLASLt's top candidates for every problem (LLMT_GEMM_TUNE=1) against the
# heuristic's first stream-K solution (default), alternating runs on one box, Llama-3-8B PT
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r6_tune_ab.jsonl
for i in 1 2 3; do
  for v in 0 1; do
    LLMT_GEMM_TUNE=$v timeout -k 10 400 python bench.py --gpus 1 --steps 12 --warmup 3 > gpurun_out/tab_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/tab_$v.log | sed "s/^{/{\"arm\": \"pt gemm_tune=$v\", /" >> gpurun_out/r6_tune_ab.jsonl
  done
done
cut -c1-200 gpurun_out/r6_tune_ab.jsonl
