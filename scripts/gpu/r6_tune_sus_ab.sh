# Round 6: in-step A/B of hipBLASLt solutions timed over 8 interleaved rounds per problem (LLMT_GEMM_TUNE=1,
# LLMT_GEMM_TUNE_ROUNDS=8) against the heuristic's first (default), alternating runs on one box, Llama-3-8B PT;
# the tuned run exports its choices (gpurun_out/r6_lt_tuned_*.txt)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r6_tune_sus_ab.jsonl
for i in 1 2 3; do
  for v in 0 1; do
    LLMT_GEMM_TUNE=$v LLMT_GEMM_TUNE_ROUNDS=8 LLMT_GEMM_LT_EXPORT=gpurun_out/r6_lt_tuned_$v.txt \
      timeout -k 10 500 python bench.py --gpus 1 --steps 12 --warmup 3 > gpurun_out/tsa_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/tsa_$v.log | sed "s/^{/{\"arm\": \"pt gemm_tune_rounds8=$v\", /" >> gpurun_out/r6_tune_sus_ab.jsonl
  done
done
cut -c1-200 gpurun_out/r6_tune_sus_ab.jsonl
