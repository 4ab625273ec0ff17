# Round 6: in-step A/B of timing the non-stream-K hipBLASLt candidates on first sight (LLMT_GEMM_NOSK_TIME=1,
# default) against the heuristic's first non-stream-K solution (0): the multi-GPU engine schedule on one GPU
# (every GEMM non-stream-K) and the one-GPU step (the table's /nosk twins), alternating runs on one box
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r6_nosk_ab.jsonl
for i in 1 2 3; do
  for v in 1 0; do
    LLMT_GEMM_NOSK_TIME=$v timeout -k 10 400 python bench.py --force-sharded --zero-stage 2 --steps 10 --warmup 3 > gpurun_out/nab_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/nab_$v.log | sed "s/^{/{\"arm\": \"z2 sharded nosk_time=$v\", /" >> gpurun_out/r6_nosk_ab.jsonl
  done
done
for i in 1 2; do
  for v in 1 0; do
    LLMT_GEMM_NOSK_TIME=$v timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/nab1_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/nab1_$v.log | sed "s/^{/{\"arm\": \"pt nosk_time=$v\", /" >> gpurun_out/r6_nosk_ab.jsonl
  done
done
cut -c1-200 gpurun_out/r6_nosk_ab.jsonl
