# GQA head pairs (two q heads per 8-wave workgroup sharing the K/V ring) vs one head per workgroup:
# forward (LLMT_FA_FWD_VARIANT 4 vs 7) and dQ (LLMT_FA_DQ_VARIANT 2 vs 3), in one process per shape
set -o pipefail
mkdir -p gpurun_out
for sh in "4 8192 32 8 128" "32 1024 32 8 128" "2 4096 32 8 128"; do
  timeout -k 10 120 python benchmarks/ab/ab_attention_fwd.py $sh 4,7 >> gpurun_out/ab_pair.log 2>&1 || exit $?
  timeout -k 10 120 python benchmarks/ab/ab_attention_bwd.py $sh 2,3 LLMT_FA_DQ_VARIANT >> gpurun_out/ab_pair.log 2>&1 || exit $?
done
grep '^{' gpurun_out/ab_pair.log
