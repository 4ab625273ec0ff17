# In-process A/B of the attention store-tail variants (see profiles/r3_attention_wide_store_ab.jsonl)
set -o pipefail
mkdir -p gpurun_out
for sh in "4 8192 32 8 128" "32 1024 32 8 128" "64 512 32 8 128"; do
  timeout -k 10 120 python benchmarks/ab/ab_attention_bwd.py $sh 3,4 LLMT_FA_BWD_VARIANT >> gpurun_out/ab_dkdv_ws.log 2>&1 || exit $?
done
grep '^{' gpurun_out/ab_dkdv_ws.log
