set -o pipefail
mkdir -p gpurun_out
for sh in "4 8192 32 8 128" "32 1024 32 8 128" "64 512 32 8 128" "8 4096 32 32 96"; do
  timeout -k 10 120 python benchmarks/ab_attention_fwd.py $sh 3,4 >> gpurun_out/ab_fwd_ws.log 2>&1 || exit $?
done
for sh in "4 8192 32 8 128" "32 1024 32 8 128"; do
  timeout -k 10 120 python benchmarks/ab_attention_bwd.py $sh 1,2 LLMT_FA_DQ_VARIANT >> gpurun_out/ab_dq_ws.log 2>&1 || exit $?
done
cat gpurun_out/ab_fwd_ws.log gpurun_out/ab_dq_ws.log | grep '^{'
