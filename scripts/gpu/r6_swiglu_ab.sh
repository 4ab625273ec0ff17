# Round 6: in-step A/B of the fused SwiGLU-backward GEMM (default) against hipBLASLt + swiglu_bwd_tr
# (LLMT_SWIGLU_GEMM=0), alternating runs on one box: Llama-3-8B PT and Phi-3-mini IT
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r6_swiglu_ab.jsonl
for i in 1 2 3; do
  for v in 1 0; do
    LLMT_SWIGLU_GEMM=$v timeout -k 10 300 python bench.py --gpus 1 --steps 12 --warmup 3 > gpurun_out/ab_pt_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/ab_pt_$v.log | sed "s/^{/{\"arm\": \"pt swiglu_gemm=$v\", /" >> gpurun_out/r6_swiglu_ab.jsonl
  done
done
for i in 1 2; do
  for v in 1 0; do
    LLMT_SWIGLU_GEMM=$v timeout -k 10 300 python bench.py --workload it --steps 6 --warmup 3 > gpurun_out/ab_it_$v.log 2>&1 || exit $?
    grep '^{"metric"' gpurun_out/ab_it_$v.log | sed "s/^{/{\"arm\": \"it swiglu_gemm=$v\", /" >> gpurun_out/r6_swiglu_ab.jsonl
  done
done
cut -c1-150 gpurun_out/r6_swiglu_ab.jsonl
