# Head-chained forward: in-process A/B (LLMT_FA_FWD_VARIANT 3/4 = one head per workgroup for D=96 / the
# default, 5 / 6 = chains of 2 / 4), attention tests, Phi-3 IT bench with and without chains
set -o pipefail
mkdir -p gpurun_out
for sh in "8 4096 32 32 96" "16 2048 32 32 96" "8 4096 32 32 64"; do
  timeout -k 10 120 python benchmarks/ab/ab_attention_fwd.py $sh 3,4 >> gpurun_out/ab_chain.log 2>&1 || exit $?
done
grep '^{' gpurun_out/ab_chain.log
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or attention or flash or varlen or phi" > gpurun_out/gt_chain.log 2>&1; tail -2 gpurun_out/gt_chain.log
timeout -k 10 200 python bench.py --workload it --steps 8 --warmup 3 > gpurun_out/it_chain.log 2>&1 && grep metric gpurun_out/it_chain.log | cut -c1-200
LLMT_FA_FWD_VARIANT=3 timeout -k 10 200 python bench.py --workload it --steps 8 --warmup 3 > gpurun_out/it_nochain.log 2>&1 && grep metric gpurun_out/it_nochain.log | cut -c1-200
