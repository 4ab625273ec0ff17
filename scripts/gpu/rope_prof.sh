# per-kernel times of rope_attention fwd+bwd, fused vs standalone RoPE (Llama-3-8B shape) -> gpurun_out/rope_prof_*
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in fused standalone; do
  LLMT_AB_ONLY=$m timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/rope_prof_$m -o run -- python benchmarks/ab/ab_rope_attention.py > gpurun_out/rope_prof_$m.log 2>&1
  python scripts/prof_summary.py gpurun_out/rope_prof_$m/run_results.db --steps 30 --top 8 > gpurun_out/rope_prof_$m.md
  cat gpurun_out/rope_prof_$m.md
done
