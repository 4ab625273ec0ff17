# Llama-3-8B at S = 131072 (the reference TP example's length) on one GPU with full_keep_attention recompute,
# round-6 kernels -> gpurun_out/r6_long_context.log
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --seq 131072 --micro-batch 1 --ckpt --ckpt-keep-attn --steps 3 --warmup 2 > gpurun_out/r6_long_context.log 2>&1
grep '^{"metric"' gpurun_out/r6_long_context.log | cut -c1-300
