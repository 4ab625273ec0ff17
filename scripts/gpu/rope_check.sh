# RoPE fused into attention: GPU numerics tests, the attention kernel tests, same-process A/B (Llama-3-8B dense
# S8192 mb4; Phi-3-mini packed 8 docs S4096 mb8 / mb16) -> gpurun_out/rope_*.log, gpurun_out/ab_rope.jsonl
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rope_fused_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rope_tests.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_fwd4_gpu.py -x -q -k "attn or rope or flash or attention" --timeout 120 --timeout-method thread > gpurun_out/rope_attn_tests.log 2>&1
timeout -k 10 180 python -u benchmarks/ab/ab_rope_attention.py > gpurun_out/ab_rope.jsonl
timeout -k 10 180 python -u benchmarks/ab/ab_rope_attention.py 4096 8 32 32 96 8 >> gpurun_out/ab_rope.jsonl
timeout -k 10 180 python -u benchmarks/ab/ab_rope_attention.py 4096 16 32 32 96 8 >> gpurun_out/ab_rope.jsonl
cat gpurun_out/ab_rope.jsonl
tail -n 3 gpurun_out/rope_tests.log gpurun_out/rope_attn_tests.log
