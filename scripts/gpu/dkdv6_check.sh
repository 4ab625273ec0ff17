# fa_bwd_dkdv6 (64 keys per wave) numerics, RoPE fusion modes, then same-process A/B of the backward
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_dkdv6_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dkdv6_tests.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_rope_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rope_tests.log 2>&1
timeout -k 10 300 python -u benchmarks/ab/ab_attention_bwd.py 4 8192 32 8 128 5,7 > gpurun_out/ab_dkdv6.jsonl
timeout -k 10 300 python -u benchmarks/ab/ab_attention_bwd.py 16 2048 32 8 128 5,7 >> gpurun_out/ab_dkdv6.jsonl
timeout -k 10 180 python -u benchmarks/ab/ab_rope_attention.py > gpurun_out/ab_rope.jsonl
timeout -k 10 180 python -u benchmarks/ab/ab_rope_attention.py 4096 8 32 32 96 8 >> gpurun_out/ab_rope.jsonl
cat gpurun_out/ab_dkdv6.jsonl gpurun_out/ab_rope.jsonl
tail -n 3 gpurun_out/dkdv6_tests.log gpurun_out/rope_tests.log
