# fa_bwd_dkdv6 numerics + same-process A/B against dkdv5
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_dkdv6_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dkdv6_tests.log 2>&1
timeout -k 10 300 python -u benchmarks/ab/ab_attention_bwd.py 4 8192 32 8 128 5,7 > gpurun_out/ab_dkdv6.jsonl
timeout -k 10 300 python -u benchmarks/ab/ab_attention_bwd.py 16 2048 32 8 128 5,7 >> gpurun_out/ab_dkdv6.jsonl
cat gpurun_out/ab_dkdv6.jsonl
tail -n 3 gpurun_out/dkdv6_tests.log
