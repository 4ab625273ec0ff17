# Round 6: the pruned attention dispatch (one kernel per pass) — attention GPU tests, the headline bench,
# and the hand-written GEMM against hipBLASLt at 32768 tokens
set -o pipefail
scripts/gpu/steps.sh \
  "r6_attn_tests|600|python -u -m pytest tests/test_kernels_gpu.py tests/test_varlen_gpu.py tests/test_rope_fused_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "r6_pt|300|python bench.py --gpus 1 --steps 20 --warmup 5" \
  "r6_gemm_hip|300|python benchmarks/bench_gemm_hip.py --tokens 32768 --rounds 3"
