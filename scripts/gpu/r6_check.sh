# Round 6 checks on one box: the pruned attention dispatch + fused SwiGLU GEMM (GPU tests), the fused
# SwiGLU-backward GEMM against the unfused pair, the staged TP GEMM sequences, then the headline bench
set -o pipefail
scripts/gpu/steps.sh \
  "r6_swiglu_tests|300|python -u -m pytest tests/test_swiglu_gemm_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "r6_swiglu_bench|300|python benchmarks/bench_swiglu_gemm.py --rounds 5" \
  "r6_attn_tests|600|python -u -m pytest tests/test_kernels_gpu.py tests/test_varlen_gpu.py tests/test_rope_fused_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "r6_pt|300|python bench.py --gpus 1 --steps 20 --warmup 5" \
  "r6_pt_nofuse|300|LLMT_SWIGLU_GEMM=0 python bench.py --gpus 1 --steps 20 --warmup 5" \
  "r6_tp_gemms|400|python benchmarks/bench_tp_gemms.py --rounds 2"
