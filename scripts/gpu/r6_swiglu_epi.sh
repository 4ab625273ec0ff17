# Round 6: the fused SwiGLU-backward GEMM with double-buffered epilogue loads: numerics, then its rate
set -o pipefail
scripts/gpu/steps.sh \
  "r6_epi_tests|300|python -u -m pytest tests/test_swiglu_gemm_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "r6_epi_bench|300|python benchmarks/bench_swiglu_gemm.py --rounds 5" \
  "r6_tp_gemms2|400|python benchmarks/bench_tp_gemms.py --rounds 2"
