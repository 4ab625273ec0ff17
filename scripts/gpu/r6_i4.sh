# Round 6: the interleaved 4-wave GEMM (gemm_i4_kernel): numerics of every layout / output mode and of the
# fused SwiGLU form, then its rate against the ping-pong kernel and hipBLASLt on the down-projection dgrad
set -o pipefail
scripts/gpu/steps.sh \
  "r6_i4_tests|300|python -u -m pytest tests/test_kernels_gpu.py -k gemm_layouts -x -q --timeout 120 --timeout-method thread" \
  "r6_i4_swiglu_tests|300|python -u -m pytest tests/test_swiglu_gemm_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "r6_i4_bench|300|python benchmarks/bench_swiglu_gemm.py --rounds 5"
