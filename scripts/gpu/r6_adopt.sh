# Round 6: hipBLASLt choice adoption (gemm_lt_adopt) single-process and through the two-rank engine, and the
# opt-in fused SwiGLU GEMM tests after its default flipped off
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_swiglu_gemm_gpu.py \
  tests/test_multirank_gpu.py > gpurun_out/r6_adopt_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r6_adopt_tests.log
exit $rc
