# Round 6: hipBLASLt's own split-K (GSU via hipblaslt_ext::GemmTuning) as extra timed candidates for GEMMs whose
# output has < 1024 tiles (the weight gradients): correctness, then the step's GEMMs standalone with every layout
# timed, with and without GSU, then the in-step SwiGLU A/B
set -o pipefail
scripts/gpu/steps.sh \
  "r6_gsu_tests|300|LLMT_GEMM_GSU=2,4,8 LLMT_GEMM_LAYOUTS=timed python -u -m pytest tests/test_kernels_gpu.py -k 'gemm_lt or linear or backward_gemms or wgrad' -x -q --timeout 120 --timeout-method thread" \
  "r6_roof_table|300|python benchmarks/gemm_roofline.py --tag table" \
  "r6_roof_timed|400|LLMT_GEMM_LAYOUTS=timed python benchmarks/gemm_roofline.py --tag timed" \
  "r6_roof_gsu|500|LLMT_GEMM_LAYOUTS=timed LLMT_GEMM_GSU=2,4,8 python benchmarks/gemm_roofline.py --tag gsu" \
  "r6_swiglu_ab|700|bash scripts/gpu/r6_swiglu_ab.sh"
