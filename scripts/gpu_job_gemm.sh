#!/usr/bin/env bash
# One gpurun job: GEMM numerics (both workgroup shapes) -> GEMM micro-bench -> end-to-end bench with
# HIP GEMMs. Each step has its own time limit; the chain stops at the first failure.
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local name=$1 t=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"
  tail -n 4 "gpurun_out/$name.log"
  return $rc
}
run gemm_tests_w4 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "gemm or linear_hip" --timeout 120 --timeout-method thread &&
run gemm_tests_w8 300 env LLMT_GEMM_WAVES=8 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread &&
run bench_gemm_w4 300 python -u benchmarks/bench_gemm_hip.py &&
run bench_hip_w4 400 python -u bench.py --steps 6 --warmup 2
