#!/usr/bin/env bash
# One gpurun job: GEMM numerics -> GEMM micro-bench -> end-to-end bench with HIP and with library GEMMs
# -> every GPU test. Each step has its own time limit; the chain stops at the first failure.
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
run gemm_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "gemm or linear_hip" --timeout 120 --timeout-method thread &&
run bench_gemm 300 python -u benchmarks/bench_gemm_hip.py &&
run bench_hip 400 python -u bench.py --steps 6 --warmup 2 &&
run bench_blas 400 env LLMT_GEMM=blas python -u bench.py --steps 6 --warmup 2 &&
run gpu_tests 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
