#!/usr/bin/env bash
# Optimizer offload: GPU equivalence test, then the 8B bench with host AdamW.
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"
  tail -n 3 "gpurun_out/$name.log"
  return $rc
}
run offload_test 300 python -u -m pytest tests/test_model_gpu.py -x -v -k "offload or async" --timeout 120 --timeout-method thread &&
run bench_offload 500 python -u bench.py --steps 2 --warmup 1 --offload-optimizer
