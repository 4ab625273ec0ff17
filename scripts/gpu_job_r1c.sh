#!/usr/bin/env bash
# Default-config bench (micro-batch 2, library GEMMs) + micro-batch 3, rocprofv3 kernel stats, all GPU tests.
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
  tail -n 2 "gpurun_out/$name.log"
  return $rc
}
run bench_default 400 python -u bench.py --steps 6 --warmup 2 &&
run bench_mb3 400 python -u bench.py --steps 4 --warmup 2 --micro-batch 3 &&
run prof_default 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1c -o run -- python3 bench.py --steps 2 --warmup 1 &&
run gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
