#!/usr/bin/env bash
# Default bench (micro-batch 3), AdamW-stream overlap off, threaded host-AdamW offload bench.
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
  tail -n 1 "gpurun_out/$name.log"
  return $rc
}
run bench_mb3_default 400 python -u bench.py --steps 5 --warmup 2 &&
run bench_mb3_nooverlap 400 env LLMT_OVERLAP_STEP=0 python -u bench.py --steps 5 --warmup 2 &&
run bench_offload2 500 python -u bench.py --steps 2 --warmup 1 --offload-optimizer
