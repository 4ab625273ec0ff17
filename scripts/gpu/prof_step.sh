#!/bin/bash
# Kernel table of N timed bench.py steps: rocprofv3 kernel trace -> markdown summary; the raw database
# is deleted (it is too large to bring back).   scripts/gpu/prof_step.sh NAME STEPS [bench.py args...]
set -eo pipefail
name=$1; steps=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace -d "gpurun_out/prof_$name" -o run -- \
  python bench.py --steps "$steps" --warmup 2 "$@" > "gpurun_out/prof_$name.bench.log" 2> "gpurun_out/prof_$name.err"
db=$(find "gpurun_out/prof_$name" -name '*results.db' | head -n 1)
python scripts/prof_summary.py "$db" --bench-log "gpurun_out/prof_$name.bench.log" --top 40 > "gpurun_out/prof_$name.md"
rm -rf "gpurun_out/prof_$name"
grep '^{"metric"' "gpurun_out/prof_$name.bench.log"
head -5 "gpurun_out/prof_$name.md"
