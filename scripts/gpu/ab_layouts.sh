#!/bin/bash
# Headline step with the shipped GEMM layout table against per-process timing, alternating on one box
# (the table must be within noise of the timed choice), after dumping the no-stream-K choices (dp > 1).
set -o pipefail
mkdir -p gpurun_out
WORKLOADS= bash scripts/gpu/make_layout_table.sh || exit $?
for i in 1 2; do
  for m in table timed; do
    LLMT_GEMM_LAYOUTS=$m timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/ablay_${m}_$i.log 2>&1 || exit $?
    echo "$m $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ablay_${m}_$i.log) $(grep -o '"gemm_layouts": {[^}]*}' gpurun_out/ablay_${m}_$i.log)"
  done
done
