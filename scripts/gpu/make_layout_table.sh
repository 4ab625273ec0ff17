#!/bin/bash
# Time every GEMM layout of the BASELINE workloads on this box (LLMT_GEMM_LAYOUTS=timed) and dump each
# workload's choices to gpurun_out/layouts_<workload>.json; scripts/merge_layout_tables.py merges them into
# the shipped table llm_training_amd/tuning/gemm_layouts_gfx950.json. The headline workload is timed twice:
# with stream-K GEMM solutions (one GPU) and without (LLMT_GEMM_STREAMK=0: what dp > 1 / tp > 1 runs).
# Each decision is timed over ROUNDS (default 10) interleaved rounds: short bursts favour layouts that lose
# under the step's sustained load (profiles/r6_sustained_table_*_ab.jsonl).
set -eo pipefail
mkdir -p gpurun_out
run() {  # name, env..., -- bench args
  local name=$1; shift
  env LLMT_GEMM_LAYOUTS=timed LLMT_GEMM_LAYOUT_ROUNDS=${ROUNDS-10} LLMT_GEMM_LAYOUT_DUMP=gpurun_out/layouts_$name.json "$@" \
    > gpurun_out/layouts_$name.log 2>&1
  grep '^{"metric"' gpurun_out/layouts_$name.log | cut -c1-160
}
for w in ${WORKLOADS-pt it dpo orpo}; do
  run $w timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 2
done
run pt_nosk LLMT_GEMM_STREAMK=0 timeout -k 10 300 python bench.py --workload pt --steps 3 --warmup 2
run it_nosk LLMT_GEMM_STREAMK=0 timeout -k 10 300 python bench.py --workload it --steps 3 --warmup 2
# Phi-3 IT at micro-batch 8 (the round-4 verdict's comparison point): its 32768-token problems
run it8 timeout -k 10 300 python bench.py --workload it --micro-batch 8 --steps 3 --warmup 2
run it8_nosk LLMT_GEMM_STREAMK=0 timeout -k 10 300 python bench.py --workload it --micro-batch 8 --steps 3 --warmup 2
