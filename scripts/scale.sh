#!/bin/bash
# Scaling sweep on one MI355X node: bench.py at 1/2/4/8 GPUs (one process per GPU, RCCL over xGMI) for
# ZeRO stages 1/2/3 and the TP=2 + SP layout, one JSON line per run in $OUT/scale.jsonl.
#
#   scripts/scale.sh [OUT_DIR] [STEPS] [WARMUP]
#
# Each run is bounded by its own time limit; a run that faults or times out stops the sweep (its log
# is kept in $OUT/<name>.log). HSA_ENABLE_IPC_MODE_LEGACY=0 is required for RCCL on this driver.
set -u
OUT=${1:-gpurun_out/scale}
STEPS=${2:-10}
WARMUP=${3:-3}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
NGPU=$(python -c "import torch; print(torch.cuda.device_count())")
PORT=29611
run() {  # name nproc extra-args...
  local name=$1 n=$2; shift 2
  [ "$n" -gt "$NGPU" ] && { echo "skip $name: $n GPUs > $NGPU"; return 0; }
  PORT=$((PORT + 1))
  echo "== $name"
  timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
      --master-port $PORT bench.py --gpus "$n" --steps "$STEPS" --warmup "$WARMUP" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  grep '^{"metric"' "$OUT/$name.log" | tee -a "$OUT/scale.jsonl"
  if [ $rc -ne 0 ]; then echo "== $name failed (rc=$rc), stopping"; exit $rc; fi
}
for n in 1 2 4 8; do run "dp${n}_zero2" "$n"; done
for s in 1 3; do run "dp8_zero${s}" 8 --zero-stage "$s"; done
run "dp4_tp2_sp" 8 --tp 2
run "dp8_zero3_ckpt" 8 --zero-stage 3 --ckpt
