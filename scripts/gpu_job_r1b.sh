#!/usr/bin/env bash
# ZeRO-2 engine path under RCCL (torchrun, 1 rank) + GEMM routing A/B on the end-to-end bench.
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
run z2_rccl 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --zero-stage 2 --steps 4 --warmup 2 &&
run z3_rccl 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --zero-stage 3 --steps 4 --warmup 2 &&
run gemm_wgrad 400 env LLMT_GEMM=wgrad python -u bench.py --steps 6 --warmup 2 &&
run gemm_blas 400 env LLMT_GEMM=blas python -u bench.py --steps 6 --warmup 2 &&
run gemm_blas_mb2 400 env LLMT_GEMM=blas python -u bench.py --steps 4 --warmup 2 --micro-batch 2
