# Round 6: the dp = 8 engine schedule end to end on ONE GPU (8 rank processes over gloo, every rank on GPU 0,
# a 2-layer Llama-3-8B-width model: a plumbing rehearsal of bench.py --gpus 8, not a throughput number), ZeRO-2
# and ZeRO-3
set -o pipefail
mkdir -p gpurun_out
export LLMT_DIST_BACKEND=gloo LLMT_SHARED_DEVICE=1 OMP_NUM_THREADS=2
scripts/gpu/steps.sh \
  "r6_dp8_z2|400|python bench.py --gpus 8 --layers 2 --seq 2048 --micro-batch 1 --steps 3 --warmup 1 --probe-mb 8" \
  "r6_dp8_z3|400|python bench.py --gpus 8 --layers 2 --seq 2048 --micro-batch 1 --steps 3 --warmup 1 --probe-mb 8 --zero-stage 3"
grep -h '^{"metric"' gpurun_out/r6_dp8_*.log | cut -c1-400
