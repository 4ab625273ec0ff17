# Round 6 evidence runs on one box: the remaining BASELINE workloads, the multi-GPU engine schedule on one GPU
# (ZeRO-2 / ZeRO-3 over a one-rank RCCL group), the S=131072 long-context step and the IT kernel table
set -o pipefail
mkdir -p gpurun_out
scripts/gpu/steps.sh \
  "r6e_pt|300|python bench.py --gpus 1 --steps 12 --warmup 3" \
  "r6e_dpo|250|python bench.py --workload dpo --steps 6 --warmup 3" \
  "r6e_orpo|250|python bench.py --workload orpo --steps 6 --warmup 3" \
  "r6e_z2sharded|300|python bench.py --force-sharded --zero-stage 2 --steps 8 --warmup 3" \
  "r6e_z3sharded|300|python bench.py --force-sharded --zero-stage 3 --steps 8 --warmup 3" \
  "r6e_long|400|python bench.py --seq 131072 --micro-batch 1 --ckpt --ckpt-keep-attn --steps 2 --warmup 1" \
  "r6e_prof_it|400|bash scripts/gpu/prof_step.sh r6e_it 3 --workload it"
grep -h '^{"metric"' gpurun_out/r6e_*.log | cut -c1-220
