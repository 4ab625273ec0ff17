# Round 6 closing numbers for the workloads r6_final3.sh did not run: Phi-3 IT (mb 16, mb 8) and pt-packed
set -o pipefail
mkdir -p gpurun_out
scripts/gpu/steps.sh \
  "r6l_it|250|python bench.py --workload it --steps 6 --warmup 3" \
  "r6l_it8|250|python bench.py --workload it --micro-batch 8 --steps 8 --warmup 3" \
  "r6l_ptpacked|200|python bench.py --workload pt-packed --steps 8 --warmup 3" \
  "r6l_pt|240|python bench.py --gpus 1 --steps 20 --warmup 5"
grep -h '^{"metric"' gpurun_out/r6l_*.log | cut -c1-200
