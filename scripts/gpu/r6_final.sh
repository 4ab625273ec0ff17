# Round 6 verification on one box: the GPU suite as the driver runs it, smoke(), the headline bench as the
# driver runs it, the Phi-3 IT workloads, and the kernel table of the PT step (default path: unfused SwiGLU)
set -o pipefail
mkdir -p gpurun_out
scripts/gpu/steps.sh \
  "r6f_gpu_suite|900|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "r6f_smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r6f_pt|300|python bench.py --gpus 1 --steps 20 --warmup 5" \
  "r6f_it|250|python bench.py --workload it --steps 6 --warmup 3" \
  "r6f_it8|250|python bench.py --workload it --micro-batch 8 --steps 8 --warmup 3" \
  "r6f_ptpacked|200|python bench.py --workload pt-packed --steps 8 --warmup 3" \
  "r6f_prof_pt|400|bash scripts/gpu/prof_step.sh r6f_pt 3"
grep -h '^{"metric"' gpurun_out/r6f_*.log | cut -c1-200
