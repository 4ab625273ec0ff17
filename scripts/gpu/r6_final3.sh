# Round 6 verification after the one-pass cross-entropy kernel: the GPU suite as the driver runs it, smoke(),
# the CE check / timing script, the headline bench, DPO and ORPO (log-prob heads), and a kernel table of the PT step
set -o pipefail
mkdir -p gpurun_out
scripts/gpu/steps.sh \
  "r6j_gpu_suite|700|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "r6j_smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r6j_ce|200|python -u benchmarks/ab/ab_ce.py" \
  "r6j_pt|240|python bench.py --gpus 1 --steps 20 --warmup 5" \
  "r6j_dpo|200|python bench.py --workload dpo --steps 6 --warmup 3" \
  "r6j_orpo|200|python bench.py --workload orpo --steps 6 --warmup 3" \
  "r6j_prof|400|bash scripts/gpu/prof_step.sh r6j_pt 3"
grep -h '^{"metric"' gpurun_out/r6j_*.log | cut -c1-200
