# End-of-session verification on one box: smoke, the headline bench as the driver runs it, every
# BASELINE workload, and kernel tables of the PT and IT steps (gpurun_out/verify_*.log, prof_*.md)
set -o pipefail
mkdir -p gpurun_out
scripts/gpu/steps.sh \
  "verify_smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "verify_pt|300|python bench.py --gpus 1 --steps 20 --warmup 5" \
  "verify_ptpacked|200|python bench.py --workload pt-packed --steps 8 --warmup 3" \
  "verify_it|250|python bench.py --workload it --steps 6 --warmup 3" \
  "verify_it8|250|python bench.py --workload it --micro-batch 8 --steps 8 --warmup 3" \
  "verify_dpo|200|python bench.py --workload dpo --steps 6 --warmup 3" \
  "verify_orpo|200|python bench.py --workload orpo --steps 6 --warmup 3" \
  "verify_prof_pt|400|bash scripts/gpu/prof_step.sh pt 3" \
  "verify_prof_it|400|bash scripts/gpu/prof_step.sh it 3 --workload it"
grep -h '^{"metric"' gpurun_out/verify_*.log | cut -c1-160
