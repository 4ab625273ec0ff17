# Round 6: the whole GPU suite as the driver runs it, smoke(), then a kernel table of the PT step
set -o pipefail
mkdir -p gpurun_out
scripts/gpu/steps.sh \
  "r6_gpu_suite|900|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "r6_smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r6_prof_pt|400|bash scripts/gpu/prof_step.sh r6_pt 3"
