# Round 6 verification after the RMSNorm backward change: the GPU suite as the driver runs it, smoke(), the
# headline bench as the driver runs it and the Phi-3 IT workload
set -o pipefail
mkdir -p gpurun_out
scripts/gpu/steps.sh \
  "r6g_gpu_suite|700|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "r6g_smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r6g_pt|240|python bench.py --gpus 1 --steps 20 --warmup 5" \
  "r6g_it|200|python bench.py --workload it --steps 6 --warmup 3"
grep -h '^{"metric"' gpurun_out/r6g_*.log | cut -c1-200
