# RMSNorm backward after the A/B (only the two-waves-per-row kernel left): kernel tests, the shape check /
# timing script, and one headline bench run
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "rmsnorm" > gpurun_out/r6_rms_final_tests.log 2>&1
tail -1 gpurun_out/r6_rms_final_tests.log
timeout -k 10 300 python -u benchmarks/ab/ab_rmsnorm_bwd.py > gpurun_out/r6_rmsnorm_bwd_final.jsonl
cat gpurun_out/r6_rmsnorm_bwd_final.jsonl
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r6_rms_bench.log 2>&1
grep '^{"metric"' gpurun_out/r6_rms_bench.log | cut -c1-200
