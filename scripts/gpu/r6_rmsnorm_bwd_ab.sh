# RMSNorm backward A/B as run in round 6 (LLMT_RMSNORM_BWD_PAIR 0 / 1 / 2 selected the one-wave-per-row kernel and
# two two-waves-per-row forms; only the winner is left, so the variable is now ignored) -> profiles/r6_rmsnorm_bwd_ab.jsonl
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "rmsnorm" > gpurun_out/r6_rms_tests.log 2>&1
tail -2 gpurun_out/r6_rms_tests.log
for v in 0 1 2; do
  LLMT_RMSNORM_BWD_PAIR=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "rmsnorm" > gpurun_out/r6_rms_tests_v$v.log 2>&1
  echo "variant $v: $(tail -1 gpurun_out/r6_rms_tests_v$v.log)"
done
timeout -k 10 300 python -u benchmarks/ab/ab_rmsnorm_bwd.py >> gpurun_out/r6_rmsnorm_bwd_ab.jsonl
tail -1 gpurun_out/r6_rmsnorm_bwd_ab.jsonl
