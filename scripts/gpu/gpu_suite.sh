# the whole GPU test suite in one process (as the driver runs it), log under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?
tail -n 15 gpurun_out/gpu_suite.log
exit $rc
