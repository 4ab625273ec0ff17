set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu1.log 2>&1; echo "pytest exit $?" >> gpurun_out/pytest_gpu1.log
tail -30 gpurun_out/pytest_gpu1.log
