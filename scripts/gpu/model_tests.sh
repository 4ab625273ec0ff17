set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_model_gpu.py -x -q -m gpu -s -k "${K:-gpu}" > gpurun_out/model_tests.log 2>&1; rc=$?
tail -30 gpurun_out/model_tests.log
exit $rc
