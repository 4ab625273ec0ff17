# run GPU tests (args: pytest selection)
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 ${T:-600} python -m pytest ${@:-tests} -x -q -m gpu > gpurun_out/pytest.log 2>&1; rc=$?
tail -40 gpurun_out/pytest.log
exit $rc
