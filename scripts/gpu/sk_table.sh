# per-problem stream-K choice: GEMM GPU tests, then the layout table re-timed with the /nosk twins
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/sk_tests.log 2>&1
tail -2 gpurun_out/sk_tests.log
WORKLOADS="pt it dpo orpo" bash scripts/gpu/make_layout_table.sh
