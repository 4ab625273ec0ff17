# RMSNorm backward after the A/B (two waves per row) and the 256-block column sum: kernel tests, the shape check /
# timing script (benchmarks/ab/ab_rmsnorm_bwd.py), and a kernel table of the headline step
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "rmsnorm" > gpurun_out/r6_rms_final_tests.log 2>&1
tail -1 gpurun_out/r6_rms_final_tests.log
timeout -k 10 300 python -u benchmarks/ab/ab_rmsnorm_bwd.py > gpurun_out/r6_rmsnorm_bwd_colsum.jsonl
cat gpurun_out/r6_rmsnorm_bwd_colsum.jsonl
timeout -k 10 400 bash scripts/gpu/prof_step.sh r6i_pt 3

