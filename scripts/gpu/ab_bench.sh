# attention numerics (new fwd + bwd), fwd kernel A/B, then bench A/B: GEMM tuning file on/off
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for v in 0 1; do
  echo "fwd variant $v"
  LLMT_FA_FWD_VARIANT=$v timeout -k 10 300 python benchmarks/bench_attention.py --S 8192 --Hq 32 --Hkv 8 --D 128 2>&1 | grep -v amdgpu.ids || exit 1
done
for g in use off; do
  timeout -k 10 600 python bench.py --steps 6 --warmup 2 --gemm-tuning $g > gpurun_out/bench_$g.log 2>&1 || { echo "bench $g failed"; tail -30 gpurun_out/bench_$g.log; exit 1; }
  tail -1 gpurun_out/bench_$g.log | cut -c1-400
done
