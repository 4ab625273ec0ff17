set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
LLMT_FA_FWD_VARIANT=1 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "flash or rope_attention" > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
for v in 0 1; do
  LLMT_FA_FWD_VARIANT=$v timeout -k 10 300 python benchmarks/bench_attention.py --S 8192 --Hq 32 --Hkv 8 --D 128 2>&1 | grep -v amdgpu.ids || exit 1
done
