set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python benchmarks/bench_gemm_layouts.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/gemm_layouts.jsonl
