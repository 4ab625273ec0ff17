set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for shp in "--S 8192 --Hq 32 --Hkv 8 --D 128 --sdpa" "--S 4096 --Hq 32 --Hkv 32 --D 96 --sdpa" "--S 2048 --B 4 --Hq 32 --Hkv 8 --D 128"; do
  timeout -k 10 300 python benchmarks/bench_attention.py $shp 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/attn_bench.log || exit 1
done
