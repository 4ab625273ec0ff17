# per-kernel times of the attention microbench (rocprofv3 kernel trace + stats)
set -o pipefail
R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/astats -o attn \
  -- python3 $R/benchmarks/bench_attention.py --S 8192 --Hq 32 --Hkv 8 --D 128 > $R/gpurun_out/astats.log 2>&1 || { tail -20 $R/gpurun_out/astats.log; exit 1; }
f=$(find $R/gpurun_out/astats -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -12
