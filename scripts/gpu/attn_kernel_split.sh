# per-kernel times of short dense rows vs long rows (same token count): which kernel carries the per-block cost
set -eo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in "32 512 32 32 96" "4 4096 32 32 96" "64 512 32 8 128" "4 8192 32 8 128"; do
  tag=$(echo $cfg | tr ' ' _)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/split_$tag -o run -- python3 benchmarks/attn_one_shape.py $cfg 1 20 > /dev/null 2>&1
  f=$(find gpurun_out/split_$tag -name '*kernel_stats.csv' | head -1)
  echo "== $cfg"; cut -d, -f1-5 "$f" | head -6
done
