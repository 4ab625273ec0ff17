# per-kernel times of short dense rows vs long rows (same token count): which kernel carries the per-block cost
set -eo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "32 512 32 32 96" "4 4096 32 32 96" "64 512 32 8 128" "4 8192 32 8 128"; do
  tag=$(echo $cfg | tr ' ' _)
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/split_$tag -o run -- python3 benchmarks/probes/attn_probe.py $cfg 1 20 > /dev/null 2>&1
  db=$(find gpurun_out/split_$tag -name '*results.db' | head -n 1)
  python scripts/prof_summary.py "$db" --top 6 > gpurun_out/split_$tag.md
  rm -rf gpurun_out/split_$tag
  echo "== $cfg"; cut -c1-160 gpurun_out/split_$tag.md | sed -n 3,10p
done
