# Phi-3 IT mb 8: RoPE "full" (Q rotated on load, only k rotated in place) vs "bwd", alternating
set -eo pipefail
mkdir -p gpurun_out
out=gpurun_out/it_rope_full.jsonl
: > $out
for m in bwd full bwd full; do
  LLMT_ROPE_FUSED=$m timeout -k 10 300 python bench.py --workload it --micro-batch 8 --steps 10 --warmup 3 > gpurun_out/it_rope_$m.log 2>&1
  grep '^{"metric"' gpurun_out/it_rope_$m.log | sed "s/^{/{\"rope\": \"$m\", /" >> $out
done
cut -c1-200 $out
