# Phi-3-mini IT (8 packed docs per 4096 row, D=96, MHA) at micro-batch 8: RoPE fused into attention
# (LLMT_ROPE_FUSED bwd / full) against the standalone passes (off), alternating runs on one box
set -eo pipefail
mkdir -p gpurun_out
: > gpurun_out/bench_rope_it_ab.jsonl
for m in bwd full off bwd full off; do
  LLMT_ROPE_FUSED=$m timeout -k 10 300 python -u bench.py --workload it --micro-batch 8 --steps 10 --warmup 3 \
    > gpurun_out/bench_rope_it_$m.log 2>&1
  grep '^{"metric"' gpurun_out/bench_rope_it_$m.log | sed "s/^{/{\"rope\": \"$m\", /" >> gpurun_out/bench_rope_it_ab.jsonl
done
cut -c1-200 gpurun_out/bench_rope_it_ab.jsonl
