set -eo pipefail
mkdir -p gpurun_out
: > gpurun_out/bench_rope_ab3.jsonl
for m in bwd full off bwd full off; do
  LLMT_ROPE_FUSED=$m timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_rope_$m.log 2>&1
  grep '^{"metric"' gpurun_out/bench_rope_$m.log | sed "s/^{/{\"rope\": \"$m\", /" >> gpurun_out/bench_rope_ab3.jsonl
done
cut -c1-200 gpurun_out/bench_rope_ab3.jsonl
