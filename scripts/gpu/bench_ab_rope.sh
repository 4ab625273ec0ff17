# headline step: RoPE fused (auto) vs standalone (off), alternating, then a kernel table of the default
set -eo pipefail
mkdir -p gpurun_out
: > gpurun_out/bench_rope_ab.jsonl
for m in auto off auto off; do
  LLMT_ROPE_FUSED=$m timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_rope_$m.log 2>&1
  grep '^{"metric"' gpurun_out/bench_rope_$m.log | sed "s/^{/{\"rope\": \"$m\", /" >> gpurun_out/bench_rope_ab.jsonl
done
cat gpurun_out/bench_rope_ab.jsonl | cut -c1-260
bash scripts/gpu/prof_step.sh pt_r5 3
