set -eo pipefail
mkdir -p gpurun_out
: > gpurun_out/dkdv6_probe2.jsonl
for p in 0 16 32 4; do
  LLMT_FA_D6_PROBE=$p timeout -k 10 200 python -u benchmarks/ab/ab_attention_bwd.py 4 8192 32 8 128 5,7 | sed "s/^{/{\"probe\": $p, /" >> gpurun_out/dkdv6_probe2.jsonl
done
cut -c1-170 gpurun_out/dkdv6_probe2.jsonl
