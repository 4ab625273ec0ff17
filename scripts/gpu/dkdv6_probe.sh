# diagnostic probes of fa_bwd_dkdv6 (wrong results by design): which part of the loop costs what
set -eo pipefail
mkdir -p gpurun_out
: > gpurun_out/dkdv6_probe.jsonl
for p in 0 1 2 4 8 12 15; do
  LLMT_FA_D6_PROBE=$p timeout -k 10 200 python -u benchmarks/ab/ab_attention_bwd.py 4 8192 32 8 128 5,7 | sed "s/^{/{\"probe\": $p, /" >> gpurun_out/dkdv6_probe.jsonl
done
cat gpurun_out/dkdv6_probe.jsonl
