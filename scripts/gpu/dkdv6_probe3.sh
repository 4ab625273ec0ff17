set -eo pipefail
mkdir -p gpurun_out
LLMT_FA_D6_PROBE=16 timeout -k 10 200 python -u -m pytest tests/test_attention_dkdv6_gpu.py -q --timeout 120 --timeout-method thread -x > gpurun_out/p16_test.log 2>&1 || true
tail -n 3 gpurun_out/p16_test.log
: > gpurun_out/dkdv6_probe3.jsonl
for p in 0 4 64 68 15; do
  LLMT_FA_D6_PROBE=$p timeout -k 10 200 python -u benchmarks/ab/ab_attention_bwd.py 4 8192 32 8 128 5,7 | sed "s/^{/{\"probe\": $p, /" >> gpurun_out/dkdv6_probe3.jsonl
done
cut -c1-170 gpurun_out/dkdv6_probe3.jsonl
