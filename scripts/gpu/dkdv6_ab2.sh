set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_dkdv6_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dkdv6_tests.log 2>&1
: > gpurun_out/dkdv6_probe.jsonl
for p in 0 4 15; do
  LLMT_FA_D6_PROBE=$p timeout -k 10 200 python -u benchmarks/ab/ab_attention_bwd.py 4 8192 32 8 128 5,7 | sed "s/^{/{\"probe\": $p, /" >> gpurun_out/dkdv6_probe.jsonl
done
timeout -k 10 300 python -u benchmarks/ab/ab_attention_bwd.py 16 2048 32 8 128 5,7 >> gpurun_out/dkdv6_probe.jsonl
cat gpurun_out/dkdv6_probe.jsonl
tail -n 2 gpurun_out/dkdv6_tests.log
