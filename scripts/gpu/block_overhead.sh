set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/probes/attn_block_overhead.py 16384 32 32 96 > gpurun_out/block_overhead.jsonl
timeout -k 10 300 python -u benchmarks/probes/attn_block_overhead.py 32768 32 8 128 >> gpurun_out/block_overhead.jsonl
cat gpurun_out/block_overhead.jsonl
