set -eo pipefail
mkdir -p gpurun_out
: > gpurun_out/block_probe.jsonl
for cfg in "32 512 32 32 96" "4 4096 32 32 96" "64 512 32 8 128" "4 8192 32 8 128"; do
  timeout -k 10 120 python -u benchmarks/probes/attn_block_probe.py $cfg >> gpurun_out/block_probe.jsonl
done
LLMT_FA_EARLY_DMA=0 timeout -k 10 120 python -u benchmarks/probes/attn_block_probe.py 32 512 32 32 96 >> gpurun_out/block_probe.jsonl
cat gpurun_out/block_probe.jsonl
