set -eo pipefail
mkdir -p gpurun_out
: > gpurun_out/seg_order.jsonl
for cfg in "4 4096 32 32 96 8" "8 4096 32 32 96 8" "4 4096 32 32 96 8 equal" "1 16384 32 32 96 16 equal" \
           "4 8192 32 8 128 8" "4 8192 32 8 128 32"; do
  timeout -k 10 150 python -u benchmarks/ab/ab_seg_order.py $cfg >> gpurun_out/seg_order.jsonl
done
cat gpurun_out/seg_order.jsonl
