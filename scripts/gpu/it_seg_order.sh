# Phi-3-mini IT at micro-batch 8: document-major packed block order (MHA default) vs heaviest-first,
# alternating runs; varlen GPU tests first
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_varlen_gpu.py > gpurun_out/varlen.log 2>&1
tail -2 gpurun_out/varlen.log
: > gpurun_out/it_seg_order.jsonl
for o in 2 1 2 1; do
  LLMT_SEG_ORDER=$o timeout -k 10 300 python -u bench.py --workload it --micro-batch 8 --steps 10 --warmup 3 \
    > gpurun_out/it_order_$o.log 2>&1
  grep '^{"metric"' gpurun_out/it_order_$o.log | sed "s/^{/{\"seg_order\": \"$o\", /" >> gpurun_out/it_seg_order.jsonl
done
cut -c1-220 gpurun_out/it_seg_order.jsonl
