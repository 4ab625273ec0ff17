# Packed attention: work-ordered blocks (segment_info orders) vs index order, in one process per shape;
# attention GPU tests with the ordered layout
set -o pipefail
mkdir -p gpurun_out
LLMT_SEG_ORDER_AB=1 timeout -k 10 150 python benchmarks/bench_packed_attention.py --B 8 --S 4096 --Hq 32 --Hkv 32 --D 96 --docs 8 > gpurun_out/pk_order_phi3.log 2>&1 || exit $?
LLMT_SEG_ORDER_AB=1 timeout -k 10 150 python benchmarks/bench_packed_attention.py --B 4 --S 8192 --docs 8 > gpurun_out/pk_order_llama.log 2>&1 || exit $?
grep fwd_ms_ordered gpurun_out/pk_order_*.log
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or attention or flash or varlen or phi or long" > gpurun_out/gt_order.log 2>&1; tail -2 gpurun_out/gt_order.log
