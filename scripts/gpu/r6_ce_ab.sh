# Cross-entropy A/B as run in round 6 (LLMT_CE_REG 0 / 1 selected the two-pass / one-pass kernel; the switch is gone,
# the one-pass kernel is used for every aligned row of up to 131072 logits) -> profiles/r6_ce_ab.jsonl
set -eo pipefail
mkdir -p gpurun_out
for v in 1 0; do
  LLMT_CE_REG=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_tp_gpu.py -k "cross_entropy or logps or kernel_index or loss_head or vocab" > gpurun_out/r6_ce_tests_v$v.log 2>&1
  echo "variant $v: $(tail -1 gpurun_out/r6_ce_tests_v$v.log)"
done
timeout -k 10 300 python -u benchmarks/ab/ab_ce.py > gpurun_out/r6_ce_ab.jsonl
cat gpurun_out/r6_ce_ab.jsonl
