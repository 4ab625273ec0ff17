# shipped layout table (per-problem stream-K twins) vs the previous table, alternating bench runs
set -eo pipefail
mkdir -p gpurun_out
out=gpurun_out/table_ab.jsonl
: > $out
OLD=llm_training_amd/tuning/_old_table_tmp.json
for t in new old new old; do
  if [ $t = old ]; then export LLMT_GEMM_LAYOUT_TABLE=$OLD; else unset LLMT_GEMM_LAYOUT_TABLE; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/table_ab_$t.log 2>&1
  grep '^{"metric"' gpurun_out/table_ab_$t.log | sed "s/^{/{\"table\": \"$t\", /" >> $out
done
unset LLMT_GEMM_LAYOUT_TABLE
# Phi-3 IT at micro-batch 8 (its M=32768 problems are not in either table: timed on first sight) -> dumps
for s in 1 0; do
  LLMT_GEMM_STREAMK=$s LLMT_GEMM_LAYOUTS=timed LLMT_GEMM_LAYOUT_DUMP=gpurun_out/layouts_it8_sk$s.json timeout -k 10 300 \
    python bench.py --workload it --micro-batch 8 --steps 6 --warmup 3 > gpurun_out/table_it8_$s.log 2>&1
  grep '^{"metric"' gpurun_out/table_it8_$s.log | sed "s/^{/{\"it8_streamk\": \"$s\", /" >> $out
done
cut -c1-200 $out
