# pt-packed workload (8 isolated documents per 8192 row, GQA D128): dK/dV ring 8 (default) vs 6, alternating
set -eo pipefail
mkdir -p gpurun_out
out=gpurun_out/ptpacked_ring.jsonl
: > $out
for r in 8 6 8 6; do
  LLMT_FA_D5_RING=$r timeout -k 10 300 python bench.py --workload pt-packed --steps 8 --warmup 3 > gpurun_out/ptp_ring_$r.log 2>&1
  grep '^{"metric"' gpurun_out/ptp_ring_$r.log | sed "s/^{/{\"ring\": \"$r\", /" >> $out
done
cut -c1-200 $out
