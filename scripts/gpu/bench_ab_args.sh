# alternating headline bench runs with two extra argument strings: scripts/gpu/bench_ab_args.sh TAG "ARGS_A" "ARGS_B" [steps]
set -eo pipefail
tag=$1; a=$2; b=$3; steps=${4:-10}
mkdir -p gpurun_out
out=gpurun_out/bench_ab_$tag.jsonl
: > $out
i=0
for args in "$a" "$b" "$a" "$b"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps $steps --warmup 3 $args > gpurun_out/bench_ab_${tag}_$i.log 2>&1 || true
  grep '^{"metric"' gpurun_out/bench_ab_${tag}_$i.log | sed "s/^{/{\"args\": \"$args\", /" >> $out || echo "{\"args\": \"$args\", \"failed\": true}" >> $out
done
cut -c1-200 $out
grep -h -i "out of memory\|Error" gpurun_out/bench_ab_${tag}_*.log | head -3 || true
