# alternating headline bench runs under two values of one env knob: scripts/gpu/bench_ab_env.sh VAR A B [steps]
set -eo pipefail
var=$1; a=$2; b=$3; steps=${4:-10}
mkdir -p gpurun_out
out=gpurun_out/bench_ab_${var}.jsonl
: > $out
for v in $a $b $a $b; do
  env $var=$v timeout -k 10 300 python bench.py --steps $steps --warmup 3 > gpurun_out/bench_ab_${var}_$v.log 2>&1
  grep '^{"metric"' gpurun_out/bench_ab_${var}_$v.log | sed "s/^{/{\"$var\": \"$v\", /" >> $out
done
cut -c1-190 $out
