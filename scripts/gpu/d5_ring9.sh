set -eo pipefail
mkdir -p gpurun_out
out=gpurun_out/d5_ring9.jsonl
: > $out
timeout -k 10 200 python -u benchmarks/ab/ab_attention_bwd.py 4 8192 32 8 128 8,9 LLMT_FA_D5_RING >> $out
timeout -k 10 200 python -u benchmarks/ab/ab_attention_bwd.py 1 32768 32 8 128 8,9 LLMT_FA_D5_RING >> $out
timeout -k 10 200 python -u benchmarks/ab/ab_attention_bwd.py 4 8192 32 8 128 8,9 LLMT_FA_D5_RING >> $out
timeout -k 10 300 python -u benchmarks/bench_packed_attention.py --B 4 --S 8192 --docs 8 --ab LLMT_FA_D5_RING:8,9 >> $out
grep -v attended $out
