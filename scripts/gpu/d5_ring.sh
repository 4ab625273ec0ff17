# dK/dV ring depth (LLMT_FA_D5_RING 6 / 8): dense and packed, D=96 MHA and D=128 GQA, same process
set -eo pipefail
mkdir -p gpurun_out
out=gpurun_out/d5_ring.jsonl
: > $out
timeout -k 10 200 python -u benchmarks/ab/ab_attention_bwd.py 8 4096 32 32 96 6,8 LLMT_FA_D5_RING >> $out
timeout -k 10 200 python -u benchmarks/ab/ab_attention_bwd.py 4 8192 32 8 128 6,8 LLMT_FA_D5_RING >> $out
LLMT_SEG_ORDER=2 timeout -k 10 300 python -u benchmarks/bench_packed_attention.py --B 8 --S 4096 --Hq 32 --Hkv 32 --D 96 \
  --docs 8 --ab LLMT_FA_D5_RING:6,8 >> $out
timeout -k 10 300 python -u benchmarks/bench_packed_attention.py --B 4 --S 8192 --docs 8,32 --ab LLMT_FA_D5_RING:6,8 >> $out
grep -v attended $out
