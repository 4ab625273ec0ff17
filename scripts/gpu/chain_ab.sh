# MHA head chains of the forward (LLMT_FA_FWD_VARIANT 5 / 6) under the document-major packed order
set -eo pipefail
mkdir -p gpurun_out
out=gpurun_out/chain_ab.jsonl
: > $out
LLMT_SEG_ORDER=2 timeout -k 10 300 python -u benchmarks/bench_packed_attention.py --B 8 --S 4096 --Hq 32 --Hkv 32 --D 96 \
  --docs 1,8 --ab LLMT_FA_FWD_VARIANT:4,5,6 >> $out
grep -v attended $out
