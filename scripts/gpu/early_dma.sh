# attention prologues with the first ring tiles issued before the row loads (LLMT_FA_EARLY_DMA=1) vs rows
# first (0): GPU attention tests, bitwise A/B on dense rows, packed-row A/B (Phi-3 D=96 MHA, Llama D=128 GQA)
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_varlen_gpu.py \
  tests/test_rope_fused_gpu.py > gpurun_out/early_tests.log 2>&1
tail -3 gpurun_out/early_tests.log
timeout -k 10 200 python -u benchmarks/ab/ab_attention_bwd.py 4 8192 32 8 128 0,1 LLMT_FA_EARLY_DMA > gpurun_out/early_ab.jsonl
timeout -k 10 200 python -u benchmarks/ab/ab_attention_bwd.py 8 4096 32 32 96 0,1 LLMT_FA_EARLY_DMA >> gpurun_out/early_ab.jsonl
timeout -k 10 300 python -u benchmarks/bench_packed_attention.py --B 4 --S 4096 --Hq 32 --Hkv 32 --D 96 --docs 1,8 \
  --ab LLMT_FA_EARLY_DMA:0,1 >> gpurun_out/early_ab.jsonl
timeout -k 10 300 python -u benchmarks/bench_packed_attention.py --B 4 --S 8192 --docs 1,8,32 \
  --ab LLMT_FA_EARLY_DMA:0,1 >> gpurun_out/early_ab.jsonl
cat gpurun_out/early_ab.jsonl
