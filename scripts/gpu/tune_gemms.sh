# hipBLASLt solution tuning (TunableOp) on the Llama-3-8B bench shapes, then bench with the results.
# Continues from the shipped results file (already-tuned shapes are skipped).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
F=$R/gpurun_out/tunableop_gfx950.csv
cp llm_training_amd/tuning/tunableop_gfx950.csv $F
(while true; do date >> gpurun_out/heartbeat.log; wc -l $F >> gpurun_out/heartbeat.log; sleep 50; done) &
HB=$!
LLMT_GEMM_TUNING_MS=${TUNE_MS:-60} LLMT_GEMM_TUNING_ITERS=${TUNE_ITERS:-20} LLMT_GEMM_TUNING_FILE=$F \
  timeout -k 10 1000 python bench.py --steps 1 --warmup 1 --gemm-tuning tune > gpurun_out/tune.log 2>&1 || { kill $HB; echo "tune failed"; tail -30 gpurun_out/tune.log; exit 1; }
kill $HB
tail -1 gpurun_out/tune.log
wc -l $F
LLMT_GEMM_TUNING_FILE=$F timeout -k 10 600 python bench.py --steps 5 --warmup 2 --gemm-tuning use > gpurun_out/bench_tuned.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_tuned.log; exit 1; }
tail -1 gpurun_out/bench_tuned.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --gemm-tuning off > gpurun_out/bench_untuned.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_untuned.log; exit 1; }
tail -1 gpurun_out/bench_untuned.log
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k adamw 2>&1 | tail -1
