set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for o in 1 0; do
  LLMT_OVERLAP_STEP=$o timeout -k 10 600 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_ov$o.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_ov$o.log; exit 1; }
  echo "overlap_step=$o"; tail -1 gpurun_out/bench_ov$o.log | cut -c1-330
done
