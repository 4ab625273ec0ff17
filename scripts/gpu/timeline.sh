# rocprofv3 kernel trace of 3 bench steps; per-dispatch timeline of the attention forward and AdamW
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/tl -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/tl.bench.log 2>&1
db=$(find gpurun_out/tl -name '*results.db' | head -n 1)
python scripts/diag/kernel_timeline.py "$db" 'fa_fwd3|adamw' --tail-ms 1500 > gpurun_out/tl_fwd.txt
rm -rf gpurun_out/tl
head -80 gpurun_out/tl_fwd.txt
