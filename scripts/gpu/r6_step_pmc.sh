# Whole-step PMC counters of the headline bench (Llama-3-8B PT, mb 4 x 8192, 1 GPU): three passes (SQ issue /
# MFMA counters; L2 fetch bytes; L2 write bytes), each one warm-up + one timed bench.py step, reduced on the box
# to per-kernel sums (scripts/pmc_kernels_json.py) -> gpurun_out/step_pmc_{1,2,3}.json
# (merged by scripts/pmc_step_table.py into profiles/r6_step_pmc.md).
#   scripts/gpu/r6_step_pmc.sh [NAME [bench.py args...]]   (default NAME step_pmc, the headline bench)
set -eo pipefail
name=${1:-step_pmc}; shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="FETCH_SIZE SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P3="WRITE_SIZE SQ_INSTS_VMEM SQ_INSTS_SALU"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 420 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/${name}_$i -o run -- \
    python bench.py --steps 1 --warmup 1 "$@" > gpurun_out/${name}_$i.log 2>&1
  db=$(find gpurun_out/${name}_$i -name '*results.db' | head -n 1)
  python scripts/pmc_kernels_json.py "$db" > gpurun_out/${name}_$i.json
  rm -rf gpurun_out/${name}_$i
  echo "pass $i done"
done
