# PMC passes of the own ping-pong GEMM vs hipBLASLt on the down-projection input gradient
# (benchmarks/probes/gemm_pair_probe.py) -> gpurun_out/pmc_pair_*.txt
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/pmc_pair_$i -o run -- python benchmarks/probes/gemm_pair_probe.py > gpurun_out/pmc_pair_$i.log 2>&1
  db=$(find gpurun_out/pmc_pair_$i -name '*results.db' | head -n 1)
  python scripts/pmc_summary.py "$db" --match "gemm_pp|Cijk" > gpurun_out/pmc_pair_$i.txt
  rm -rf gpurun_out/pmc_pair_$i
done
cat gpurun_out/pmc_pair_*.txt
