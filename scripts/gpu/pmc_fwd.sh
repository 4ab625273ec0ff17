# PMC pass of the forward attention variants (default fwd3 = 4, hand-allocated fwd4 = 10) at B4 S8192:
# issue / wait shares, MFMA busy, LDS waits and conflicts, clock -> gpurun_out/pmc_fwd_*.txt
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
C2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
for v in 4 10; do
  for pass in 1 2; do
    if [ $pass = 1 ]; then CC=$C; else CC=$C2; fi
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CC -d gpurun_out/pmc_fwd_${v}_$pass -o run -- python benchmarks/probes/attn_fwd_probe.py $v > gpurun_out/pmc_fwd_${v}_$pass.log 2>&1
    python scripts/pmc_summary.py gpurun_out/pmc_fwd_${v}_$pass/run_results.db --match fa_fwd --last 2 > gpurun_out/pmc_fwd_${v}_$pass.txt
    rm -rf gpurun_out/pmc_fwd_${v}_$pass
  done
done
cat gpurun_out/pmc_fwd_*.txt
