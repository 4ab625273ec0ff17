# PMC of the dK/dV kernels (v5 = fa_bwd_dkdv5, v7 = fa_bwd_dkdv6) at B4 S8192 Hq32 Hkv8 D128, two counter passes
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
C2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"
for v in 5 7; do
  export LLMT_FA_BWD_VARIANT=$v
  for p in 1 2; do
    if [ $p = 1 ]; then CC=$C1; else CC=$C2; fi
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CC -d gpurun_out/pmc_dkdv_${v}_$p -o run -- python benchmarks/probes/attn_probe.py > gpurun_out/pmc_dkdv_${v}_$p.log 2>&1
    python scripts/pmc_summary.py gpurun_out/pmc_dkdv_${v}_$p/run_results.db --match dkdv --last 2 > gpurun_out/pmc_dkdv_${v}_$p.txt
    rm -rf gpurun_out/pmc_dkdv_${v}_$p
  done
done
cat gpurun_out/pmc_dkdv_*.txt
