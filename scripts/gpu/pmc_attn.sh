# PMC pass of the attention kernels (dense Llama shape and 8 packed documents): SQ issue / wait shares, MFMA
# busy and the effective clock (GRBM_GUI_ACTIVE) -> gpurun_out/pmc_attn_*.txt
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
export LLMT_SEG_ORDER=2  # (GQA rows ignore it in the models; set here so the Phi-3 shape runs its model order)
for spec in "dense:4 8192 32 8 128 1" "packed:4 8192 32 8 128 8" "phi3packed:8 4096 32 32 96 8"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc_attn_$name -o run -- python benchmarks/probes/attn_probe.py $args > gpurun_out/pmc_attn_$name.log 2>&1
  python scripts/pmc_summary.py gpurun_out/pmc_attn_$name/run_results.db --match fa_ --last 2 > gpurun_out/pmc_attn_$name.txt
  rm -rf gpurun_out/pmc_attn_$name
done
cat gpurun_out/pmc_attn_dense.txt gpurun_out/pmc_attn_phi3packed.txt
