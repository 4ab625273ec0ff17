# PMC counters for the attention kernels (kernel trace + counters only: no sys/runtime traces)
set -o pipefail
R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  n=$(echo $set | cut -c1-12 | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmc/$n -o attn --pmc $set \
    -- python3 $R/benchmarks/bench_attention.py --S 8192 --Hq 32 --Hkv 8 --D 128 > $R/gpurun_out/pmc/$n.log 2>&1 || { tail -20 $R/gpurun_out/pmc/$n.log; exit 1; }
done
find $R/gpurun_out/pmc -name "*counter_collection.csv" | head
