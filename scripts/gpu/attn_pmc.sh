set -o pipefail
R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmc -o attn \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA \
  -- python3 $R/benchmarks/bench_attention.py --S 8192 > $R/gpurun_out/pmc.log 2>&1 || { tail -20 $R/gpurun_out/pmc.log; exit 1; }
find $R/gpurun_out/pmc -name "*.csv" | head
