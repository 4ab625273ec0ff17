# PMC passes of the hand-written GEMM (benchmarks/probes/gemm_hip_probe.py) -> gpurun_out/pmc_gemm_*
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
for sk in "gate_up fwd" "gate_up wgrad"; do
  set -- $sk
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C1 -d gpurun_out/pmc_gemm_$1_$2 -o run -- python benchmarks/probes/gemm_hip_probe.py $1 $2 > gpurun_out/pmc_gemm_$1_$2.log 2>&1
done
find gpurun_out -path '*pmc_gemm*' -name '*.csv' | head -20
