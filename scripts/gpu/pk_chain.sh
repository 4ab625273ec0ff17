set -o pipefail
mkdir -p gpurun_out
for v in 3 4 5 3 4 5; do
  LLMT_FA_FWD_VARIANT=$v timeout -k 10 100 python benchmarks/bench_packed_attention.py --B 8 --S 4096 --Hq 32 --Hkv 32 --D 96 --docs 1,8 > gpurun_out/pk_v$v.log 2>&1 || exit $?
  echo "v$v"; grep '^{' gpurun_out/pk_v$v.log | cut -c1-160
done
