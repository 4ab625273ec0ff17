#!/usr/bin/env bash
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/async_race_probe.py > gpurun_out/probe_blas.log 2>&1; rc=$?; cat gpurun_out/probe_blas.log | tail -30; [ $rc -eq 0 ] &&
LLMT_GEMM=hip timeout -k 10 200 python -u scripts/async_race_probe.py > gpurun_out/probe_hip.log 2>&1; rc=$?; echo "== hip"; tail -30 gpurun_out/probe_hip.log; exit $rc
