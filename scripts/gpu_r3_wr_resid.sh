#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_wr_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_wr_test2.log 2>&1 \
  || { tail -30 gpurun_out/r3_wr_test2.log; exit 3; }
tail -1 gpurun_out/r3_wr_test2.log
timeout -k 10 300 python scripts/wr_resid_probe.py > gpurun_out/r3_wr_resid.jsonl 2>&1 || { tail -5 gpurun_out/r3_wr_resid.jsonl; exit 4; }
grep -v amdgpu gpurun_out/r3_wr_resid.jsonl
