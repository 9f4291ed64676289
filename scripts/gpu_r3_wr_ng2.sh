#!/bin/bash
# gemm_wr with two wave groups (ng = 2, bn 128) vs one (ng = 1): correctness + timing
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gemm_wr_gpu.py -x -q --timeout 60 --timeout-method thread -k "two_wave" > gpurun_out/r3_ng2_test.log 2>&1 \
  || { tail -30 gpurun_out/r3_ng2_test.log; exit 3; }
tail -1 gpurun_out/r3_ng2_test.log
timeout -k 10 200 python scripts/gemm_wr_probe.py 512,4096,4096 512,12288,4096 16384,4096,4096 > gpurun_out/r3_ng2_probe.jsonl 2>&1 || { tail -5 gpurun_out/r3_ng2_probe.jsonl; exit 4; }
grep -v amdgpu gpurun_out/r3_ng2_probe.jsonl
