#!/bin/bash
# 70B stage (10 layers, 8 micro-batches of 512): o projection on gemm_wr (one round of 256
# 128 x 128 tiles) vs gemm_sk, alternating; plus the GPU tests of the route
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/w70
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_wr_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w70/test.log 2>&1 \
  || { tail -30 gpurun_out/w70/test.log; exit 3; }
tail -1 gpurun_out/w70/test.log
for v in 0 x 0 x; do
  LSA_GEMM_WR_RESID=$v timeout -k 10 300 python -u bench.py --model llama2-70b --stage-layers 10 --microbatches 8 --steps 10 --warmup 3 \
      --latency-steps 0 > gpurun_out/w70/stage_$v.log 2>&1 || { tail -20 gpurun_out/w70/stage_$v.log; exit 5; }
  echo "LSA_GEMM_WR_RESID=$v $(tail -1 gpurun_out/w70/stage_$v.log | cut -c1-140) $(tail -1 gpurun_out/w70/stage_$v.log | grep -o '"tokens_mb0_sha16": "[0-9a-f]*"')"
done
