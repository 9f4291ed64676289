#!/bin/bash
# o projection on gemm_wr (two wave groups, EPI_RESID + fused-RMSNorm ss_out): tests, then a
# headline A/B (LSA_GEMM_WR_RESID=0 / 1, alternating)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_wr_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_wro_test.log 2>&1 \
  || { tail -30 gpurun_out/r3_wro_test.log; exit 3; }
tail -1 gpurun_out/r3_wro_test.log
for v in 0 1 0 1; do
  LSA_GEMM_WR_RESID=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --latency-steps 0 > gpurun_out/r3_wro_bench_$v.log 2>&1 || { tail -20 gpurun_out/r3_wro_bench_$v.log; exit 5; }
  echo "LSA_GEMM_WR_RESID=$v $(tail -1 gpurun_out/r3_wro_bench_$v.log | cut -c1-150) $(tail -1 gpurun_out/r3_wro_bench_$v.log | grep -o '"tokens_mb0_sha16": "[0-9a-f]*"')"
done
