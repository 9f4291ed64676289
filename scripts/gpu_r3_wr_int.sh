#!/bin/bash
# gemm_wr integration: kernel tests, probe timing, headline bench A/B (LSA_GEMM_WR=0 / 1)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_wr_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_wr_test.log 2>&1 \
  || { tail -30 gpurun_out/r3_wr_test.log; exit 3; }
tail -1 gpurun_out/r3_wr_test.log
timeout -k 10 300 python scripts/gemm_wr_probe.py 512,12288,4096 512,4096,4096 > gpurun_out/r3_wr_probe2.jsonl 2>&1 || { tail -5 gpurun_out/r3_wr_probe2.jsonl; exit 4; }
grep -v amdgpu gpurun_out/r3_wr_probe2.jsonl
for v in 0 1 0 1; do
  LSA_GEMM_WR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_wr_bench_$v.log 2>&1 || { tail -20 gpurun_out/r3_wr_bench_$v.log; exit 5; }
  echo "LSA_GEMM_WR=$v $(tail -1 gpurun_out/r3_wr_bench_$v.log | cut -c1-160) $(tail -1 gpurun_out/r3_wr_bench_$v.log | grep -o '"tokens_mb0_sha16": "[0-9a-f]*"')"
done
