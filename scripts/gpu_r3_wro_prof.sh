#!/bin/bash
# kernel trace of the headline step with the o projection on gemm_wr ng = 2 (LSA_GEMM_WR_RESID=1) vs gemm_sk
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for v in 1 0; do
  d=gpurun_out/wro$v
  mkdir -p $d
  LSA_GEMM_WR_RESID=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d/prof -o run -- \
      python3 -u bench.py --steps 10 --warmup 3 --latency-steps 0 > $d/bench.log 2>&1 || { tail -20 $d/bench.log; exit 3; }
  f=$(find $d/prof -name "*kernel_trace.csv" | head -1)
  python3 scripts/kstats.py "$f" flash_prefill 14 > $d/kstats.txt
  echo "== LSA_GEMM_WR_RESID=$v"; head -14 $d/kstats.txt
  rm -f "$f"
done
