#!/bin/bash
# long-context decode points and the bigger-batch point on the round-3 kernels
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/lc
export TMPDIR=/tmp
for cfg in "32 4000" "64 2000" "1024 128"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --latency-steps 0 --batch $1 --prompt-len $2 > gpurun_out/lc/b$1_p$2.log 2>&1 || { tail -20 gpurun_out/lc/b$1_p$2.log; exit 3; }
  echo "batch $1 prompt $2: $(tail -1 gpurun_out/lc/b$1_p$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_tpot_ms"], d["p90_tpot_ms"], d["ttft_ms"], d["mem_peak_gb"])')"
done
