#!/bin/bash
# kernel trace of the headline bench on the final round-3 kernels (decode window breakdown)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pf
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pf/prof -o run -- \
    python3 -u bench.py --steps 20 --warmup 5 --latency-steps 0 > gpurun_out/pf/bench.log 2>&1 || { tail -20 gpurun_out/pf/bench.log; exit 3; }
tail -1 gpurun_out/pf/bench.log | cut -c1-300
f=$(find gpurun_out/pf/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/kstats.py "$f" flash_prefill 14 > gpurun_out/pf/kstats.txt
head -20 gpurun_out/pf/kstats.txt
rm -f "$f"
