#!/bin/bash
# idle gaps between kernels in the headline decode steps (final round-3 kernels)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/g2
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g2/prof -o run -- \
    python3 -u bench.py --steps 20 --warmup 5 --latency-steps 0 > gpurun_out/g2/bench.log 2>&1 || { tail -20 gpurun_out/g2/bench.log; exit 3; }
f=$(find gpurun_out/g2/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/gap_pairs.py "$f" > gpurun_out/g2/gaps.txt; python3 scripts/step_gaps.py "$f" > gpurun_out/g2/step_gaps.txt; cat gpurun_out/g2/step_gaps.txt
head -25 gpurun_out/g2/gaps.txt
rm -f "$f"
