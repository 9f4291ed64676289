#!/bin/bash
# kernel trace of the headline bench (decode window breakdown per step)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pb
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pb/prof -o run -- \
    python3 -u bench.py --steps 20 --warmup 5 --latency-steps 0 > gpurun_out/pb/bench.log 2>&1
echo "rc=$?"
