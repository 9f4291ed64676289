#!/bin/bash
# one 10-layer Llama-2-70B stage (of the 8-stage plan) under rocprofv3 kernel stats
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
rm -rf gpurun_out/p70 && mkdir -p gpurun_out/p70
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p70/prof -o run -- \
    python3 -u bench.py --model llama2-70b --stage-layers 10 --microbatches 8 --steps 10 --warmup 3 \
    --latency-steps 8 > gpurun_out/p70/stage.log 2>&1
echo "rc=$?"
