#!/bin/bash
# batch-1 TTFT sweep + kernel trace (prefill attention vs GEMM split)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/ttft
timeout -k 10 300 python -u scripts/latency_sweep.py --lengths 128,512,2048,4096 --repeats 3 --decode-steps 16 \
    --decode-batches 1 > gpurun_out/ttft/sweep.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ttft/prof -o run -- \
    python3 -u scripts/latency_sweep.py --lengths 512,2048,4096 --repeats 1 --decode-steps 4 --decode-batches 1 \
    > gpurun_out/ttft/prof.log 2>&1
echo "rc=$?"
