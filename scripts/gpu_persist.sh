#!/bin/bash
# persistent batch-1 decode: correctness vs the graph step, latency, headline bench (b1 keys)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pers
timeout -k 10 240 python -u -m pytest tests/test_decode_persistent_gpu.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pers/pytest.log 2>&1 &&
timeout -k 10 240 python -u scripts/latency_sweep.py --lengths 128 --repeats 2 --decode-steps 32 --decode-batches 1 \
    > gpurun_out/pers/sweep.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/pers/bench.log 2>&1
echo "rc=$?"
