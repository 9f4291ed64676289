#!/bin/bash
# flash prefill v2: numerics, attention roofline, TTFT sweep
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pf
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "prefill" -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pf/pytest.log 2>&1 &&
timeout -k 10 200 python -u scripts/prefill_attn_bench.py > gpurun_out/pf/attn.jsonl 2> gpurun_out/pf/attn.err &&
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_hypothesis_gpu.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pf/pytest2.log 2>&1 &&
timeout -k 10 300 python -u scripts/latency_sweep.py --lengths 128,512,2048,4096 --repeats 3 --decode-steps 16 \
    --decode-batches 1 > gpurun_out/pf/sweep.log 2>&1
echo "rc=$?"
