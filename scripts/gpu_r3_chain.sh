#!/bin/bash
# Reference-API chain path with hipGraph decode: GPU tests, then 7B b1 per-token time graph vs eager.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "node_worker or profiler" \
    > gpurun_out/r3_chain_test.log 2>&1 || { tail -30 gpurun_out/r3_chain_test.log; exit 3; }
tail -2 gpurun_out/r3_chain_test.log
timeout -k 10 400 python scripts/chain_graph_bench.py --model llama2-7b --tokens 64 > gpurun_out/r3_chain_graph_bench.jsonl 2>&1 \
    || { tail -20 gpurun_out/r3_chain_graph_bench.jsonl; exit 4; }
cat gpurun_out/r3_chain_graph_bench.jsonl
