#!/bin/bash
# GQA decode kernel: tests vs fp32, then the bench (70B and 3B heads); then gemm_sk ablations.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_attn_gqa_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_gqa_test.log 2>&1 || { tail -30 gpurun_out/r3_gqa_test.log; exit 3; }
tail -2 gpurun_out/r3_gqa_test.log
timeout -k 10 300 python scripts/attn_gqa_bench.py > gpurun_out/r3_gqa_bench.jsonl 2>&1 || { tail -20 gpurun_out/r3_gqa_bench.jsonl; exit 4; }
cat gpurun_out/r3_gqa_bench.jsonl
bash scripts/gpu_r3_ablate.sh || exit 5
timeout -k 10 300 python scripts/cumask_probe.py > gpurun_out/r3_cumask.jsonl 2>&1; cat gpurun_out/r3_cumask.jsonl
