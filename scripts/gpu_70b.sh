#!/bin/bash
# 70B memory model test + one 10-layer Llama-2-70B stage (of the 8-stage plan) on one GPU under
# rocprofv3 kernel stats + the 7B headline bench with its memory report.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/p70
timeout -k 10 300 python -u -m pytest tests/test_plan_70b.py -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/p70/pytest.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p70/prof -o run -- \
    python3 -u bench.py --model llama2-70b --stage-layers 10 --microbatches 8 --steps 10 --warmup 3 \
    --latency-steps 8 > gpurun_out/p70/stage.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/p70/bench7b.log 2>&1
echo "rc=$?"
