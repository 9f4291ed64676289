#!/bin/bash
# Round 3: stage-cost planner test + a kernel trace of the headline decode (idle gaps by kernel pair).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r3gaps
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stage_costs_gpu.py -x -v -s --timeout 240 --timeout-method thread \
    > gpurun_out/r3_stage_costs.log 2>&1 || { tail -30 gpurun_out/r3_stage_costs.log; exit 3; }
grep "stage-costs" gpurun_out/r3_stage_costs.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3gaps -o run -- \
    python3 bench.py --steps 10 --warmup 3 --latency-steps 0 > gpurun_out/r3gaps/bench.log 2>&1 || { tail -20 gpurun_out/r3gaps/bench.log; exit 4; }
tail -2 gpurun_out/r3gaps/bench.log
T=$(find gpurun_out/r3gaps -name "*kernel_trace.csv" | head -1)
python scripts/gap_pairs.py "$T" > gpurun_out/r3gaps/gap_pairs.txt && cat gpurun_out/r3gaps/gap_pairs.txt

