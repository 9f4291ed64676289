#!/bin/bash
# Round 3: the 70B stage profile and Llama-3.2-3B with the new GQA decode kernel (+ kernel stats of the 70B stage).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r3m
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3m/p70 -o run -- \
    python3 -u bench.py --model llama2-70b --stage-layers 10 --microbatches 8 --steps 10 --warmup 3 \
    --latency-steps 8 > gpurun_out/r3m/stage70.log 2>&1 || { tail -20 gpurun_out/r3m/stage70.log; exit 3; }
tail -1 gpurun_out/r3m/stage70.log
T=$(find gpurun_out/r3m/p70 -name "*kernel_trace.csv" | head -1)
python scripts/gap_pairs.py "$T" --after flash_prefill_kernel > gpurun_out/r3m/p70_gaps.txt 2>&1
python scripts/kstats.py "$T" > gpurun_out/r3m/p70_kstats.txt 2>&1 || true
rm -f "$T"
timeout -k 10 400 python -u bench.py --model llama3.2-3b --steps 20 --warmup 5 > gpurun_out/r3m/b3b.log 2>&1 || { tail -20 gpurun_out/r3m/b3b.log; exit 4; }
tail -1 gpurun_out/r3m/b3b.log
