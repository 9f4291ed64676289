#!/bin/bash
# Round 5: kernel trace of the batch-1 decode pass alone (every kernel of a token)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_y}
mkdir -p $out
rm -rf $out/*
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 -u bench.py --steps 2 --warmup 1 --latency-steps 64 --mid-batch 0 --ttft-lens 0 --extras= > $out/prof_bench.log 2>&1 || { tail -20 $out/prof_bench.log; exit 5; }
grep '^{' $out/prof_bench.log | cut -c1-100
f=$(find $out/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/kstats.py "$f" flash_prefill 30 > $out/kstats.txt
python3 scripts/step_gaps.py "$f" --min-us 1 > $out/gaps.txt
head -32 $out/kstats.txt
head -30 $out/gaps.txt
rm -f "$f"
