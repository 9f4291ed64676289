#!/bin/bash
# Round 5: kernel trace of the headline bench on the current tree (per-kernel table + step gaps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_k}
mkdir -p $out
rm -rf $out/*
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 -u bench.py --steps 20 --warmup 5 --latency-steps 0 > $out/prof_bench.log 2>&1 || { tail -20 $out/prof_bench.log; exit 5; }
grep '^{' $out/prof_bench.log | tail -1
f=$(find $out/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/kstats.py "$f" flash_prefill 16 > $out/kstats.txt
python3 scripts/step_gaps.py "$f" --min-us 2 > $out/gaps.txt
head -14 $out/kstats.txt
head -20 $out/gaps.txt
gzip -c "$f" > $out/trace.csv.gz
rm -f "$f"
