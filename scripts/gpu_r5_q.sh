#!/bin/bash
# Round 5: kernel table of the Llama-3.2-3B decode at 512 sequences (the reference's configured model)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_q}
mkdir -p $out
rm -rf $out/*
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 -u bench.py --model llama3.2-3b --steps 20 --warmup 5 --latency-steps 0 --ttft-lens 0 --extras= > $out/prof_bench.log 2>&1 || { tail -20 $out/prof_bench.log; exit 5; }
grep '^{' $out/prof_bench.log | cut -c1-200
f=$(find $out/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/kstats.py "$f" flash_prefill 14 > $out/kstats.txt
head -14 $out/kstats.txt
rm -f "$f"
