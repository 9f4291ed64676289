#!/bin/bash
# round-4 batch-1 TTFT sweep (prompt 8 .. 4096) and batch-1/4/16 decode TPOT on the final kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_latency
mkdir -p $out
rm -f $out/*
timeout -k 10 500 python3 -u scripts/latency_sweep.py --lengths 8,16,32,64,128,256,512,1024,2048,4096 > $out/sweep.jsonl 2> $out/sweep.err || { tail -20 $out/sweep.err; exit 2; }
cat $out/sweep.jsonl
