#!/bin/bash
# Round 5: the bench line with its side measurements (TTFT-2048 probe, 3B / 13B / 70B-stage extras)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_n}
mkdir -p $out
rm -rf $out/*
start=$(date +%s)
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 4; }
echo "bench wall $(( $(date +%s) - start )) s"
grep '^{' $out/bench.log | tail -1
