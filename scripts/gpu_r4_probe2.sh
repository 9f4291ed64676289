#!/bin/bash
# hipBLASLt refresh (7B / 70B projections) and the coop GEMV ring-depth probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_probe2
mkdir -p $out
rm -f $out/*
timeout -k 10 400 python3 scripts/probes/coop_depth_probe.py > $out/coop_depth.jsonl 2> $out/coop_depth.err || { tail -20 $out/coop_depth.err; exit 6; }
cat $out/coop_depth.jsonl
timeout -k 10 600 bash scripts/gpu_r4_blaslt.sh || exit 5
