#!/bin/bash
# Round 5: batch-1 decode attention time against the context length (small-grid kernel vs the
# 4-wave split kernel), back-to-back in a hipGraph, with a trivial-kernel floor.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_s}
mkdir -p $out
rm -rf $out/*
timeout -k 10 120 python3 scripts/attn_small_probe.py > $out/small.jsonl 2>&1 || { tail -20 $out/small.jsonl; exit 2; }
LSA_ATTN_SMALL_MAX_WGS=0 timeout -k 10 120 python3 scripts/attn_small_probe.py > $out/split.jsonl 2>&1 || { tail -20 $out/split.jsonl; exit 3; }
cat $out/small.jsonl $out/split.jsonl
