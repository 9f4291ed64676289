#!/bin/bash
# fused QKV + attention: consumer unroll variants (scripts/probes/qa_stamps.py --build first)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_qa4
rm -f gpurun_out/r4_qa4/*
for T in 150 500; do
  timeout -k 10 120 python3 scripts/probes/qa_stamps.py $T >> gpurun_out/r4_qa4/stamps.jsonl 2>> gpurun_out/r4_qa4/err.log || { tail -20 gpurun_out/r4_qa4/err.log; exit 1; }
done
cat gpurun_out/r4_qa4/stamps.jsonl
