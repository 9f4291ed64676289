#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/wr_partial_probe.py 128 64 > gpurun_out/r3_wr_partial128.jsonl 2>&1 || { tail -5 gpurun_out/r3_wr_partial128.jsonl; exit 4; }
grep -v amdgpu gpurun_out/r3_wr_partial128.jsonl
