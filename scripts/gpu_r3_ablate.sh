#!/bin/bash
# gemm_sk ablation builds at the headline decode shapes (M = 512) and at M = 16384
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
# M N K bn split
timeout -k 10 500 python scripts/sk_ablate.py 512 12288 4096 128 1  512 12288 4096 256 2  512 22016 4096 192 1 \
    512 4096 11008 128 0  16384 4096 4096 256 0 > gpurun_out/r3_ablate.jsonl 2>&1; rc=$?
cat gpurun_out/r3_ablate.jsonl
exit $rc
