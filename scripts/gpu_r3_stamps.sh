#!/bin/bash
# gemm_sk phase stamps (prologue / main loop / fixup / epilogue per workgroup) at the headline
# decode shapes (M = 512, Llama-2-7B projections, the engine's tuned plans), cold weights.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r3_stamps.txt
: > $O
# M N K bn grid dp split reps bm
for cfg in "512 12288 4096 128 256 1 6 6 256" "512 12288 4096 192 256 1 2 6 256" "512 12288 4096 256 256 1 2 6 256" \
           "512 22016 4096 192 256 1 1 6 256" "512 4096 11008 128 256 1 0 6 256" "512 4096 4096 128 256 1 0 6 128" \
           "16384 4096 4096 256 256 1 0 3 256"; do
  timeout -k 10 120 python scripts/gemm_stamps.py $cfg >> $O 2>&1 || { echo "FAILED $cfg"; tail -5 $O; exit 3; }
done
cat $O
