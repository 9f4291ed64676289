#!/bin/bash
# Round 4: which Tensile kernels hipBLASLt picks for the 7B projection shapes (kernel names encode
# the tiling: MT, MI, DepthU, LDS buffering, prefetch, WGM, stream-K), plus a baseline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_names
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_names/prof -o run -- \
    python3 scripts/gemm_vs_hipblaslt.py 384,512,768,2048,16384 > gpurun_out/r4_names/cmp.jsonl 2> gpurun_out/r4_names/cmp.err || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4_names/bench.log 2>&1 || exit 2
tail -2 gpurun_out/r4_names/bench.log
