#!/bin/bash
# gemm_wr at the other models' qkv shapes where one round of 192-256 tiles exists (13B: 15360 x 5120
# at 320-384 rows; 70B: 10240 x 8192 at 384 rows with bn 128), vs gemm_sk's plan and hipBLASLt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_wr_shapes
mkdir -p $out
rm -f $out/*
timeout -k 10 400 python3 scripts/gemm_wr_probe.py ${WR_SHAPES:-384,15360,5120 320,15360,5120 384,10240,8192 448,10240,8192} \
    > $out/wr.jsonl 2> $out/wr.err || { tail -20 $out/wr.err; exit 2; }
cat $out/wr.jsonl
