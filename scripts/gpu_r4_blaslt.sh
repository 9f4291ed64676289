#!/bin/bash
# round-4 refresh: hand-written GEMM dispatch vs hipBLASLt (7B: 5 row counts; 70B: 512 rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_blaslt
mkdir -p $out
rm -f $out/*
timeout -k 10 500 python3 scripts/gemm_vs_hipblaslt.py 384,512,768,2048,16384 > $out/7b.jsonl 2> $out/7b.err || { tail -20 $out/7b.err; exit 1; }
cat $out/7b.jsonl
timeout -k 10 400 python3 scripts/gemm_vs_hipblaslt.py 512,4096 llama2-70b > $out/70b.jsonl 2> $out/70b.err || { tail -20 $out/70b.err; exit 2; }
cat $out/70b.jsonl
