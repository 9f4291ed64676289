#!/bin/bash
# gemm_wr prefetch depth (ns 4 / 6 / 8): fp32 tests, then the cold-weight probe vs gemm_sk
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_wr
mkdir -p $out
rm -f $out/*
timeout -k 10 400 python -u -m pytest tests/test_gemm_wr_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
timeout -k 10 400 python3 scripts/gemm_wr_probe.py 512,12288,4096 512,4096,4096 512,22016,4096 512,4096,11008 \
    2048,12288,4096 2048,4096,4096 384,12288,4096 768,4096,4096 > $out/probe.jsonl 2> $out/probe.err || { tail -20 $out/probe.err; exit 3; }
cat $out/probe.jsonl
