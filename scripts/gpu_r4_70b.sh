#!/bin/bash
# round-4 Llama-2-70B: projection GEMMs vs fp32 at the stage's 512-row micro-batch, then one
# 10-layer stage of the 8-stage plan under rocprofv3 kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_70b
mkdir -p $out
rm -f $out/*
timeout -k 10 300 python -u -m pytest tests/test_gemm_sk_gpu.py -k llama70b -q --timeout 120 --timeout-method thread \
    > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 -u bench.py --model llama2-70b --stage-layers 10 --microbatches 8 --steps 10 --warmup 3 \
    --latency-steps 8 > $out/stage.log 2>&1 || { tail -20 $out/stage.log; exit 3; }
grep '^{' $out/stage.log | tail -1
