#!/bin/bash
# gemm_wr SwiGLU: fp32 tests, then the Llama-3.2-3B engine A/B (route on / off)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_swiglu
mkdir -p $out
rm -f $out/*
timeout -k 10 400 python -u -m pytest tests/test_gemm_wr_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
for wr in 0 1 0 1; do
  LSA_GEMM_WR=$wr timeout -k 10 300 python3 -u bench.py --model llama3.2-3b --steps 20 --warmup 5 --latency-steps 0 > $out/b3.log 2>&1 || { tail -20 $out/b3.log; exit 3; }
  echo "llama3.2-3b gemm_wr=$wr $(grep '^\[bench\] load' $out/b3.log)" | tee -a $out/ab.txt
done
