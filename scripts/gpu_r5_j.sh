#!/bin/bash
# Round 5: write-through (sc1) epilogue output stores (LSA_EPI_WT=1 variant library) vs the shipped
# library: GEMM numerics with the variant, then the headline bench alternating, 3 pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_j}
mkdir -p $out
rm -rf $out/*
WT=$PWD/llm_sharding_amd/_native/variants/liblsa_kernels_wt.so
LSA_KERNELS_SO=$WT timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -q \
    --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
for i in 1 2 3; do
  for v in wt base; do
    if [ $v = wt ]; then export LSA_KERNELS_SO=$WT; else unset LSA_KERNELS_SO; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --latency-steps 16 > $out/b_${v}_$i.log 2>&1 || { tail -20 $out/b_${v}_$i.log; exit 4; }
    echo "$v $i: $(grep '^{' $out/b_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "ms", d["ms_per_step"], "b1", d["b1_p50_tpot_ms"], "mid", d["mid_p50_tpot_ms"])')"
  done
done
