#!/bin/bash
# Round 5: write-through (sc1) stores of the fp32 split-K partials (coop EPI_PARTIAL: the 7B down
# at 65-128 rows; gemm_sk EPI_PARTIAL: 768-row down) vs the previous tree, alternating, 3 rounds:
# kernel GPU tests of the partial paths, then the latency passes (b1 / batch 128) and the headline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_p}
mkdir -p $out
rm -rf $out/*
BASE=$PWD/llm_sharding_amd/_native/variants/liblsa_kernels_base.so
timeout -k 10 300 python -u -m pytest tests/ -m gpu -k "partial or coop or resid" -q \
    --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
for i in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then export LSA_KERNELS_SO=$BASE; else unset LSA_KERNELS_SO; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --latency-steps 64 --ttft-lens 0 --extras= > $out/b_${v}_$i.log 2>&1 || { tail -20 $out/b_${v}_$i.log; exit 4; }
    echo "$v $i: $(grep '^{' $out/b_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "b1", d["b1_p50_tpot_ms"], "mid", d["mid_p50_tpot_ms"])')"
  done
done
