#!/bin/bash
# Round 5: batch-1 decode with the 8-wave small-grid attention kernel (default) vs the 4-wave
# split kernel (LSA_ATTN_SMALL_MAX_WGS=0), alternating, 3 rounds (bench latency pass only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_t}
mkdir -p $out
rm -rf $out/*
for i in 1 2 3; do
  for v in small split; do
    if [ $v = split ]; then export LSA_ATTN_SMALL_MAX_WGS=0; else unset LSA_ATTN_SMALL_MAX_WGS; fi
    timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --latency-steps 128 --mid-batch 16 --ttft-lens 0 --extras= > $out/b_${v}_$i.log 2>&1 || { tail -20 $out/b_${v}_$i.log; exit 4; }
    echo "$v $i: $(grep '^{' $out/b_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("b1", d["b1_p50_tpot_ms"], "b16", d["mid_p50_tpot_ms"])')"
  done
done
