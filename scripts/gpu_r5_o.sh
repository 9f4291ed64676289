#!/bin/bash
# Round 5: 65-128-row decode on the GEMM path (LSA_GEMV_MAX_ROWS=64) vs the coop GEMV for the
# large-hidden models: Llama-2-13B (batch-128 latency pass) and one Llama-2-70B 10-layer stage at
# 128 / 96 rows per micro-batch (8 micro-batches), alternating, 2 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_o}
mkdir -p $out
rm -rf $out/*
B="--ttft-lens 0 --extras="
for i in 1 2; do
  for v in gemm coop; do
    if [ $v = gemm ]; then export LSA_GEMV_MAX_ROWS=64; else unset LSA_GEMV_MAX_ROWS; fi
    timeout -k 10 300 python3 bench.py --model llama2-13b --steps 4 --warmup 2 --latency-steps 32 $B > $out/b13_${v}_$i.log 2>&1 || { tail -20 $out/b13_${v}_$i.log; exit 4; }
    echo "13B $v $i: $(grep '^{' $out/b13_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("mid", d["mid_p50_tpot_ms"])')"
    for bt in 128 96; do
      timeout -k 10 300 python3 bench.py --model llama2-70b --stage-layers 10 --microbatches 8 --batch $bt --steps 8 --warmup 2 --latency-steps 0 $B > $out/b70_${bt}_${v}_$i.log 2>&1 || { tail -20 $out/b70_${bt}_${v}_$i.log; exit 5; }
      echo "70B stage b$bt $v $i: $(grep '^{' $out/b70_${bt}_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("ms/step", d["ms_per_step"])')"
    done
  done
done
unset LSA_GEMV_MAX_ROWS
