#!/bin/bash
# Round 5: 65-128-row decode on the MFMA GEMM path (LSA_GEMV_MAX_ROWS=64: gemm_sk / gemm_wr with the
# fused-norm ss epilogues) vs the cooperative GEMV (default), batch-128 latency pass of the 7B bench and
# of the 70B / 13B / 3B bench, alternating; plus the engine test of that path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_i}
mkdir -p $out
rm -rf $out/*
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "gemm_path_below_128 or big_batch or coop_partials" -q \
    --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
for i in 1 2; do
  for v in gemm coop; do
    if [ $v = gemm ]; then export LSA_GEMV_MAX_ROWS=64; else unset LSA_GEMV_MAX_ROWS; fi
    timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --latency-steps 32 > $out/b7_${v}_$i.log 2>&1 || { tail -20 $out/b7_${v}_$i.log; exit 4; }
    echo "7B $v $i: $(grep '^{' $out/b7_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("b1", d["b1_p50_tpot_ms"], "mid", d["mid_p50_tpot_ms"])')"
  done
done
for m in llama3.2-3b llama2-13b; do
  for v in gemm coop; do
    if [ $v = gemm ]; then export LSA_GEMV_MAX_ROWS=64; else unset LSA_GEMV_MAX_ROWS; fi
    timeout -k 10 300 python3 bench.py --model $m --steps 4 --warmup 2 --latency-steps 16 > $out/b_${m}_${v}.log 2>&1 || { tail -20 $out/b_${m}_${v}.log; exit 5; }
    echo "$m $v: $(grep '^{' $out/b_${m}_${v}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("mid", d["mid_p50_tpot_ms"])')"
  done
done
unset LSA_GEMV_MAX_ROWS
