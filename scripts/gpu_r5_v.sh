#!/bin/bash
# Round 5: Llama-2-13B 65-128-row decode on the MFMA GEMMs by default (StageEngine.MID_GEMM_SHAPES)
# vs the coop GEMV (LSA_GEMV_MAX_ROWS=128), alternating; engine GPU tests of the GEMM path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_v}
mkdir -p $out
rm -rf $out/*
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "gemm_path_below_128 or big_batch or coop_partials" -q \
    --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
for i in 1 2 3; do
  for v in default coop; do
    if [ $v = coop ]; then export LSA_GEMV_MAX_ROWS=128; else unset LSA_GEMV_MAX_ROWS; fi
    timeout -k 10 300 python3 bench.py --model llama2-13b --steps 4 --warmup 2 --latency-steps 32 --ttft-lens 0 --extras= > $out/b13_${v}_$i.log 2>&1 || { tail -20 $out/b13_${v}_$i.log; exit 4; }
    echo "13B $v $i: $(grep '^{' $out/b13_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("b1", d["b1_p50_tpot_ms"], "mid", d["mid_p50_tpot_ms"], "tok/s", d["value"])')"
  done
done
