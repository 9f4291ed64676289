#!/bin/bash
# Round 5: flash prefill with 4 waves x 32 query rows (LSA_PREFILL_RB=2: every K / V^T fragment
# read feeds two row blocks) vs 8 waves x 16 rows (default): prefill attention GPU tests with
# RB=2, the prefill-attention roofline bench, and batch-1 TTFT (latency sweep), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_u}
mkdir -p $out
rm -rf $out/*
LSA_PREFILL_RB=2 timeout -k 10 300 python -u -m pytest tests/ -m gpu -k "prefill or flash or full_depth or engine" -q \
    --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
for rb in 2 1; do
  LSA_PREFILL_RB=$rb timeout -k 10 200 python3 scripts/prefill_attn_bench.py > $out/roof_rb$rb.jsonl 2>&1 || { tail -20 $out/roof_rb$rb.jsonl; exit 3; }
  echo "rb$rb"; cat $out/roof_rb$rb.jsonl | cut -c1-200
done
for i in 1 2; do
  for rb in 2 1; do
    LSA_PREFILL_RB=$rb timeout -k 10 200 python3 scripts/latency_sweep.py --lengths 512,2048,4096 --decode-batches 1 --decode-steps 8 > $out/ttft_rb${rb}_$i.log 2>&1 || { tail -20 $out/ttft_rb${rb}_$i.log; exit 4; }
    echo "rb$rb $i: $(grep '^{' $out/ttft_rb${rb}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ttft_ms"])')"
  done
done
