#!/bin/bash
# Round 5: decode attention A/B - the 8-wave / 256-keys-per-trip kernel for every one-split decode
# grid (LSA_ATTN_SMALL_MAX_WGS=1000000) vs the default (only <= 128 (row, kv-head) items): headline,
# batch 1 and batch 128, alternating; plus the attention GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_g}
mkdir -p $out
rm -rf $out/*
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k attention -q --timeout 120 --timeout-method thread \
    > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
for i in 1 2; do
  for v in all default; do
    if [ $v = all ]; then export LSA_ATTN_SMALL_MAX_WGS=1000000; else unset LSA_ATTN_SMALL_MAX_WGS; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/b_${v}_$i.log 2>&1 || { tail -20 $out/b_${v}_$i.log; exit 4; }
    echo "$v $i: $(grep '^{' $out/b_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["b1_p50_tpot_ms"], d["mid_p50_tpot_ms"])')"
  done
done
unset LSA_ATTN_SMALL_MAX_WGS
