#!/bin/bash
# Round 5: batch-1 decode attention issuing slot + length together and the first K/V trip before q
# (product build) vs the previous tree (variants/liblsa_kernels_base.so), with a control: the
# product sources built by scripts/probes/build_kernels_variant.sh (variants/liblsa_kernels_same.so)
# to measure any bias of loading a variant library. 3 rounds of product / same / base.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_m}
mkdir -p $out
rm -rf $out/*
V=$PWD/llm_sharding_amd/_native/variants
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "attention or attn or decode or graph" -q \
    --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
for i in 1 2 3; do
  for v in product same base; do
    if [ $v = product ]; then unset LSA_KERNELS_SO; else export LSA_KERNELS_SO=$V/liblsa_kernels_$v.so; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --latency-steps 64 --ttft-lens 0 > $out/b_${v}_$i.log 2>&1 || { tail -20 $out/b_${v}_$i.log; exit 4; }
    echo "$v $i: $(grep '^{' $out/b_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "b1", d["b1_p50_tpot_ms"], "mid", d["mid_p50_tpot_ms"])')"
  done
done
