#!/bin/bash
# Round 5: decode attention with DPP / permlane-swap lane exchanges instead of ds_bpermute shuffles
# (product build) vs the previous build (LSA_KERNELS_SO=variants/liblsa_kernels_base.so):
# attention + engine GPU tests, then batch-1 / batch-128 latency alternating, 3 pairs, and a
# kernel trace of the batch-1 pass on the product build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_l}
mkdir -p $out
rm -rf $out/*
BASE=$PWD/llm_sharding_amd/_native/variants/liblsa_kernels_base.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "attention or attn or decode or graph" -q \
    --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
for i in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then export LSA_KERNELS_SO=$BASE; else unset LSA_KERNELS_SO; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --latency-steps 64 > $out/b_${v}_$i.log 2>&1 || { tail -20 $out/b_${v}_$i.log; exit 4; }
    echo "$v $i: $(grep '^{' $out/b_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "b1", d["b1_p50_tpot_ms"], "mid", d["mid_p50_tpot_ms"])')"
  done
done
unset LSA_KERNELS_SO
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 -u bench.py --steps 2 --warmup 1 --latency-steps 32 > $out/prof_bench.log 2>&1 || { tail -20 $out/prof_bench.log; exit 5; }
f=$(find $out/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/kstats.py "$f" attn_small 12 > $out/kstats.txt
head -12 $out/kstats.txt
rm -f "$f"
