#!/bin/bash
# Round 5: GQA decode with K in registers and V-only LDS staging (product) vs the previous tree:
# GQA GPU tests, then Llama-3.2-3B at 512 sequences and one Llama-2-70B 10-layer stage, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_w}
mkdir -p $out
rm -rf $out/*
BASE=$PWD/llm_sharding_amd/_native/variants/liblsa_kernels_base.so
timeout -k 10 300 python -u -m pytest tests/ -m gpu -k "gqa or decode_mfma or llama32 or 3b" -q \
    --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
X="--ttft-lens 0 --extras= --latency-steps 0"
for i in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then export LSA_KERNELS_SO=$BASE; else unset LSA_KERNELS_SO; fi
    timeout -k 10 300 python3 bench.py --model llama3.2-3b --steps 20 --warmup 5 $X > $out/b3_${v}_$i.log 2>&1 || { tail -20 $out/b3_${v}_$i.log; exit 4; }
    timeout -k 10 300 python3 bench.py --model llama2-70b --stage-layers 10 --microbatches 8 --steps 8 --warmup 2 $X > $out/b70_${v}_$i.log 2>&1 || { tail -20 $out/b70_${v}_$i.log; exit 5; }
    echo "$v $i: 3B $(grep '^{' $out/b3_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')  70B-stage $(grep '^{' $out/b70_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
