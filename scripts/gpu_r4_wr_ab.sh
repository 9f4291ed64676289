#!/bin/bash
# engine A/B of the gemm_wr qkv route on Llama-3.2-3B and Llama-2-13B at 512 sequences
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_wr_ab
mkdir -p $out
rm -f $out/*
for m in llama3.2-3b llama2-13b; do
  for wr in 0 1 0 1; do
    LSA_GEMM_WR=$wr timeout -k 10 300 python3 -u bench.py --model $m --steps 20 --warmup 5 --latency-steps 0 > $out/$m.log 2>&1 || { tail -20 $out/$m.log; exit 2; }
    echo "$m gemm_wr=$wr $(grep '^\[bench\] load' $out/$m.log) $(grep '^{' $out/$m.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["tokens_mb0_sha16"])')" | tee -a $out/ab.txt
  done
done
