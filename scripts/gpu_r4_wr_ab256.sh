#!/bin/bash
# engine A/B of the gemm_wr routes at 256 sequences (Llama-3.2-3B, Llama-2-7B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${AB_OUT:-r4_wr_ab256}
mkdir -p $out
rm -f $out/*
for m in ${AB_MODELS:-llama3.2-3b llama2-7b}; do
  for wr in 0 1 0 1; do
    LSA_GEMM_WR=$wr timeout -k 10 300 python3 -u bench.py --model $m --batch 256 --steps 20 --warmup 5 --latency-steps 0 > $out/$m.log 2>&1 || { tail -20 $out/$m.log; exit 2; }
    echo "$m batch 256 gemm_wr=$wr $(grep '^\[bench\] load' $out/$m.log)" | tee -a $out/ab.txt
  done
done
