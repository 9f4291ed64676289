#!/bin/bash
# gemm_wr ablation builds at the 7B qkv decode shape (M=512, bn 192) and M=16384 (bn 256)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r3_wr_ablate.jsonl
: > $O
for n in 0 5; do
  if [ $n = 0 ]; then unset WR_LIB; else export WR_LIB=llm_sharding_amd/_native/liblsa_wr_abl$n.so; fi
  echo "{\"ablate\": $n}" >> $O
  WR_ONLY=192,1,256 timeout -k 10 60 python scripts/gemm_wr_probe.py 512,12288,4096 >> $O 2>&1 || exit 3
  WR_ONLY=256,1,512 timeout -k 10 60 python scripts/gemm_wr_probe.py 16384,4096,4096 >> $O 2>&1 || exit 3
done
grep -v amdgpu.ids $O
