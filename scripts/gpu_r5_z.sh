#!/bin/bash
# Round 5: persistent-chain probe (one launch, run-ahead LDS-DMA loader, granule hand-offs) vs the
# library's decode GEMV launched per op, batch 1, Llama-2-7B weight chain.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_z}
mkdir -p $out
rm -rf $out/*
bash scripts/probes/build_chain_probe.sh > $out/build.log 2>&1 || { tail -20 $out/build.log; exit 2; }
timeout -k 10 120 python3 scripts/probes/chain_probe.py > $out/chain.log 2>&1 || { tail -20 $out/chain.log; exit 13; }
grep '^{' $out/chain.log
timeout -k 10 120 python3 scripts/probes/chain_probe.py > $out/chain2.log 2>&1 || { tail -20 $out/chain2.log; exit 14; }
grep '^{' $out/chain2.log
