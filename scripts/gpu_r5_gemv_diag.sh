#!/bin/bash
# GEMV nondeterminism diagnosis: the shared-body probe builds (SLP on / library flags / index-checked) and
# the library, config (2, 4, 8, 2) at 33 / 44 / 64 rows, 8 launches each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r5_gemv_diag
mkdir -p $out
rm -rf $out/*
bash scripts/probes/build_gemv_body.sh > $out/build.log 2>&1 || { tail -20 $out/build.log; exit 1; }
for lib in "" build/probes/liblsa_gemv_body_slp.so build/probes/liblsa_gemv_body.so build/probes/liblsa_gemv_body_chk.so; do
  name=$(basename "${lib:-library}")
  timeout -k 10 120 python3 scripts/gemv_det_probe.py ${lib:+--lib $lib} --only 2,4,8,2 --launches 8 > $out/$name.jsonl 2>&1
  rc=$?
  echo "== $name (rc $rc)"; cut -c1-220 $out/$name.jsonl
  [ $rc -le 1 ] || exit 2
done
