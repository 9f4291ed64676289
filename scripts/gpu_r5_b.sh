#!/bin/bash
# Round 5: GPU suite on the -fno-slp-vectorize library, then the headline bench A/B against the
# previous (SLP-vectorised) build of the same sources (LSA_KERNELS_SO), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_b}
mkdir -p $out
rm -rf $out/*
bash scripts/probes/build_gemv_body.sh > $out/probe_build.log 2>&1 || { tail -20 $out/probe_build.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $out/pytest.log 2>&1
rc=$?
tail -15 $out/pytest.log
grep -q "Timeout\|Fatal Python\|core dumped" $out/pytest.log && exit 2
[ $rc -le 1 ] || exit 2
SLP=scripts/probes/bin/liblsa_kernels_slp.so
for i in 1 2; do
  for v in noslp slp; do
    if [ $v = slp ]; then export LSA_KERNELS_SO=$GRAFT_REPO_ROOT/$SLP; else unset LSA_KERNELS_SO; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench_${v}_$i.log 2>&1 || { tail -20 $out/bench_${v}_$i.log; exit 4; }
    echo "$v $i: $(grep '^{' $out/bench_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["b1_p50_tpot_ms"], d["mid_p50_tpot_ms"])')"
  done
done
unset LSA_KERNELS_SO
