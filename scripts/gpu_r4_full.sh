#!/bin/bash
# round-4 check: full GPU suite, smoke, the driver's bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_full
mkdir -p $out
rm -f $out/*
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $out/pytest.log 2>&1; rc=$?
tail -15 $out/pytest.log
grep -q "Timeout\|Fatal Python\|core dumped" $out/pytest.log && exit 2
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 3; }
tail -2 $out/smoke.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 4; }
grep '^{' $out/bench.log | tail -1
