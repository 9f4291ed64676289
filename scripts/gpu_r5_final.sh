#!/bin/bash
# Round 5 final check: full GPU suite, smoke, the driver's bench line (incl. the batch-1 TTFT
# probe), kernel trace of the headline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_final}
mkdir -p $out
rm -rf $out/*
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $out/pytest.log 2>&1
tail -12 $out/pytest.log
grep -q "Timeout\|Fatal Python\|core dumped" $out/pytest.log && exit 2
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 3; }
tail -1 $out/smoke.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 4; }
grep '^{' $out/bench.log | tail -1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 -u bench.py --steps 20 --warmup 5 --latency-steps 0 --ttft-lens 0 --extras= > $out/prof_bench.log 2>&1 || { tail -20 $out/prof_bench.log; exit 5; }
f=$(find $out/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/kstats.py "$f" flash_prefill 14 > $out/kstats.txt
head -12 $out/kstats.txt
rm -f "$f"
