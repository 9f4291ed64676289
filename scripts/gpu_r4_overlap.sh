#!/bin/bash
# decode attention on C CU-masked CUs beside the qkv GEMM on the rest: per-kernel times alone
# and concurrent (kernel trace), C = 8 .. 64
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_overlap2
mkdir -p $out
rm -rf $out/*
CUMASK_TRACE=8,16,24,32,64 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/masked -o run -- \
    python3 scripts/cumask_probe.py > $out/masked.log 2>&1
rc=$?
grep '^{' $out/masked.log
echo "probe exit $rc"
