set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ipcdbg
rm -f gpurun_out/ipcdbg/*
P=29611
timeout -k 5 60 python -u scripts/ipc_pipeline_check.py --rank 0 --port $P --streams 1 --timeout 8 > gpurun_out/ipcdbg/r0.log 2>&1 &
A=$!
timeout -k 5 60 python -u scripts/ipc_pipeline_check.py --rank 1 --port $P --streams 1 --timeout 8 > gpurun_out/ipcdbg/r1.log 2>&1 &
B=$!
wait $A; echo "r0 rc=$?"
wait $B; echo "r1 rc=$?"
