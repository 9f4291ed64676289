set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ipc
timeout -k 10 200 python -u -m pytest tests/test_ipc_ring_gpu.py -x -q -s --timeout 150 --timeout-method thread > gpurun_out/ipc/pytest.log 2>&1
echo rc=$?
