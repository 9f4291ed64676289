set -o pipefail
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python scripts/gemm_wr_probe.py > gpurun_out/r3_wr_probe.jsonl 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r3_wr_probe.jsonl | tail -20; exit $rc
