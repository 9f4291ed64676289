set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 120 ./probe_bin/pk_hazard_probe > gpurun_out/r6/pk_hazard.txt 2>&1 || { tail -5 gpurun_out/r6/pk_hazard.txt; exit 1; }
tail -3 gpurun_out/r6/pk_hazard.txt
timeout -k 10 400 python -u scripts/slp_kernel_diff.py --out gpurun_out/r6/slp_kernel_diff.jsonl > gpurun_out/r6/slp_kernel_diff.log 2>&1 || { tail -30 gpurun_out/r6/slp_kernel_diff.log; exit 2; }
tail -2 gpurun_out/r6/slp_kernel_diff.log
