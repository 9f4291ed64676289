set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6/base_bench.log 2>&1 && tail -3 gpurun_out/r6/base_bench.log
