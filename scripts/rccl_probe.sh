set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 scripts/rccl_same_gpu_probe.py > gpurun_out/probe2.log 2>&1; echo "probe rc=$?"; tail -5 gpurun_out/probe2.log
