set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
rm -f gpurun_out/probe/sk.jsonl
for cfg in "512 4096 4096 128 4" "512 4096 4096 128 0" "512 4096 11008 128 0" "512 12288 4096 192 3" "512 22016 4096 192 6" "16384 12288 4096 256 0" "4096 4096 4096 256 0"; do
  timeout -k 10 90 python -u scripts/sk_one.py $cfg >> gpurun_out/probe/sk.jsonl 2>> gpurun_out/probe/sk.err || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/probe/blas -o blas -- python3 -c "
import torch
for M, N, K in ((512, 4096, 4096), (512, 12288, 4096), (512, 22016, 4096), (512, 4096, 11008), (16384, 12288, 4096)):
    x = torch.randn(M, K, device='cuda').bfloat16(); w = torch.randn(N, K, device='cuda').bfloat16()
    for i in range(5): y = torch.matmul(x, w.t())
torch.cuda.synchronize()
" > gpurun_out/probe/blas.log 2>&1
echo rc=$?
