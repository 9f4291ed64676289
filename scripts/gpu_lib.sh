#!/bin/bash
# Library-GEMM path: targeted GPU tests, then bench configurations around it.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import torch; print('blas', torch.backends.cuda.preferred_blas_library())" > gpurun_out/lib_blas.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v --timeout 120 \
    --timeout-method thread -k "qkv_rope or library or big_batch or golden or concurrent or multistage or server" \
    > gpurun_out/pt_lib.log 2>&1 || { tail -40 gpurun_out/pt_lib.log; exit 1; }
tail -3 gpurun_out/pt_lib.log
for cfg in "384 1" "512 1" "384 2" "256 2" "768 1" "128 3"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 32 --warmup 4 --batch $1 --streams $2 > gpurun_out/bl_b$1_s$2.log 2>&1 \
      || { tail -30 gpurun_out/bl_b$1_s$2.log; exit 2; }
  echo "b$1 s$2: $(grep '^\[bench\] load' gpurun_out/bl_b$1_s$2.log)"
done
