#!/bin/bash
# Build the shared-body GEMV probe libraries (plain + index-checked) into build/probes/ (run on the
# GPU box or here; never shipped in llm_sharding_amd/_native/).
set -e
cd "$(dirname "$0")/../.."
mkdir -p build/probes
F="-O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Icsrc/kernels"
/opt/rocm/bin/hipcc $F scripts/probes/gemv_body_lib.hip -o build/probes/liblsa_gemv_body.so &
/opt/rocm/bin/hipcc $F -DLSA_GEMV_CHK scripts/probes/gemv_body_lib.hip -o build/probes/liblsa_gemv_body_chk.so &
wait
ls -la build/probes/*.so
