#!/bin/bash
# Build the shared-body GEMV probe libraries into probe_bin/ (git-ignored, travels with gpurun; never
# shipped in llm_sharding_amd/_native/). The first two use the library's compile flags
# (csrc/build.py: -fno-slp-vectorize) and are run by tests/test_gemv_determinism_gpu.py;
# liblsa_gemv_body_slp.so keeps SLP vectorisation on - the round-4 build that computed wrong rows
# nondeterministically (profiles/r5_gemv_nondeterminism.md) - for the diagnosis script only.
set -e
cd "$(dirname "$0")/../.."
mkdir -p probe_bin
F="-O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Icsrc/kernels"
/opt/rocm/bin/hipcc $F -fno-slp-vectorize scripts/probes/gemv_body_lib.hip -o probe_bin/liblsa_gemv_body.so &
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -DLSA_GEMV_CHK scripts/probes/gemv_body_lib.hip -o probe_bin/liblsa_gemv_body_chk.so &
/opt/rocm/bin/hipcc $F scripts/probes/gemv_body_lib.hip -o probe_bin/liblsa_gemv_body_slp.so &
wait
ls -la probe_bin/*.so
