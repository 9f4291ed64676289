#!/bin/bash
# Probe build of the one-wave-per-SIMD GEMM experiment (scripts/probes/gemm_w4.hip, round 6;
# profiles/r6_gemm_w4.md) into probe_bin/ (git-ignored, travels with gpurun; never _native/).
set -e
cd "$(dirname "$0")/../.."
mkdir -p probe_bin
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics \
    -fno-slp-vectorize scripts/probes/gemm_w4.hip -o probe_bin/liblsa_gemm_w4.so
python3 csrc/isa_audit.py probe_bin/liblsa_gemm_w4.so
