#!/bin/bash
# Probe build of the stream-K 65..128-row projection experiment (scripts/probes/gemv_stream.hip,
# round 6; profiles/r6_gemv_stream.md) into probe_bin/ (git-ignored, travels with gpurun; never
# _native/): the kernel and its timing-only ablation builds (-DLSA_STREAM_ABLATE=4 / 5).
set -e
cd "$(dirname "$0")/../.."
mkdir -p probe_bin
FLAGS="-O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics -fno-slp-vectorize -Icsrc/kernels"
/opt/rocm/bin/hipcc $FLAGS scripts/probes/gemv_stream.hip -o probe_bin/liblsa_gemv_stream.so &
for v in ${LSA_STREAM_ABLATE:-4 5}; do
    /opt/rocm/bin/hipcc $FLAGS -DLSA_STREAM_ABLATE=$v scripts/probes/gemv_stream.hip -o probe_bin/liblsa_stream_ab$v.so &
done
wait
python3 csrc/isa_audit.py probe_bin/liblsa_gemv_stream.so
