#!/bin/bash
# Ablation builds of the fused batch-1 attention + o projection (csrc/kernels/attn_oproj.hip,
# LSA_AO_ABLATE 1..4) for scripts/attn_oproj_probe.py: probe_bin/liblsa_ao_ab<N>.so, never in _native/.
set -e
cd "$(dirname "$0")/../.."
mkdir -p probe_bin
for n in 0 1 2 3 4; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize \
      -Icsrc/kernels -DLSA_AO_ABLATE=$n csrc/kernels/attn_oproj.hip -o probe_bin/liblsa_ao_ab$n.so &
done
wait
ls -la probe_bin/liblsa_ao_ab*.so
