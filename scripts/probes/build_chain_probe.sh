#!/bin/bash
# Build the persistent-chain probe (scripts/probes/chain_probe.hip) into build/probes/ (never part
# of llm_sharding_amd/_native/); same flags as csrc/build.py.
set -e
cd "$(dirname "$0")/../.."
mkdir -p build/probes
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics \
    -fno-slp-vectorize -Icsrc/kernels scripts/probes/chain_probe.hip -o build/probes/libchain_probe.so
python3 csrc/isa_audit.py build/probes/libchain_probe.so
