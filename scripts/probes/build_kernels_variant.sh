#!/bin/bash
# Build an A/B variant of the kernel library with extra compile defines into probe_bin/
# (git-ignored, travels to the GPU box; never into llm_sharding_amd/_native/). Same flags as
# csrc/build.py. Select it at run time with LSA_KERNELS_SO=probe_bin/liblsa_kernels_<name>.so
# (llm_sharding_amd/ops/hip.py).
#   usage: scripts/probes/build_kernels_variant.sh <name> [-DFOO=1 ...]
#   LSA_VARIANT_SLP=1: build WITH SLP vectorisation (the round-1..4 flags); the ISA audit then
#   only reports (such a library carries the VALU -> packed-FP32 pattern the product build forbids)
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
obj=build/probes/obj_$name
mkdir -p $obj probe_bin
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics"
[ -n "${LSA_VARIANT_SLP:-}" ] || F="$F -fno-slp-vectorize"
for s in csrc/kernels/*.hip; do
  /opt/rocm/bin/hipcc $F "$@" -c $s -o $obj/$(basename $s).o &
  while [ "$(jobs -r | wc -l)" -ge 8 ]; do sleep 0.5; done
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $obj/*.o -o probe_bin/liblsa_kernels_$name.so
if [ -n "${LSA_VARIANT_SLP:-}" ]; then
  python3 csrc/isa_audit.py probe_bin/liblsa_kernels_$name.so || true
else
  python3 csrc/isa_audit.py probe_bin/liblsa_kernels_$name.so
fi
