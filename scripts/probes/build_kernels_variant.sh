#!/bin/bash
# Build an A/B variant of the kernel library with extra compile defines into build/probes/
# (never into llm_sharding_amd/_native/). Same flags as csrc/build.py. Select it at run time with
# LSA_KERNELS_SO=build/probes/liblsa_kernels_<name>.so (llm_sharding_amd/ops/hip.py).
#   usage: scripts/probes/build_kernels_variant.sh <name> [-DFOO=1 ...]
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
obj=build/probes/obj_$name
mkdir -p $obj
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics -fno-slp-vectorize"
for s in csrc/kernels/*.hip; do
  /opt/rocm/bin/hipcc $F "$@" -c $s -o $obj/$(basename $s).o &
  while [ "$(jobs -r | wc -l)" -ge 8 ]; do sleep 0.5; done
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $obj/*.o -o build/probes/liblsa_kernels_$name.so
python3 csrc/isa_audit.py build/probes/liblsa_kernels_$name.so
