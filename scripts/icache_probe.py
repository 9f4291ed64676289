#!/usr/bin/env python3
"""Per-launch instruction-fetch cost (scripts/probes/icache_probe.hip): an unrolled block of
512..3072 independent VALU ops run once / twice / four times per launch, one wave on each of
256 CUs, hipGraph of 20 launches; cold = t(1) - (t(2) - t(1)) - t(empty). Build: python
scripts/icache_probe.py --build (CPU); run on the GPU without args."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "llm_sharding_amd", "_native", "liblsa_icache_probe.so")


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--build":
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950",
                               os.path.join(ROOT, "scripts", "probes", "icache_probe.hip"), "-o", SO])
        return
    import torch
    sys.path.insert(0, ROOT)
    from scripts.bench_kernels import timeit
    L = ctypes.CDLL(SO)
    L.run_icache.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    out = torch.zeros(64, device="cuda")
    def t(reps, nops):
        def run(i):
            assert L.run_icache(reps, nops, out.data_ptr(), 256, torch.cuda.current_stream().cuda_stream) == 0
        return timeit(run)
    empty = t(1, 8)
    for nops in (512, 1024, 2048, 3072):
        t1, t2, t4 = t(1, nops), t(2, nops), t(4, nops)
        warm = (t4 - t2) / 2
        print(json.dumps({"valu_ops": nops, "code_bytes_approx": nops * 8, "empty_launch_us": round(empty, 2),
                          "t1_us": round(t1, 2), "t2_us": round(t2, 2), "t4_us": round(t4, 2),
                          "warm_pass_us": round(warm, 2), "cold_fetch_extra_us": round(t1 - empty - warm, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
