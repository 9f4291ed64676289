#!/usr/bin/env python3
"""What bounds skinny_gemm.hip: the same configuration timed (hipGraph, cold weights) on timing
builds (-DLSA_SKINNY_ABLATE=n, outputs garbage): 0 = production, 1 = no A loads, 2 = no weight
loads, 3 = loads only (no MFMA), 4 = no reduction / epilogue, 5 = barrier after the loop then
exit, 6 = reduction without the epilogue.

    python scripts/skinny_ablate.py --build                   (CPU host: hipcc every variant)
    python scripts/skinny_ablate.py M N K tn nwv depth sk [...] (GPU: one JSON line per config)"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = (0, 2, 4, 5, 6)
NAMES = ["prod", "no_a", "no_w", "loads_only", "no_epilogue", "barrier_exit", "reduce_no_epilogue"]


def so(v):
    return os.path.join(ROOT, "llm_sharding_amd", "_native", f"liblsa_skinny_abl{v}.so")


def build():
    for v in VARIANTS:
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                               f"-DLSA_SKINNY_ABLATE={v}", "-I", os.path.join(ROOT, "csrc", "kernels"),
                               os.path.join(ROOT, "csrc", "kernels", "skinny_gemm.hip"), "-o", so(v)])
        print("built", so(v))


def main():
    if sys.argv[1] == "--build":
        build()
        return
    import torch
    sys.path.insert(0, ROOT)
    from llm_sharding_amd.ops import hip, packing
    from scripts.bench_kernels import timeit
    args = [int(v) for v in sys.argv[1:]]
    vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    libs = {}
    for v in VARIANTS:
        L = ctypes.CDLL(so(v))
        L.lsa_skinny.argtypes = [vp, i, vp, vp, i, i, i, i, f, i, ctypes.POINTER(hip.EpiArgs), i, i, i, i, vp,
                                 ctypes.c_longlong, vp, i, vp]
        libs[v] = L
    ws = hip.CoopWorkspace("cuda", slab_floats=1 << 25)
    for c in range(0, len(args), 7):
        M, N, K, tn, nwv, depth, sk = args[c:c + 7]
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
        ep = hip.make_epi(out=out, ldo=N)
        res = {}
        for v in VARIANTS:
            L = libs[v]

            def run(j):
                rc = L.lsa_skinny(x.data_ptr(), K, None, wps[j % nbuf].data_ptr(), M, N, K, 0, 1e-5, hip.EPI_STORE,
                                  ctypes.byref(ep), tn, nwv, depth, sk, ws.slab.data_ptr(), ws.slab.numel(),
                                  ws.counters.data_ptr(), ws.counters.numel(), torch.cuda.current_stream().cuda_stream)
                assert rc == 0, rc
            res[NAMES[v]] = round(timeit(run), 2)
        print(json.dumps({"M": M, "N": N, "K": K, "cfg": [tn, nwv, depth, sk], "us": res,
                          "weight_TBps_prod": round(N * K * 2 / res["prod"] / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
