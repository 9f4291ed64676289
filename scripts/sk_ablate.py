#!/usr/bin/env python3
"""What bounds gemm_sk's main loop: the same configuration timed (hipGraph, cold weights) on
ablation builds of gemm_sk.hip (-DLSA_SK_ABLATE=n; outputs are garbage, only the time matters):
0 = production code, 1 = no counted DMA waits, 2 = no DMA, 3 = no MFMA, 4 = no loop barriers,
5 = A gathered as half-line fragment blocks (pre-swizzle layout), 6 = no A DMA, 7 = no weight DMA,
8 = DMA only (no LDS reads, no MFMA), 9 = non-temporal weight DMA, 10 = DMA + MFMA without LDS
reads, 11 = MFMA only.

    python scripts/sk_ablate.py --build                 (CPU host: hipcc every variant)
    python scripts/sk_ablate.py M N K bn split [...]    (GPU: one JSON line per config)"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = tuple(range(12))


NAMES = ["prod", "no_wait", "no_dma", "no_mfma", "no_barrier", "a_full_lines", "no_a_dma", "no_w_dma", "dma_only", "w_nt", "dma_mfma_no_reads", "mfma_only"]


def so(v):
    return os.path.join(ROOT, "llm_sharding_amd", "_native", f"liblsa_sk_abl{v}.so")


def build():
    for v in VARIANTS:
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                               f"-DLSA_SK_ABLATE={v}", "-I", os.path.join(ROOT, "csrc", "kernels"),
                               os.path.join(ROOT, "csrc", "kernels", "gemm_sk.hip"), "-o", so(v)])
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
    vp, i = ctypes.c_void_p, ctypes.c_int
    libs = {}
    for v in VARIANTS:
        L = ctypes.CDLL(so(v))
        L.lsa_gemm_sk.argtypes = [vp, i, vp, i, i, i, i, ctypes.POINTER(hip.EpiArgs), i, i, i, i, i, i, i, vp, vp,
                                  ctypes.c_longlong, i, i, vp]
        libs[v] = L
    ws = hip.SkWorkspace("cuda")
    for c in range(0, len(args), 5):
        M, N, K, bn, split = args[c:c + 5]
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
        ep = hip.make_epi(out=out, ldo=N)
        res = {}
        for v, L in libs.items():
            def run(it, L=L):
                rc = L.lsa_gemm_sk(x.data_ptr(), x.stride(0), wps[it % nbuf].data_ptr(), M, N, K, hip.EPI_STORE,
                                   ctypes.byref(ep), 256, bn, 0, hip.N_CU, 1, split, 8, ws.slab.data_ptr(),
                                   ws.counters.data_ptr(), ws.slab.numel(), ws.counters.numel(),
                                   torch.cuda.current_stream().cuda_stream)
                assert rc == 0, rc
            res[v] = round(timeit(run), 2)
        print(json.dumps({"M": M, "N": N, "K": K, "bn": bn, "split": split,
                          "us": {NAMES[v]: t for v, t in res.items()}}),
              flush=True)
        del wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
