#!/usr/bin/env python3
"""A/B of two gemm_sk builds in ONE process on ONE box (box-to-box spread is ~10 %): the in-tree
library against llm_sharding_amd/_native/liblsa_gemm_sk_prev.so (a build of an older
gemm_sk.hip), interleaved rounds, cold weights, hipGraph-timed; engine epilogues.

usage: gemm_sk_ab.py M N K epi bn split bm [...]   (epi: 1 resid, 2 swiglu, 3 qkv-as-store)"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import timeit  # noqa: E402


def main():
    args = [int(v) for v in sys.argv[1:]]
    vp, i = ctypes.c_void_p, ctypes.c_int
    libs = {"new": hip.lib(), "prev": ctypes.CDLL(os.path.join(ROOT, "llm_sharding_amd", "_native",
                                                               "liblsa_gemm_sk_prev.so"))}
    libs["prev"].lsa_gemm_sk.argtypes = hip.lib().lsa_gemm_sk.argtypes
    ws = hip.SkWorkspace("cuda")
    for c in range(0, len(args), 7):
        M, N, K, epi, bn, split, bm = args[c:c + 7]
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        cols = N // 2 if epi == hip.EPI_SWIGLU else N
        out = torch.zeros(M, cols, dtype=torch.bfloat16, device="cuda")
        e = hip.EPI_STORE if epi == 3 else epi
        ep = hip.make_epi(out=out, resid=out, ldo=cols, ldr=cols)
        res = {"new": [], "prev": []}
        outs = {}
        for rnd in range(5):
            for name, L in libs.items():
                def run(j, L=L):
                    rc = L.lsa_gemm_sk(x.data_ptr(), K, wps[j % nbuf].data_ptr(), M, N, K, e, ctypes.byref(ep), bm, bn,
                                       0, hip.N_CU, 1, split, 8, ws.slab.data_ptr(), ws.counters.data_ptr(),
                                       ws.slab.numel(), ws.counters.numel(), torch.cuda.current_stream().cuda_stream)
                    assert rc == 0, rc
                res[name].append(timeit(run))
                if rnd == 0:
                    out.zero_()
                    run(0)
                    torch.cuda.synchronize()
                    outs[name] = out.clone()
        same = bool(torch.equal(outs["new"], outs["prev"]))
        med = {k: round(sorted(v)[len(v) // 2], 2) for k, v in res.items()}
        print(json.dumps({"M": M, "N": N, "K": K, "epi": epi, "bn": bn, "split": split, "bm": bm, "median_us": med,
                          "new_vs_prev": round(med["prev"] / med["new"], 3), "bitwise_equal": same}), flush=True)
        del wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
