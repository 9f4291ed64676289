#!/usr/bin/env python3
"""Projection GEMMs at decode-batch and prompt-sized M: the engine's hand-written GEMM dispatch
(hip.gemm: gemm_wr.hip where its route applies, else gemm_sk.hip with the plan the engine uses;
plain-store epilogue) against torch.matmul
(hipBLASLt on ROCm, plain GEMM, no epilogue). Weights rotate over > 600 MB of copies so they
stream from HBM (beyond the 256 MB Infinity Cache) as in a decode step; both timed as
20 launches captured in one hipGraph (no host overhead).

usage: gemm_vs_hipblaslt.py [M,M,...] [model]   (default 384,512,768,2048,16384 llama2-7b)
One JSON line per (shape, M)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import MODEL_SHAPES, timeit  # noqa: E402


def main():
    rows = [int(r) for r in sys.argv[1].split(",")] if len(sys.argv) > 1 else [384, 512, 768, 2048, 16384]
    sk_ws = hip.SkWorkspace("cuda")
    model = sys.argv[2] if len(sys.argv) > 2 else "llama2-7b"
    for name, (N, K) in MODEL_SHAPES[model].items():
        if name == "lm_head":
            continue
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        ws_ = [torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16) for _ in range(nbuf)]
        wps = [packing.pack_b(w) for w in ws_]
        for M in rows:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            ref = torch.empty_like(out)
            ep = hip.make_epi(out=out, ldo=N)
            wr = hip.gemm_wr_plan(M, N, K, hip.EPI_STORE, ep)
            plan = ["gemm_wr", wr] if wr else list(hip.gemm_sk_plan(M, N, K))
            t_ours = timeit(lambda i: hip.gemm(x, wps[i % nbuf], M, N, K, hip.EPI_STORE, ep, sk_ws=sk_ws))
            t_blas = timeit(lambda i: torch.matmul(x, ws_[i % nbuf].t(), out=ref))
            hip.gemm(x, wps[0], M, N, K, hip.EPI_STORE, ep, sk_ws=sk_ws)
            torch.matmul(x, ws_[0].t(), out=ref)
            err = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
            fl = 2.0 * M * N * K
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "cold_weights": True, "plan": plan,
                              "ours_us": round(t_ours, 2), "ours_tflops": round(fl / t_ours / 1e6, 1),
                              "hipblaslt_us": round(t_blas, 2), "hipblaslt_tflops": round(fl / t_blas / 1e6, 1),
                              "speedup": round(t_blas / t_ours, 3), "relerr_vs_hipblaslt": float(f"{err:.2e}")}),
                  flush=True)
        del ws_, wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
