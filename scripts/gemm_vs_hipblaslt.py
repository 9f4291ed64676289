#!/usr/bin/env python3
"""Prefill projection GEMMs: the hand-written MFMA GEMM (gemm.hip, fused epilogue) against
torch.matmul (hipBLASLt on ROCm, plain GEMM, no epilogue) at prompt-sized M."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import MODEL_SHAPES  # noqa: E402


def timeit(fn, iters=20):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    rows = [int(r) for r in sys.argv[1].split(",")] if len(sys.argv) > 1 else [384, 2048, 16384]
    ws = hip.CoopWorkspace("cuda", slab_floats=1 << 26, groups=1 << 15)
    for name, (N, K) in MODEL_SHAPES["llama2-7b"].items():
        if name == "lm_head":
            continue
        # rotate over copies totalling > 600 MB so the weights stream from HBM (beyond the
        # 256 MB Infinity Cache), as they do in a decode step
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        ws_ = [torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16) for _ in range(nbuf)]
        wps = [packing.pack_b(w) for w in ws_]
        for M in rows:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            ep = hip.make_epi(out=out, ldo=N)
            tn = 2 if N % 128 == 0 else 1
            sk = hip.gemm_split(M, N, K, tn)
            t_ours = timeit(lambda i: hip.gemm(x, wps[i % nbuf], M, N, K, hip.EPI_STORE, ep, tn=tn, sk=sk, ws=ws))
            t_blas = timeit(lambda i: torch.matmul(x, ws_[i % nbuf].t(), out=out))
            fl = 2.0 * M * N * K
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "cold_weights": True, "ours_us": round(t_ours, 2),
                              "ours_tflops": round(fl / t_ours / 1e6, 1), "hipblaslt_us": round(t_blas, 2),
                              "hipblaslt_tflops": round(fl / t_blas / 1e6, 1),
                              "hipblaslt_weight_TBps": round(N * K * 2 / t_blas / 1e6, 2)}), flush=True)
        del ws_, wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
