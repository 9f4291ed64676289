#!/usr/bin/env python3
"""Projection GEMMs above 128 rows: gemm_sk.hip (LDS-DMA 256 x BN tiles, stream-K, fused
epilogue) against torch.matmul (hipBLASLt, plain GEMM) on the same random data, weights rotated
over > 600 MB of copies so they stream from HBM as in a decode step.

usage: bench_gemm_sk.py [rows,rows,...] [--configs bn:grid:dp[:nb[:split]],...] [--model llama2-7b]
Prints one JSON line per (shape, M) with every config's time and the library's."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import MODEL_SHAPES  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for i in range(warm):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("rows", nargs="?", default="512,2048,16384")
    ap.add_argument("--configs", default="")
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--shapes", default="")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    rows = [int(r) for r in args.rows.split(",")]
    cfgs = [tuple(int(v) for v in c.split(":")) for c in args.configs.split(",") if c]
    ws = hip.SkWorkspace("cuda", grid=1024, bn=256)
    for name, (N, K) in MODEL_SHAPES[args.model].items():
        if name == "lm_head" or (args.shapes and name not in args.shapes.split(",")):
            continue
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        w_rm = [torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16) for _ in range(nbuf)]
        wps = [packing.pack_b(w) for w in w_rm]
        for M in rows:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            ref = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            ep = hip.make_epi(out=out, ldo=N)
            fl = 2.0 * M * N * K
            rec = {"shape": name, "M": M, "N": N, "K": K, "plan": list(hip.gemm_sk_plan(M, N, K))}
            todo = [(0, 0, 1, 0, -1)] + [c + (0, -1)[len(c) - 3:] if len(c) < 5 else c for c in cfgs]
            for (bn, grid, dp, nb, split) in todo:
                if bn and N % bn:
                    continue
                hip.gemm_sk(x, wps[0], M, N, K, hip.EPI_STORE, ep, bn=bn, grid=grid, dp=dp, nb=nb, split=split, ws=ws)
                torch.matmul(x, w_rm[0].t(), out=ref)
                torch.cuda.synchronize()
                err = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
                t = timeit(lambda i: hip.gemm_sk(x, wps[i % nbuf], M, N, K, hip.EPI_STORE, ep, bn=bn, grid=grid, dp=dp,
                                                 nb=nb, split=split, ws=ws), iters=args.iters)
                key = "sk" if (bn, grid, dp, nb, split) == (0, 0, 1, 0, -1) else f"sk_{bn}_{grid}_{dp}_{nb}_{split}"
                rec[key + "_us"] = round(t, 2)
                rec[key + "_tflops"] = round(fl / t / 1e6, 1)
                rec[key + "_relerr"] = float(f"{err:.2e}")
            t_blas = timeit(lambda i: torch.matmul(x, w_rm[i % nbuf].t(), out=ref), iters=args.iters)
            rec["hipblaslt_us"] = round(t_blas, 2)
            rec["hipblaslt_tflops"] = round(fl / t_blas / 1e6, 1)
            print(json.dumps(rec), flush=True)
        del w_rm, wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
