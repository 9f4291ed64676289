#!/usr/bin/env python3
"""Experimental W-in-registers GEMM (csrc/kernels/gemm_wr.hip) vs gemm_sk: correctness against
fp32 torch and timing (cold weights: a ring of weight copies larger than the Infinity Cache).
usage: gemm_wr_probe.py [M,N,K ...]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip, packing  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for r in range(reps):
        e0.record()
        fn(r)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [
        (512, 12288, 4096), (512, 22016, 4096), (512, 4096, 11008), (512, 4096, 4096), (16384, 4096, 4096)]
    for M, N, K in shapes:
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        ws = [torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16) for _ in range(nbuf)]
        wps = [packing.pack_b(w) for w in ws]
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        ref = (x.float() @ ws[0].float().T)
        res = {"M": M, "N": N, "K": K}
        only = os.environ.get("WR_ONLY")  # "bn,grid": one configuration (profiling)
        cfgs = [tuple(int(v) for v in only.split(","))] if only else [(bn, 256) for bn in (128, 192, 256)]
        for bn, grid in cfgs:
            if N % bn:
                continue
            out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            epw = hip.make_epi(out=out, ldo=N)

            def run(r=0, bn=bn, grid=grid, epw=epw):
                hip.gemm_wr(x, wps[r % nbuf], M, N, K, hip.EPI_STORE, epw, bn=bn, grid=grid)
            run(0)
            torch.cuda.synchronize()
            err = ((out.float() - ref).norm() / ref.norm()).item()
            us = timeit(run)
            res[f"bn{bn}"] = [round(us, 2), round(2 * M * N * K / us / 1e6, 1), f"{err:.1e}"]
        if not only:  # gemm_sk's plan for the shape, same cold-weight ring
            out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            eps_ = hip.make_epi(out=out, ldo=N)
            ws_sk = hip.SkWorkspace("cuda")
            res["gemm_sk"] = round(timeit(lambda r=0: hip.gemm_sk(x, wps[r % nbuf], M, N, K, hip.EPI_STORE, eps_, ws=ws_sk)), 2)
            refo = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            res["hipblaslt"] = round(timeit(lambda r=0: torch.matmul(x, ws[r % nbuf].t(), out=refo)), 2)
        print(json.dumps(res), flush=True)
        del ws, wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
