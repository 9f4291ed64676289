#!/usr/bin/env python3
"""Residual projections (o / down) at decode batch sizes: the engine's current path (gemm_sk
EPI_RESID with the fused-RMSNorm sums of squares, or its tuned EPI_PARTIAL plan) against
gemm_wr EPI_PARTIAL (K split) + lsa_resid_rmsnorm_partials, cold weights, both checked against
fp32. usage: wr_resid_probe.py [M,N,K ...]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip, packing  # noqa: E402


def timeit(fn, reps=20):
    fn(0)
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
    return round(ts[len(ts) // 2], 2)


def main():
    hip.lib()
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [
        (512, 4096, 4096), (512, 4096, 11008), (384, 4096, 4096), (384, 4096, 11008), (256, 4096, 11008)]
    ws = hip.SkWorkspace("cuda", grid=1024, bn=256)
    for M, N, K in shapes:
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        w0 = torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)
        wps = [packing.pack_b(w0)] + [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16))
                                      for _ in range(nbuf - 1)]
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        r0 = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        ref = r0.float() + x.float() @ w0.float().T
        h = r0.clone()
        ss = torch.empty(M, N // 64, device="cuda")
        part = torch.empty(8, 1024, N, device="cuda")
        res = {"M": M, "N": N, "K": K}
        ep = hip.make_epi(out=h, resid=h, ldo=N, ldr=N, ss_out=ss)

        def fused(r):
            hip.gemm(x, wps[r % nbuf], M, N, K, hip.EPI_RESID, ep, sk_ws=ws)
        h.copy_(r0)
        fused(0)
        torch.cuda.synchronize()
        res["sk_resid_fused"] = [timeit(fused), f"{((h.float() - ref).norm() / ref.norm()).item():.1e}"]
        pp = hip.gemm_sk_partial_plan(M, N, K)
        if pp:
            def skp(r, pp=pp):
                hip.gemm_sk(x, wps[r % nbuf], M, N, K, hip.EPI_PARTIAL, hip.make_epi(out=part, ldo=N), bn=pp[0],
                            grid=hip.N_CU, dp=0, split=pp[1], ws=ws, out_numel=part.numel())
                hip.resid_rmsnorm_partials(h, part, pp[1], M, 1e-5)
            res[f"sk_partial_bn{pp[0]}_s{pp[1]}"] = [timeit(skp)]
        for bn in (128, 256):
            for sp in (1, 2, 3, 4):
                if K // 256 < sp:
                    continue

                def wrp(r, bn=bn, sp=sp):
                    hip.gemm_wr(x, wps[r % nbuf], M, N, K, hip.EPI_PARTIAL, hip.make_epi(out=part, ldo=N), bn=bn,
                                split=sp, out_numel=part.numel())
                    hip.resid_rmsnorm_partials(h, part, sp, M, 1e-5)

                def wr_only(r, bn=bn, sp=sp):
                    hip.gemm_wr(x, wps[r % nbuf], M, N, K, hip.EPI_PARTIAL, hip.make_epi(out=part, ldo=N), bn=bn,
                                split=sp, out_numel=part.numel())
                h.copy_(r0)
                wrp(0)
                torch.cuda.synchronize()
                err = ((h.float() - ref).norm() / ref.norm()).item()
                res[f"wr_partial_bn{bn}_s{sp}"] = [timeit(wrp), timeit(wr_only), f"{err:.1e}"]
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
