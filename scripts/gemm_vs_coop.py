#!/usr/bin/env python3
"""Decode-size projections (M = 32/64/128 rows): the stream-K MFMA GEMM (gemm_sk.hip, with the
engine's fused-RMSNorm epilogues: ss_in on qkv / gate_up, ss_out on the residual projections)
against the cooperative GEMV (gemv_coop.hip, norm folded in), on Llama-2-7B / 70B shapes with
the real epilogues. Weights rotated beyond the Infinity Cache (bench_kernels.timeit). One JSON
line per (model, shape, M): coop time, best gemm_sk (bn, split, bm) and every candidate, and the
weight-stream rate of each.

usage: gemm_vs_coop.py [models] [rows]      e.g. gemm_vs_coop.py llama2-7b 32,64,96,128"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import EPIS, MODEL_HEADS, MODEL_SHAPES, timeit  # noqa: E402

DEV = "cuda"


def main():
    from llm_sharding_amd.models.rope import rope_table
    from llm_sharding_amd.config import llama2_7b
    cos, sin = rope_table(llama2_7b(), 1024, DEV)
    ws = hip.CoopWorkspace(DEV, slab_floats=1 << 26, groups=1 << 15)
    sk_ws = hip.SkWorkspace(DEV)
    models = sys.argv[1].split(",") if len(sys.argv) > 1 else ["llama2-7b"]
    rows = [int(r) for r in sys.argv[2].split(",")] if len(sys.argv) > 2 else [32, 64, 128]
    for model in models:
        for name, (N, K) in MODEL_SHAPES[model].items():
            epi = EPIS[name]
            if epi == hip.EPI_ARGMAX:
                continue
            nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
            wts = [packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
            for M in rows:
                x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
                ss = torch.zeros(M, K // 64, dtype=torch.float32, device=DEV)
                if K % 256 == 0:
                    hip.row_ss(x, M, ss)
                nh, nkv = MODEL_HEADS[model]
                norm = epi in (hip.EPI_QKV, hip.EPI_SWIGLU)
                if epi == hip.EPI_QKV:
                    q = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
                    kc = torch.zeros(M, nkv, 1024, 128, dtype=torch.bfloat16, device=DEV)
                    slot = torch.arange(M, dtype=torch.int32, device=DEV)
                    pos = torch.full((M,), 100, dtype=torch.int32, device=DEV)
                    kw = dict(out=q, k_cache=kc, v_cache=kc, slot=slot, pos=pos, cos=cos, sin=sin,
                              ldo=N, n_heads=nh, n_kv=nkv, head_dim=128, t_max=1024)
                    ep = hip.make_epi(**kw)
                    ep_sk = hip.make_epi(**kw, ss_in=ss, ss_eps=1e-5)
                elif epi == hip.EPI_SWIGLU:
                    out = torch.zeros(M, N // 2, dtype=torch.bfloat16, device=DEV)
                    ep = hip.make_epi(out=out, ldo=N // 2)
                    ep_sk = hip.make_epi(out=out, ldo=N // 2, ss_in=ss, ss_eps=1e-5)
                else:
                    out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
                    sso = torch.zeros(M, N // 64, dtype=torch.float32, device=DEV)
                    ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
                    ep_sk = hip.make_epi(out=out, resid=out, ldo=N, ldr=N, ss_out=sso)
                coop_us = timeit(lambda i: hip.gemv(x, wts[i % nbuf], M, N, K, epi, ep, norm=norm, ws=ws))
                res = []
                for bm in (128, 256):
                    for bn in (256, 192, 128):
                        if N % (16 if bn == 192 else bn) or (bn == 192 and epi == hip.EPI_RESID):
                            continue
                        for sp in (0, 1, 2, 3, 4, 6, 8):
                            t = timeit(lambda i: hip.gemm_sk(x, wts[i % nbuf], M, N, K, epi, ep_sk, bn=bn, grid=hip.N_CU,
                                                              dp=1, split=sp, ws=sk_ws, bm=bm))
                            res.append((round(t, 2), bn, sp, bm))
                res.sort()
                wb = N * K * 2
                print(json.dumps({"model": model, "shape": name, "N": N, "K": K, "M": M,
                                  "coop_us": round(coop_us, 2), "coop_TBps": round(wb / coop_us / 1e6, 2),
                                  "sk_us": res[0][0], "sk_TBps": round(wb / res[0][0] / 1e6, 2),
                                  "sk_cfg": res[0][1:], "all_sk": res}), flush=True)
            del wts
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
