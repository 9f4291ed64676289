#!/usr/bin/env python3
"""Decode-size projections (M = 32/64/128 rows): the prefill GEMM (+ its split-K) against the
tuned cooperative GEMV, on Llama-2-7B / 70B / 3.2-3B shapes with the real epilogues, plus the
standalone RMSNorm the GEMM path needs in front of QKV and gate/up. Weights rotated beyond
the Infinity Cache (bench_kernels.timeit). Prints one JSON line per (model, shape, M)."""
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
    models = sys.argv[1].split(",") if len(sys.argv) > 1 else ["llama2-7b"]
    for model in models:
        for name, (N, K) in MODEL_SHAPES[model].items():
            epi = EPIS[name]
            if epi == hip.EPI_ARGMAX:
                continue
            nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
            wts = [packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
            for M in (32, 64, 128):
                x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
                xn = torch.empty_like(x)
                out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
                nh, nkv = MODEL_HEADS[model]
                if epi == hip.EPI_QKV:
                    q = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
                    kc = torch.zeros(M, nkv, 1024, 128, dtype=torch.bfloat16, device=DEV)
                    slot = torch.arange(M, dtype=torch.int32, device=DEV)
                    pos = torch.full((M,), 100, dtype=torch.int32, device=DEV)
                    ep = hip.make_epi(out=q, k_cache=kc, v_cache=kc, slot=slot, pos=pos, cos=cos, sin=sin,
                                      ldo=N, n_heads=nh, n_kv=nkv, head_dim=128, t_max=1024)
                else:
                    ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
                norm = epi in (hip.EPI_QKV, hip.EPI_SWIGLU)
                coop_us = timeit(lambda i: hip.gemv(x, wts[i % nbuf], M, N, K, epi, ep, norm=norm, ws=ws))
                tn = 2 if N % 128 == 0 else 1
                res = []
                for sk in (1, 2, 3, 4, 6, 8):
                    if (K // 64) < sk * 2 or hip.gemm_slab_floats(M, N, sk) > ws.slab.numel():
                        continue

                    def run(i, sk=sk):
                        if norm:
                            hip.rmsnorm(x, None, xn, M, 1e-5, K)
                        hip.gemm(xn if norm else x, wts[i % nbuf], M, N, K, epi, ep, tn=tn, sk=sk, ws=ws)
                    res.append((round(timeit(run), 2), sk))
                res.sort()
                rms_us = timeit(lambda i: hip.rmsnorm(x, None, xn, M, 1e-5, K)) if norm else 0.0
                print(json.dumps({"model": model, "shape": name, "N": N, "K": K, "M": M,
                                  "coop_us": round(coop_us, 2), "coop_cfg": list(packing.proj_config(
                                      N // 16, M, need_even=epi == hip.EPI_SWIGLU, k=K)[1]),
                                  "gemm_us(incl_rmsnorm)": res[0][0], "gemm_sk": res[0][1], "rmsnorm_us": round(rms_us, 2),
                                  "all_gemm": res}), flush=True)
            del wts
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
