#!/usr/bin/env python3
"""Decode projections at 256-512 rows on the prefill GEMM with weights streamed from HBM
(rotated copies beyond the Infinity Cache), incl. the standalone RMSNorm for QKV / gate-up."""
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
    rows_list = [int(r) for r in sys.argv[1].split(",")] if len(sys.argv) > 1 else [256, 384, 512]
    for name, (N, K) in MODEL_SHAPES["llama2-7b"].items():
        epi = EPIS[name]
        if epi == hip.EPI_ARGMAX:
            continue
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        wts = [packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        for M in rows_list:
            x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
            xn = torch.empty_like(x)
            out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
            nh, nkv = MODEL_HEADS["llama2-7b"]
            if epi == hip.EPI_QKV:
                kc = torch.zeros(M, nkv, 256, 128, dtype=torch.bfloat16, device=DEV)
                slot = torch.arange(M, dtype=torch.int32, device=DEV)
                pos = torch.full((M,), 100, dtype=torch.int32, device=DEV)
                ep = hip.make_epi(out=out, k_cache=kc, v_cache=kc, slot=slot, pos=pos, cos=cos, sin=sin,
                                  ldo=N, n_heads=nh, n_kv=nkv, head_dim=128, t_max=256)
            else:
                ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
            norm = epi in (hip.EPI_QKV, hip.EPI_SWIGLU)
            tn = 2 if N % 128 == 0 else 1
            res = []
            for sk in (1, 2, 3, 4, 6, 8):
                if (K // 64) < sk * 8 or hip.gemm_slab_floats(M, N, sk) > ws.slab.numel():
                    continue

                def run(i, sk=sk):
                    if norm:
                        hip.rmsnorm(x, None, xn, M, 1e-5, K)
                    hip.gemm(xn if norm else x, wts[i % nbuf], M, N, K, epi, ep, tn=tn, sk=sk, ws=ws)
                res.append((round(timeit(run), 2), sk))
            res.sort()
            print(json.dumps({"shape": name, "M": M, "gemm_us": res[0][0], "sk": res[0][1],
                              "auto_sk": hip.gemm_split(M, N, K, tn), "us_per_row": round(res[0][0] / M, 3),
                              "all": res}), flush=True)
        del wts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
