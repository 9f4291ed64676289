#!/usr/bin/env python3
"""The coop GEMV's ragged mode (sk = 0: no K split, tiles dealt evenly to one workgroup per CU)
against the tuned coop config at decode batch 65..128 on the Llama-2-7B projections with their
real epilogues, weights rotated beyond the Infinity Cache (bench_kernels.timeit). One JSON line
per (shape, rows): the tuned config's time and every ragged candidate's.

usage: coop_ragged_probe.py [rows,rows,...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import EPIS, MODEL_HEADS, MODEL_SHAPES, timeit  # noqa: E402

DEV = "cuda"


def main():
    from llm_sharding_amd.config import llama2_7b
    from llm_sharding_amd.models.rope import rope_table
    cos, sin = rope_table(llama2_7b(), 1024, DEV)
    rows = [int(r) for r in sys.argv[1].split(",")] if len(sys.argv) > 1 else [128]
    ws = hip.CoopWorkspace(DEV, slab_floats=1 << 25, groups=1 << 15)
    nh, nkv = MODEL_HEADS["llama2-7b"]
    for name, (N, K) in MODEL_SHAPES["llama2-7b"].items():
        epi = EPIS[name]
        even = epi == hip.EPI_SWIGLU
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        wts = [packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        for M in rows:
            x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
            norm = epi in (hip.EPI_QKV, hip.EPI_SWIGLU)
            if epi == hip.EPI_QKV:
                q = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
                kc = torch.zeros(M, nkv, 1024, 128, dtype=torch.bfloat16, device=DEV)
                ep = hip.make_epi(out=q, k_cache=kc, v_cache=kc, slot=torch.arange(M, dtype=torch.int32, device=DEV),
                                  pos=torch.full((M,), 100, dtype=torch.int32, device=DEV), cos=cos, sin=sin, ldo=N,
                                  n_heads=nh, n_kv=nkv, head_dim=128, t_max=1024)
            elif epi == hip.EPI_SWIGLU:
                ep = hip.make_epi(out=torch.zeros(M, N // 2, dtype=torch.bfloat16, device=DEV), ldo=N // 2)
            elif epi == hip.EPI_ARGMAX:
                ep = hip.make_epi(keys=torch.zeros(M, dtype=torch.int64, device=DEV))
            else:
                out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
                ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
            algo, tuned = packing.proj_config(N // 16, M, even, K)
            t_tuned = timeit(lambda i: hip.gemv(x, wts[i % nbuf], M, N, K, epi, ep, norm=norm, ws=ws))
            res = []
            for c in packing.coop_candidates(N // 16, K, M, even):
                if c[3] != 0:
                    continue
                t = timeit(lambda i: hip.gemv(x, wts[i % nbuf], M, N, K, epi, ep, norm=norm, coop=c, ws=ws))
                res.append((round(t, 2), list(c)))
            res.sort()
            print(json.dumps({"shape": name, "M": M, "tuned": [algo, list(tuned)], "tuned_us": round(t_tuned, 2),
                              "ragged_best": res[0] if res else None,
                              "gain": round(t_tuned / res[0][0], 3) if res else None, "ragged_all": res}), flush=True)
        del wts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
