#!/usr/bin/env python3
"""Activation row-stride probe for the 32..128-row projections: same GEMM, A rows padded by
0 / 64 / 128 / 256 / 512 elements (row stride 8 KiB + pad). A power-of-two row stride sends every
row of one k column block to the same memory channel; this measures whether that matters.
One JSON line per (shape, M, kernel, pad)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import timeit  # noqa: E402

DEV = "cuda"
hip.lib()
cws = hip.CoopWorkspace(DEV, slab_floats=1 << 25)
for name, (N, K, epi) in {"qkv": (12288, 4096, hip.EPI_STORE), "o": (4096, 4096, hip.EPI_RESID),
                          "down": (4096, 11008, hip.EPI_RESID)}.items():
    nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
    ws = [packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
    for M in (64, 128):
        out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
        ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
        cands = {"coop": [("coop", c) for c in packing.coop_candidates(N // 16, K, M)],
                 "skinny": [("skinny", c) for c in packing.skinny_candidates(N // 16, K, M)]}
        for pad in (0, 64, 128, 256, 512):
            xb = torch.randn(M, K + pad, device=DEV).to(torch.bfloat16)
            x = xb[:, :K]
            for kern, cl in cands.items():
                best = None
                for algo, c in cl:
                    kw = {algo: c}
                    us = timeit(lambda i: hip.gemv(x, ws[i % nbuf], M, N, K, epi, ep, ws=cws, **kw))
                    if best is None or us < best[0]:
                        best = (us, c)
                print(json.dumps({"shape": name, "M": M, "kernel": kern, "pad": pad, "us": round(best[0], 2),
                                  "TBps": round(N * K * 2 / best[0] / 1e6, 2), "cfg": list(best[1])}), flush=True)
    del ws
    torch.cuda.empty_cache()
