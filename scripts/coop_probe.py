#!/usr/bin/env python3
"""Fixed-cost probe for the coop GEMV: time vs K for each split count at fixed N, M, config
(t = a + b*K separates per-launch latency from streaming rate)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import timeit  # noqa: E402

DEV = "cuda"
hip.lib()
ws_ = hip.CoopWorkspace(DEV, slab_floats=1 << 25)
for N, M, cfg in ((4096, 64, (1, 8, 4)), (4096, 32, (1, 8, 4)), (12288, 64, (1, 8, 4))):
    for K in (512, 1024, 2048, 4096, 8192):
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        ws = [packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
        out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
        ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
        row = {"N": N, "M": M, "K": K}
        for sk in (1, 2, 4, 8):
            c = cfg + (sk, 1)
            if c not in packing.coop_candidates(N // 16, K, M):
                continue
            row[f"coop_sk{sk}"] = round(timeit(lambda i: hip.gemv(x, ws[i % nbuf], M, N, K, hip.EPI_RESID, ep,
                                                                  coop=c, ws=ws_)), 2)
        best = min(timeit(lambda i: hip.gemv(x, ws[i % nbuf], M, N, K, hip.EPI_RESID, ep, tn=t, nw=n, u=u))
                   for t, n, u in packing.gemv_candidates(N // 16, K, M))
        row["gemv_best"] = round(best, 2)
        row["hbm_us_at_5TBps"] = round(N * K * 2 / 5e6, 2)
        print(json.dumps(row), flush=True)
        del ws
        torch.cuda.empty_cache()
