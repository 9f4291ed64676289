#!/usr/bin/env python3
"""Workload for rocprofv3 --pmc passes: the gemm_w4 probe kernel and the engine's GEMM (gemm_sk /
gemm_wr via hip.gemm) at one projection shape, 4 launches each after a warm-up, plain-store
epilogue. Summarise with scripts/pmc_summary.py.   usage: gemm_w4_pmc.py [M] [N] [K]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.gemm_w4_probe import gemm_w4  # noqa: E402

M, N, K = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (16384, 4096, 4096)))
w = torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)
wp = packing.pack_b(w)
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
ep = hip.make_epi(out=out, ldo=N)
ws = hip.SkWorkspace("cuda")
for _ in range(5):
    gemm_w4(x, wp, M, N, K, ep)
    hip.gemm(x, wp, M, N, K, hip.EPI_STORE, ep, sk_ws=ws)
torch.cuda.synchronize()
print("done", M, N, K)
