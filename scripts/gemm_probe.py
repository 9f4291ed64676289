#!/usr/bin/env python3
"""Run ONE gemm_sk configuration repeatedly (for rocprofv3 counter passes).

usage: gemm_probe.py M N K bn grid dp split [iters]
Weights rotate over > 600 MB of copies (HBM-streamed, as in a decode step)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402


def main():
    M, N, K, bn, grid, dp, split = (int(v) for v in sys.argv[1:8])
    iters = int(sys.argv[8]) if len(sys.argv) > 8 else 20
    nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
    wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    ep = hip.make_epi(out=out, ldo=N)
    ws = hip.SkWorkspace("cuda", grid=max(256, grid), bn=256)
    for i in range(iters):
        hip.gemm_sk(x, wps[i % nbuf], M, N, K, hip.EPI_STORE, ep, bn=bn, grid=grid, dp=dp, split=split, ws=ws)
    torch.cuda.synchronize()
    print("done", M, N, K, bn, grid, dp, split, flush=True)


if __name__ == "__main__":
    main()
