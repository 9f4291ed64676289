#!/usr/bin/env python3
"""Batch-1 decode projections (gemv.hip, the tuned config per shape, fused RMSNorm / RoPE + KV /
SwiGLU / residual epilogues) on the Llama-2-7B shapes, 5 launches each with the weights rotated
beyond the Infinity Cache - the workload of one rocprofv3 --pmc pass (scripts/gpu_pmc_b1.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import EPIS, MODEL_SHAPES  # noqa: E402


def main():
    from llm_sharding_amd.config import llama2_7b
    from llm_sharding_amd.models.rope import rope_table
    hip.lib()
    cos, sin = rope_table(llama2_7b(), 1024, "cuda")
    M = 1
    for name, (N, K) in MODEL_SHAPES["llama2-7b"].items():
        epi = EPIS[name]
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        wts = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
        if epi == hip.EPI_QKV:
            q = torch.zeros(M, 4096, dtype=torch.bfloat16, device="cuda")
            kc = torch.zeros(1, 32, 1024, 128, dtype=torch.bfloat16, device="cuda")
            ep = hip.make_epi(out=q, k_cache=kc, v_cache=kc.clone(), slot=torch.zeros(1, dtype=torch.int32, device="cuda"),
                              pos=torch.full((1,), 100, dtype=torch.int32, device="cuda"), cos=cos, sin=sin, ldo=4096,
                              n_heads=32, n_kv=32, head_dim=128, t_max=1024)
        elif epi == hip.EPI_ARGMAX:
            ep = hip.make_epi(keys=torch.zeros(M, dtype=torch.int64, device="cuda"))
        elif epi == hip.EPI_SWIGLU:
            ep = hip.make_epi(out=torch.zeros(M, N // 2, dtype=torch.bfloat16, device="cuda"), ldo=N // 2)
        else:
            ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
        norm = epi in (hip.EPI_QKV, hip.EPI_SWIGLU, hip.EPI_ARGMAX)
        for i in range(5):
            hip.gemv(x, wts[i % nbuf], M, N, K, epi, ep, norm=norm)
        torch.cuda.synchronize()
        print(f"{name}: N={N} K={K} weight MB={N * K * 2 / 1e6:.1f}", flush=True)
        del wts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
