#!/usr/bin/env python3
"""Cost of gemm_sk's fused epilogues: the same plan (the engine's tuned decomposition) timed with
a plain bf16 store vs the engine's epilogue (QKV: RoPE + KV append; SwiGLU; residual add with
the fused-RMSNorm sum-of-squares partials), weights rotated beyond the Infinity Cache."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_gemm_sk import timeit  # noqa: E402


def main():
    from llm_sharding_amd.config import llama2_7b
    from llm_sharding_amd.models.rope import rope_table
    hip.lib()
    cos, sin = rope_table(llama2_7b(), 4096, "cuda")
    ws = hip.SkWorkspace("cuda", grid=1024, bn=256)
    for name, N, K in (("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008)):
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        for M in (512, 2048):
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
            st = hip.make_epi(out=out, ldo=N)
            if name == "qkv":
                q = torch.zeros(M, 4096, dtype=torch.bfloat16, device="cuda")
                kc = torch.zeros(M, 32, 8, 128, dtype=torch.bfloat16, device="cuda")
                vc = torch.zeros_like(kc)
                slot = torch.arange(M, dtype=torch.int32, device="cuda")
                pos = torch.full((M,), 5, dtype=torch.int32, device="cuda")
                ss = torch.rand(M, 64, device="cuda")
                epi, ep = hip.EPI_QKV, hip.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, cos=cos,
                                                    sin=sin, ldo=4096, n_heads=32, n_kv=32, head_dim=128, t_max=8,
                                                    ss_in=ss, ss_eps=1e-5)
            elif name == "gate_up":
                act = torch.zeros(M, N // 2, dtype=torch.bfloat16, device="cuda")
                ss = torch.rand(M, 64, device="cuda")
                epi, ep = hip.EPI_SWIGLU, hip.make_epi(out=act, ldo=N // 2, ss_in=ss, ss_eps=1e-5)
            else:
                h = torch.randn(M, N, device="cuda").to(torch.bfloat16)
                ss = torch.zeros(M, N // 64, device="cuda")
                epi, ep = hip.EPI_RESID, hip.make_epi(out=h, resid=h, ldo=N, ldr=N, ss_out=ss)
            # the same epilogue without the fused-RMSNorm side input / output
            if name == "qkv":
                ep0 = hip.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, cos=cos, sin=sin, ldo=4096,
                                   n_heads=32, n_kv=32, head_dim=128, t_max=8)
            elif name == "gate_up":
                ep0 = hip.make_epi(out=act, ldo=N // 2)
            else:
                ep0 = hip.make_epi(out=h, resid=h, ldo=N, ldr=N)
            t_store = timeit(lambda i: hip.gemm_sk(x, wps[i % nbuf], M, N, K, hip.EPI_STORE, st, ws=ws))
            t_epi = timeit(lambda i: hip.gemm_sk(x, wps[i % nbuf], M, N, K, epi, ep, ws=ws))
            t_epi0 = timeit(lambda i: hip.gemm_sk(x, wps[i % nbuf], M, N, K, epi, ep0, ws=ws))
            print(json.dumps({"shape": name, "M": M, "plan": list(hip.gemm_sk_plan(M, N, K)), "store_us": round(t_store, 2),
                              "engine_epilogue_us": round(t_epi, 2), "epilogue_without_norm_io_us": round(t_epi0, 2),
                              "epilogue_cost_pct": round(100 * (t_epi - t_store) / t_store, 1)}), flush=True)
        del wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
