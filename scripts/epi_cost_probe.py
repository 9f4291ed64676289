#!/usr/bin/env python3
"""Cost of gemm_sk's fused epilogues: the same plan (the engine's tuned decomposition) timed with
a plain bf16 store vs the engine's epilogue (QKV: RoPE + KV append; SwiGLU; residual add with
the fused-RMSNorm sum-of-squares partials), weights rotated beyond the Infinity Cache.

usage: epi_cost_probe.py [route] [M,M,...]   route: through hip.gemm's dispatch (gemm_wr where the
route table sends the shape, as the engine runs it) instead of gemm_sk directly"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402


def timeit(fn, iters=20):
    """us per call, the calls captured in one hipGraph (eager launches can be host-bound: the
    host-side checks of a fused-epilogue call took longer than the kernel)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(3):
            fn(i)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for i in range(iters):
                fn(i)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / iters)
    return sorted(ts)[2]


def main():
    from llm_sharding_amd.config import llama2_7b
    from llm_sharding_amd.models.rope import rope_table
    hip.lib()
    cos, sin = rope_table(llama2_7b(), 4096, "cuda")
    ws = hip.SkWorkspace("cuda", grid=1024, bn=256)
    route = "route" in sys.argv[1:]
    ms = [int(x) for a in sys.argv[1:] if a != "route" for x in a.split(",")] or [512, 2048]

    def run(x, w, M, N, K, epi, ep):
        if route:
            hip.gemm(x, w, M, N, K, epi, ep, sk_ws=ws)
        else:
            hip.gemm_sk(x, w, M, N, K, epi, ep, ws=ws)
    for name, N, K in (("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008)):
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        for M in ms:
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
            t_store = timeit(lambda i: run(x, wps[i % nbuf], M, N, K, hip.EPI_STORE, st))
            t_epi = timeit(lambda i: run(x, wps[i % nbuf], M, N, K, epi, ep))
            t_epi0 = timeit(lambda i: run(x, wps[i % nbuf], M, N, K, epi, ep0))
            print(json.dumps({"shape": name, "M": M, "route": route,
                              "wr": hip.gemm_wr_plan(M, N, K, epi, ep) if route else None, "plan": list(hip.gemm_sk_plan(M, N, K)), "store_us": round(t_store, 2),
                              "engine_epilogue_us": round(t_epi, 2), "epilogue_without_norm_io_us": round(t_epi0, 2),
                              "epilogue_cost_pct": round(100 * (t_epi - t_store) / t_store, 1)}), flush=True)
        del wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
