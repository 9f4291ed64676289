#!/usr/bin/env python3
"""Batch-1 decode GEMVs (7B shapes, the engine's tuned configs): what the fused epilogue costs
over a plain store. 32 weight copies per shape (cold, as in the decode step), one hipGraph of 32
launches per variant, us per launch (median of 15 replays).

  o / down   EPI_STORE vs EPI_RESID (in place on the residual stream, as the engine runs it)
  qkv        EPI_STORE vs EPI_QKV (RoPE + KV-cache append at pos / slot), RMSNorm folded in
  gate_up    EPI_SWIGLU (reference point; no epilogue loads)
usage: gemv_epi_probe.py [rows]   (default 1)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.config import llama2_7b  # noqa: E402
from llm_sharding_amd.models.rope import rope_table  # noqa: E402
from llm_sharding_amd.ops import hip, packing  # noqa: E402

DEV = "cuda"
hip.lib()
M = int(sys.argv[1]) if len(sys.argv) > 1 else 1
L = 32
cfg = llama2_7b()
cos, sin = rope_table(cfg, 256, DEV)
H, I, nh, nkv, hd = 4096, 11008, 32, 32, 128
g = torch.Generator(device=DEV).manual_seed(0)
h = torch.randn(M, 11008, generator=g, device=DEV).to(torch.bfloat16)
kc = torch.zeros(M, nkv, 256, hd, dtype=torch.bfloat16, device=DEV)
vc = torch.zeros_like(kc)
q = torch.zeros(M, H, dtype=torch.bfloat16, device=DEV)
slot = torch.arange(M, dtype=torch.int32, device=DEV)
pos = torch.full((M,), 150, dtype=torch.int32, device=DEV)
out = torch.zeros(M, 2 * I, dtype=torch.bfloat16, device=DEV)


def graph_us(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for li in range(L):
            fn(li)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for li in range(L):
                fn(li)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ts = []
    for _ in range(15):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        gr.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / L)
    ts.sort()
    return round(ts[len(ts) // 2], 2)


for name, N, K in (("qkv", 3 * H, H), ("o", H, H), ("gate_up", 2 * I, H), ("down", H, I)):
    ws = [packing.pack_b((torch.randn(N, K, generator=g, device=DEV) * K ** -0.5).to(torch.bfloat16)) for _ in range(L)]
    x = h[:, :K]
    res = {"shape": name, "rows": M, "config": packing.proj_config(N // 16, M, need_even=name == "gate_up", k=K)}
    st = hip.make_epi(out=out, ldo=out.stride(0))
    if name != "gate_up":
        res["store"] = graph_us(lambda li: hip.gemv(x, ws[li], M, N, K, hip.EPI_STORE, st))
    if name in ("o", "down"):
        hr = h[:, :H]
        ep = hip.make_epi(out=hr, resid=hr, ldo=h.stride(0), ldr=h.stride(0))
        res["resid"] = graph_us(lambda li: hip.gemv(x, ws[li], M, N, K, hip.EPI_RESID, ep))
    elif name == "qkv":
        ep = hip.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, cos=cos, sin=sin, ldo=q.stride(0),
                          n_heads=nh, n_kv=nkv, head_dim=hd, t_max=256)
        res["qkv_norm"] = graph_us(lambda li: hip.gemv(x, ws[li], M, N, K, hip.EPI_QKV, ep, norm=True))
        res["store_norm"] = graph_us(lambda li: hip.gemv(x, ws[li], M, N, K, hip.EPI_STORE, st, norm=True))
    else:
        ep = hip.make_epi(out=out, ldo=out.stride(0))
        res["swiglu_norm"] = graph_us(lambda li: hip.gemv(x, ws[li], M, N, K, hip.EPI_SWIGLU, ep, norm=True))
        res["store_norm"] = graph_us(lambda li: hip.gemv(x, ws[li], M, N, K, hip.EPI_STORE, st, norm=True))
    print(json.dumps(res), flush=True)
    del ws
