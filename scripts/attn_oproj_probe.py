#!/usr/bin/env python3
"""Batch-1 decode: attention + o projection (+ residual) per layer, 7B shapes, 32 layers with
their own weights and caches (cold weights, as in the decode step), one hipGraph per variant.

  two      hip.attn (small-grid kernel) then hip.gemv EPI_RESID: the engine's two launches
  attn     the attention alone              gemv     the o projection alone
  fusedN   lsa_attn_oproj from probe_bin/liblsa_ao_abN.so (scripts/probes/build_attn_oproj_ab.sh):
           0 as shipped, 1 weights loaded after the wait, 2 no wait, 3 no attention, 4 no o work

One JSON line per (variant, context): us per layer (median of 15 graph replays).
usage: attn_oproj_probe.py [T,T,...]   (default 150,200)"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip, packing  # noqa: E402

DEV = "cuda"
hip.lib()
L, nh, nkv, hd, N = 32, 32, 32, 128, 4096
K = nh * hd
TMAX = 256
TS = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [150, 200]

g = torch.Generator(device=DEV).manual_seed(0)
wps = [packing.pack_b((torch.randn(N, K, generator=g, device=DEV) * K ** -0.5).to(torch.bfloat16)) for _ in range(L)]
kcs = [torch.randn(1, nkv, TMAX, hd, generator=g, device=DEV).to(torch.bfloat16) for _ in range(L)]
vcs = [torch.randn(1, nkv, TMAX, hd, generator=g, device=DEV).to(torch.bfloat16) for _ in range(L)]
q = torch.randn(1, K, generator=g, device=DEV).to(torch.bfloat16)
slot = torch.zeros(1, dtype=torch.int32, device=DEV)
pos = torch.zeros(1, dtype=torch.int32, device=DEV)
h = torch.randn(1, N, generator=g, device=DEV).to(torch.bfloat16)
att = torch.zeros(1, K, dtype=torch.bfloat16, device=DEV)
po, pl = torch.zeros(nh * hd, device=DEV), torch.zeros(nh, device=DEV)
sync = torch.zeros(4, dtype=torch.int32, device=DEV)
ep = hip.make_epi(out=h, resid=h, ldo=N, ldr=N)

libs = {}
for n in range(5):
    p = os.path.join(ROOT, "probe_bin", f"liblsa_ao_ab{n}.so")
    if os.path.exists(p):
        lib = ctypes.CDLL(p)
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        lib.lsa_attn_oproj.argtypes = [vp, i, vp, vp, vp, vp, vp, i, i, i, i, f, vp, vp, i, i,
                                       ctypes.POINTER(hip.EpiArgs), vp, i, vp]
        lib.lsa_attn_oproj.restype = i
        libs[n] = lib


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def fused(lib, li):
    rc = lib.lsa_attn_oproj(_p(q), K, _p(kcs[li]), _p(vcs[li]), _p(slot), _p(pos), None, nh, nkv, hd, TMAX,
                            hd ** -0.5, _p(att), _p(wps[li]), N, K, ctypes.byref(ep), _p(sync), 0,
                            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc


VARIANTS = {
    "two": lambda li: (hip.attn(q, kcs[li], vcs[li], slot, pos, 1, nh, nkv, hd, 1, po, pl, att),
                       hip.gemv(att, wps[li], 1, N, K, hip.EPI_RESID, ep)),
    "attn": lambda li: hip.attn(q, kcs[li], vcs[li], slot, pos, 1, nh, nkv, hd, 1, po, pl, att),
    "gemv": lambda li: hip.gemv(att, wps[li], 1, N, K, hip.EPI_RESID, ep),
}
for n, lib in libs.items():
    VARIANTS[f"fused{n}"] = (lambda lib_: lambda li: fused(lib_, li))(lib)


def graph_us(fn):
    sync.zero_()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for li in range(L):  # eager warm-up (first-launch costs out of the graph)
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
    return ts[len(ts) // 2], ts[0]


for T in TS:
    pos.fill_(T - 1)
    for name, fn in VARIANTS.items():
        med, best = graph_us(fn)
        print(json.dumps({"variant": name, "T": T, "us_per_layer": round(med, 2), "best": round(best, 2),
                          "sync": sync.tolist()}), flush=True)
