#!/usr/bin/env python3
"""Probe of the stream-K 65..128-row decode projection (scripts/probes/gemv_stream.hip, built into
probe_bin/ by scripts/probes/build_gemv_stream.sh; round 6, profiles/r6_gemv_stream.md): the
(column group, 64-k chunk) units dealt evenly to one workgroup per CU, activations through an
LDS-DMA ring, weights straight to registers, split groups finished by their last contributor.
Measured slower than the engine's coop GEMV (gemv_coop.hip) at every Llama-2-7B shape, so it is
not in the product library.

  stream_probe.py check                 numerics vs fp32 torch (global + per-tile + per-row
                                        error), every config, split-group hand-off, fused RMSNorm,
                                        every epilogue, row gathers, hipGraph replays, determinism
  stream_probe.py bench [models] [rows] coop (tuned) vs every stream config, real epilogues,
                                        weights rotated beyond the Infinity Cache
  stream_probe.py ablate [rows]         the product build against timing-only ablation builds
                                        (probe_bin/liblsa_stream_ab{4,5}.so: 4 = no memory traffic
                                        in the main loop, 5 = no split hand-off / epilogue)"""
import ctypes
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from llm_sharding_amd.utils.numerics import rel_err  # noqa: E402
from scripts.bench_kernels import EPIS, MODEL_HEADS, MODEL_SHAPES, timeit  # noqa: E402

DEV = "cuda"
# (mb, tnw, nw, kf, d) instantiated in scripts/probes/gemv_stream.hip (LSA_STREAM_CONFIGS) - keep in sync
STREAM_CONFIGS = [(8, 2, 4, 2, 6), (8, 1, 4, 2, 6), (8, 1, 8, 2, 6), (8, 2, 8, 2, 4), (8, 1, 8, 2, 8)]
_LIBS = {}


def load(name="liblsa_gemv_stream.so"):
    if name not in _LIBS:
        L = ctypes.CDLL(os.path.join(ROOT, "probe_bin", name), mode=ctypes.RTLD_LOCAL)
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.lsa_gemv_stream.argtypes = [vp, i, vp, vp, i, i, i, i, f, i, ctypes.POINTER(hip.EpiArgs), i, i, i, i, i,
                                      vp, vp, vp]
        L.lsa_gemv_stream.restype = ctypes.c_int
        _LIBS[name] = L
    return _LIBS[name]


def slab_floats(rows, tnw, nw, grid):
    """fp32 workspace: two partial slots per workgroup (fragment-native tiles + row sums of squares)."""
    mr = 16 * packing.row_blocks(rows)
    return 2 * grid * (tnw * nw * mr * 16 + mr)


def gemv_stream(x, wp, M, N, K, epi, ep, cfg, norm=False, eps=1e-5, a_rows=None, grid=0, ws=None, lib=None):
    """y = A @ W^T for 65..128 rows, ``cfg = (tnw, nw, kf, d)`` of STREAM_CONFIGS; the epilogues and
    fused RMSNorm of hip.gemv."""
    assert 65 <= M <= 128 and epi != hip.EPI_PARTIAL
    assert wp.numel() == N * K and x.shape[1] >= K and x.stride(1) == 1
    assert a_rows is not None or x.shape[0] >= M
    tnw, nw, kf, d = (int(v) for v in cfg)
    assert (8, tnw, nw, kf, d) in STREAM_CONFIGS, cfg
    tg = tnw * nw
    assert N % (16 * tg) == 0 and K % (32 * kf) == 0 and (epi != hip.EPI_SWIGLU or tnw % 2 == 0)
    grid = grid or hip.N_CU
    assert (N // 16 // tg) * (K // (32 * kf)) >= grid, "fewer chunks than workgroups"
    assert ws.slab.numel() >= slab_floats(M, tnw, nw, grid) and ws.counters.numel() >= N // 16 // tg
    rc = (lib or load()).lsa_gemv_stream(hip._p(x), x.stride(0), hip._p(a_rows), hip._p(wp), M, N, K, int(norm),
                                         float(eps), epi, ctypes.byref(ep), tnw, nw, kf, d, grid, hip._p(ws.slab),
                                         hip._p(ws.counters), hip._stream())
    assert rc == 0, f"lsa_gemv_stream: {rc}"

MODEL_SHAPES = dict(MODEL_SHAPES)
MODEL_SHAPES.setdefault("llama2-13b", {"qkv": (15360, 5120), "o": (5120, 5120), "gate_up": (27648, 5120),
                                      "down": (5120, 13824), "lm_head": (32000, 5120)})
HEADS = dict(MODEL_HEADS, **{"llama2-13b": (40, 40)})


def _rnd(*shape, scale=1.0, gen=None):
    return (torch.randn(*shape, generator=gen, device=DEV) * scale).to(torch.bfloat16)


def _rmsnorm(x, w, eps):
    xf = x.float()
    return xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def _ws(h):
    return h.CoopWorkspace(DEV, slab_floats=1 << 25, groups=1 << 14)


def check_every_config_norm_resid(cfg):
    """RESID epilogue with the fused RMSNorm (partial sums of squares combined across the
    contributors of a split group) for every config, at grids that give one workgroup several
    whole groups (grid 7), a tail + head per workgroup (256) and tiny segments (grid 200 at K 512)."""
    h = hip
    _, tnw, nw, kf, d = cfg
    tg = tnw * nw
    ws = _ws(h)
    tested = 0
    for M, N, K in ((100, 16 * tg * 24, 11008), (128, 16 * tg * 40, 4096), (65, 16 * tg * 64, 512)):
        x = _rnd(M, K)
        g = (1 + 0.1 * torch.randn(K, device=DEV)).to(torch.bfloat16)
        w = _rnd(N, K, scale=0.02)
        wp = packing.pack_b(packing.fold_norm(w, g))
        resid = _rnd(M, N)
        ref = resid.float() + _rmsnorm(x, g, 1e-5) @ w.float().T
        units = (N // 16 // tg) * (K // (32 * kf))
        for grid in (7, 200, 256):
            if units < grid:
                continue
            out = resid.clone()
            gemv_stream(x, wp, M, N, K, h.EPI_RESID, h.make_epi(out=out, resid=out, ldo=N, ldr=N), cfg[1:],
                          norm=True, grid=grid, ws=ws)
            assert rel_err(out, ref) < 8e-3, (cfg, M, N, K, grid)
            tested += 1
    assert tested >= 6
    assert int(ws.counters.abs().sum()) == 0


def check_swiglu_argmax_graph(cfg):
    """SwiGLU (gate / up tile pairs) and argmax epilogues at 128 rows replayed in a hipGraph,
    bitwise identical across replays."""
    h = hip
    M, I, H, V = 128, 2752, 4096, 8192
    x = _rnd(M, H)
    fn = (1 + 0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16)
    wg, wu = _rnd(I, H, scale=0.05), _rnd(I, H, scale=0.05)
    lm = _rnd(V, H, scale=0.02)
    out = torch.zeros(M, I, dtype=torch.bfloat16, device=DEV)
    keys = torch.zeros(M, dtype=torch.int64, device=DEV)
    tok = torch.zeros(M, dtype=torch.int32, device=DEV)
    wgu = packing.pack_b(packing.fold_norm(packing.fuse_gate_up(wg, wu), fn))
    wlm = packing.pack_b(lm)
    ws = _ws(h)

    def step():
        gemv_stream(x, wgu, M, 2 * I, H, h.EPI_SWIGLU, h.make_epi(out=out, ldo=I), cfg[1:], norm=True, ws=ws)
        gemv_stream(x, wlm, M, V, H, h.EPI_ARGMAX, h.make_epi(keys=keys), cfg[1:], ws=ws)
        h.argmax_finalize(keys, M, tok)

    if (2 * I) % (16 * cfg[1] * cfg[2]):
        return
    step()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    xn = _rmsnorm(x, fn, 1e-5)
    ref = F.silu(xn @ wg.float().T) * (xn @ wu.float().T)
    logits = x.float() @ lm.float().T
    first = None
    for _ in range(3):
        out.zero_()
        tok.fill_(-1)
        graph.replay()
        torch.cuda.synchronize()
        assert rel_err(out, ref) < 1e-2
        chosen = logits.gather(1, tok.long()[:, None])[:, 0]
        assert torch.all(logits.max(-1).values - chosen < 2e-2 * logits.abs().max())
        if first is None:
            first = out.clone()
        else:
            assert torch.equal(out, first)
    assert int(ws.counters.abs().sum()) == 0


def _rope_ref(t, pos, cos, sin):
    half = t.shape[-1] // 2
    c, s = cos[pos][:, None, :], sin[pos][:, None, :]
    t1, t2 = t[..., :half], t[..., half:]
    return torch.cat([t1 * c - t2 * s, t2 * c + t1 * s], dim=-1)


def check_qkv_rope_kv_append_rows(nh, nkv):
    """QKV epilogue (RoPE + KV-cache append) with the fused RMSNorm and a row gather (a_rows)."""
    from llm_sharding_amd.config import tiny
    from llm_sharding_amd.models.rope import rope_table
    h = hip
    hd, H, M, slots, T = 128, 4096, 96, 128, 256
    wq, wk, wv = _rnd(nh * hd, H, scale=0.05), _rnd(nkv * hd, H, scale=0.05), _rnd(nkv * hd, H, scale=0.05)
    src = _rnd(150, H)
    rows = torch.randperm(150, device=DEV)[:M].to(torch.int32)
    fn = (1 + 0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16)
    cos, sin = rope_table(tiny(head_dim=hd), T, DEV)
    slot = torch.randperm(slots, device=DEV)[:M].to(torch.int32)
    pos = torch.randint(0, T, (M,), device=DEV, dtype=torch.int32)
    q = torch.zeros(M, nh * hd, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(slots, nkv, T, hd, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    N = (nh + 2 * nkv) * hd
    wp = packing.pack_b(packing.fold_norm(packing.fuse_qkv(wq, wk, wv, nh, nkv, hd), fn))
    ep = h.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, cos=cos, sin=sin, ldo=nh * hd,
                    n_heads=nh, n_kv=nkv, head_dim=hd, t_max=T)
    gemv_stream(src, wp, M, N, H, h.EPI_QKV, ep, (2, 4, 2, 6), norm=True, a_rows=rows, ws=_ws(h))
    xf = _rmsnorm(src[rows.long()], fn, 1e-5)
    pl = pos.long()
    assert rel_err(q, _rope_ref((xf @ wq.float().T).view(M, nh, hd), pl, cos, sin).reshape(M, -1)) < 1e-2
    sl = slot.long()
    assert rel_err(kc[sl, :, pl], _rope_ref((xf @ wk.float().T).view(M, nkv, hd), pl, cos, sin)) < 1e-2
    assert rel_err(vc[sl, :, pl], (xf @ wv.float().T).view(M, nkv, hd)) < 1e-2


def check_deterministic_and_guards():
    """Same inputs -> bitwise-equal outputs over repeated launches (split groups summed in
    contributor order); host-side guards reject shapes the kernel does not tile."""
    h = hip
    M, N, K = 128, 4096, 11008
    x = _rnd(M, K)
    wp = packing.pack_b(_rnd(N, K, scale=0.02))
    ws = _ws(h)
    outs = []
    for _ in range(4):
        out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
        gemv_stream(x, wp, M, N, K, h.EPI_STORE, h.make_epi(out=out, ldo=N), (1, 4, 2, 6), ws=ws)
        outs.append(out)
    torch.cuda.synchronize()
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    assert rel_err(outs[0], x.float() @ packing.unpack_b(wp).float().T) < 8e-3
    _raises(lambda: gemv_stream(x, wp, 64, N, K, h.EPI_STORE, h.make_epi(out=outs[0], ldo=N), (1, 4, 2, 6), ws=ws))
    _raises(lambda: gemv_stream(x, wp, M, N, K, h.EPI_STORE, h.make_epi(out=outs[0], ldo=N), (3, 4, 2, 6), ws=ws))


def _raises(fn):
    try:
        fn()
    except Exception:
        return
    raise AssertionError("expected a guard to reject the call")


def check():
    for cfg in STREAM_CONFIGS:
        check_every_config_norm_resid(cfg)
        if cfg[1] % 2 == 0:
            check_swiglu_argmax_graph(cfg)
        print("ok", cfg, flush=True)
    for nh, nkv in ((32, 32), (24, 8)):
        check_qkv_rope_kv_append_rows(nh, nkv)
    check_deterministic_and_guards()
    print("check: all passed", flush=True)


def bench(argv):
    from llm_sharding_amd.models.rope import rope_table
    from llm_sharding_amd.config import llama2_7b
    cos, sin = rope_table(llama2_7b(), 1024, DEV)
    ws = hip.CoopWorkspace(DEV, slab_floats=1 << 26, groups=1 << 15)
    models = argv[0].split(",") if len(argv) > 0 else ["llama2-7b"]
    rows = [int(r) for r in argv[1].split(",")] if len(argv) > 1 else [128]
    check = os.environ.get("STREAM_CHECK", "1") == "1"
    for model in models:
        for name, (N, K) in MODEL_SHAPES[model].items():
            epi = EPIS[name]
            nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
            wts = [packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
            for M in rows:
                x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
                nh, nkv = HEADS[model]
                norm = epi in (hip.EPI_QKV, hip.EPI_SWIGLU, hip.EPI_ARGMAX)
                if epi == hip.EPI_QKV:
                    q = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
                    kc = torch.zeros(M, nkv, 1024, 128, dtype=torch.bfloat16, device=DEV)
                    slot = torch.arange(M, dtype=torch.int32, device=DEV)
                    pos = torch.full((M,), 100, dtype=torch.int32, device=DEV)
                    ep = hip.make_epi(out=q, k_cache=kc, v_cache=kc, slot=slot, pos=pos, cos=cos, sin=sin,
                                      ldo=N, n_heads=nh, n_kv=nkv, head_dim=128, t_max=1024)
                    outt = q
                elif epi == hip.EPI_SWIGLU:
                    outt = torch.zeros(M, N // 2, dtype=torch.bfloat16, device=DEV)
                    ep = hip.make_epi(out=outt, ldo=N // 2)
                elif epi == hip.EPI_ARGMAX:
                    outt = torch.zeros(M, dtype=torch.int64, device=DEV)
                    ep = hip.make_epi(keys=outt)
                else:
                    outt = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
                    ep = hip.make_epi(out=outt, resid=outt, ldo=N, ldr=N)
                coop_us = timeit(lambda i: hip.gemv(x, wts[i % nbuf], M, N, K, epi, ep, norm=norm, ws=ws))
                ref = None
                if check and epi in (hip.EPI_SWIGLU, hip.EPI_STORE):
                    hip.gemv(x, wts[0], M, N, K, epi, ep, norm=norm, ws=ws)
                    ref = outt.clone()
                res = []
                for (_, tnw, nw, kf, d) in STREAM_CONFIGS:
                    tg = tnw * nw
                    if N % (16 * tg) or (epi == hip.EPI_SWIGLU and tnw % 2) or (N // 16 // tg) * (K // 64) < hip.N_CU:
                        continue
                    cfg = (tnw, nw, kf, d)
                    t = timeit(lambda i: gemv_stream(x, wts[i % nbuf], M, N, K, epi, ep, cfg, norm=norm, ws=ws))
                    err = None
                    if ref is not None:
                        gemv_stream(x, wts[0], M, N, K, epi, ep, cfg, norm=norm, ws=ws)
                        err = float((outt.float() - ref.float()).norm() / ref.float().norm())
                    res.append({"cfg": cfg, "us": round(t, 2), "err_vs_coop": err})
                res.sort(key=lambda r: r["us"])
                wb = N * K * 2
                best = res[0] if res else None
                print(json.dumps({"model": model, "shape": name, "N": N, "K": K, "M": M,
                                  "coop_us": round(coop_us, 2), "coop_TBps": round(wb / coop_us / 1e6, 2),
                                  "stream_us": best and best["us"], "stream_cfg": best and best["cfg"],
                                  "stream_TBps": best and round(wb / best["us"] / 1e6, 2),
                                  "speedup": best and round(coop_us / best["us"], 3), "all": res}), flush=True)
            del wts
            torch.cuda.empty_cache()
    assert int(ws.counters.abs().sum()) == 0



ABL_SHAPES = {"qkv": (12288, 4096, hip.EPI_STORE), "o": (4096, 4096, hip.EPI_RESID),
              "gate_up": (22016, 4096, hip.EPI_SWIGLU), "down": (4096, 11008, hip.EPI_RESID)}
ABL_CFGS = [(1, 4, 2, 6), (1, 8, 2, 6), (2, 8, 2, 4), (1, 8, 2, 8)]


def ablate(argv):
    M = int(argv[0]) if argv else 128
    libs = {"stream": load()}
    for v in (4, 5):
        if os.path.exists(os.path.join(ROOT, "probe_bin", f"liblsa_stream_ab{v}.so")):
            libs[f"ab{v}"] = load(f"liblsa_stream_ab{v}.so")
    ws = hip.CoopWorkspace(DEV, slab_floats=1 << 26, groups=1 << 15)
    for name, (N, K, epi) in ABL_SHAPES.items():
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        wts = [packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
        out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
        ep = hip.make_epi(out=out, resid=out, ldo=N if epi != hip.EPI_SWIGLU else N // 2, ldr=N)
        row = {"shape": name, "M": M}
        row["coop_us"] = round(timeit(lambda i: hip.gemv(x, wts[i % nbuf], M, N, K, epi, ep, ws=ws)), 2)
        for cfg in ABL_CFGS:
            if epi == hip.EPI_SWIGLU and cfg[0] % 2:
                continue
            for tag, L in libs.items():
                row[f"{tag}{list(cfg)}"] = round(timeit(lambda i: gemv_stream(x, wts[i % nbuf], M, N, K, epi, ep, cfg,
                                                                              ws=ws, lib=L)), 2)
        print(json.dumps(row), flush=True)
        del wts
        torch.cuda.empty_cache()



if __name__ == "__main__":
    cmd, rest = (sys.argv[1], sys.argv[2:]) if len(sys.argv) > 1 else ("bench", [])
    {"check": lambda a: check(), "bench": bench, "ablate": ablate}[cmd](rest)
