"""skinny_gemm.hip (register-direct MFMA projection for 17..128 rows) against plain PyTorch fp32
references: every instantiated (mb, tn, nwv, depth) x legal split, every epilogue with and
without the fused input RMSNorm, row gathers, uneven K splits and hipGraph replays (the split
tickets reset themselves)."""
import pytest
import torch
import torch.nn.functional as F

from llm_sharding_amd.ops import packing

pytestmark = pytest.mark.gpu
DEV = "cuda"


def hip():
    from llm_sharding_amd.ops import hip as h
    h.lib()
    return h


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


def _rmsnorm(x, w, eps):
    xf = x.float()
    return xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()


ROWS = {2: (17, 32), 4: (33, 64), 8: (65, 100, 128)}


@pytest.mark.parametrize("cfg", packing.SKINNY_CONFIGS)
def test_skinny_every_config(cfg):
    """RESID + fused RMSNorm (sum(x^2) across waves and splits) for every split the host
    accepts, K = 11008 (344 steps: uneven over waves / splits), 4096 and 512."""
    h = hip()
    mb, tn, nwv, depth = cfg
    N = 16 * tn * 3
    ws = h.CoopWorkspace(DEV, slab_floats=1 << 22)
    tested = 0
    for M in ROWS[mb]:
        for K in (11008, 4096, 512):
            x = _rnd(M, K)
            g = (1 + 0.1 * torch.randn(K, device=DEV)).to(torch.bfloat16)
            w = _rnd(N, K, scale=0.02)
            wp = packing.pack_b(packing.fold_norm(w, g))
            resid = _rnd(M, N)
            ref = resid.float() + _rmsnorm(x, g, 1e-5) @ w.float().T
            ref_plain = x.float() @ w.float().T
            for c in packing.skinny_candidates(N // 16, K, M):
                if c[:3] != (tn, nwv, depth):
                    continue
                tested += 1
                out = resid.clone()
                h.gemv(x, wp, M, N, K, h.EPI_RESID, h.make_epi(out=out, resid=out, ldo=N, ldr=N), norm=True,
                       skinny=c, ws=ws)
                assert rel_err(out, ref) < 8e-3, (cfg, M, K, c)
                o2 = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
                h.gemv(x, packing.pack_b(w), M, N, K, h.EPI_STORE, h.make_epi(out=o2, ldo=N), skinny=c, ws=ws)
                assert rel_err(o2, ref_plain) < 8e-3, (cfg, M, K, c)
    assert tested > 0, cfg
    assert int(ws.counters.abs().sum()) == 0


@pytest.mark.parametrize("M", [24, 64, 128])
def test_skinny_swiglu_qkv_gather_graph(M):
    """SwiGLU (+ norm) and QKV (RoPE + KV append) epilogues with a row gather, replayed in a
    hipGraph three times."""
    from llm_sharding_amd.config import tiny
    from llm_sharding_amd.models.rope import rope_table
    h = hip()
    I, H, nh, nkv, hd, T = 512, 1024, 8, 2, 128, 256
    src = _rnd(M + 7, H)
    rows = torch.randperm(M + 7, device=DEV)[:M].to(torch.int32)
    x = src[rows.long()]
    gn = (1 + 0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16)
    wg, wu = _rnd(I, H, scale=0.05), _rnd(I, H, scale=0.05)
    wgu = packing.pack_b(packing.fold_norm(packing.fuse_gate_up(wg, wu), gn))
    wq, wk, wv = _rnd(nh * hd, H, scale=0.05), _rnd(nkv * hd, H, scale=0.05), _rnd(nkv * hd, H, scale=0.05)
    Nq = (nh + 2 * nkv) * hd
    wqkv = packing.pack_b(packing.fold_norm(packing.fuse_qkv(wq, wk, wv, nh, nkv, hd), gn))
    cos, sin = rope_table(tiny(head_dim=hd), T, DEV)
    slot = torch.arange(M, device=DEV, dtype=torch.int32)
    pos = torch.randint(0, T, (M,), device=DEV, dtype=torch.int32)
    q = torch.zeros(M, nh * hd, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(M, nkv, T, hd, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    act = torch.zeros(M, I, dtype=torch.bfloat16, device=DEV)
    ws = h.CoopWorkspace(DEV, slab_floats=1 << 22)
    cg = [c for c in packing.skinny_candidates(2 * I // 16, H, M, need_even=True) if c[3] > 1][0]
    cq = [c for c in packing.skinny_candidates(Nq // 16, H, M) if c[3] > 1][-1]

    def step():
        h.gemv(src, wgu, M, 2 * I, H, h.EPI_SWIGLU, h.make_epi(out=act, ldo=I), norm=True, a_rows=rows, skinny=cg,
               ws=ws)
        h.gemv(src, wqkv, M, Nq, H, h.EPI_QKV,
               h.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, cos=cos, sin=sin, ldo=nh * hd,
                          n_heads=nh, n_kv=nkv, head_dim=hd, t_max=T), norm=True, a_rows=rows, skinny=cq, ws=ws)

    step()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    xn = _rmsnorm(x, gn, 1e-5)
    ref_act = F.silu(xn @ wg.float().T) * (xn @ wu.float().T)
    half = hd // 2
    pl = pos.long()

    def rope(t):
        c, s = cos[pl][:, None, :], sin[pl][:, None, :]
        t1, t2 = t[..., :half], t[..., half:]
        return torch.cat([t1 * c - t2 * s, t2 * c + t1 * s], dim=-1)
    qr = rope((xn @ wq.float().T).view(M, nh, hd)).reshape(M, -1)
    kr = rope((xn @ wk.float().T).view(M, nkv, hd))
    vr = (xn @ wv.float().T).view(M, nkv, hd)
    for _ in range(3):
        act.zero_()
        q.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert rel_err(act, ref_act) < 1e-2
        assert rel_err(q, qr) < 1e-2
        sl = slot.long()
        assert rel_err(kc[sl, :, pl], kr) < 1e-2
        assert rel_err(vc[sl, :, pl], vr) < 1e-2
    assert int(ws.counters.abs().sum()) == 0


def test_skinny_rejects_bad_configs():
    h = hip()
    x = _rnd(40, 512)
    wp = packing.pack_b(_rnd(256, 512))
    out = torch.zeros(40, 256, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(Exception):  # tn = 3 is not instantiated
        h.gemv(x, wp, 40, 256, 512, h.EPI_STORE, h.make_epi(out=out, ldo=256), skinny=(3, 4, 4, 1))
    with pytest.raises(Exception):  # no argmax epilogue
        h.gemv(x, wp, 40, 256, 512, h.EPI_ARGMAX, h.make_epi(keys=torch.zeros(40, dtype=torch.int64, device=DEV)),
               skinny=(4, 4, 4, 1))
