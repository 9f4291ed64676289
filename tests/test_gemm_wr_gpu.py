"""gemm_wr.hip (weights streamed straight into MFMA B registers, 128 x bn tiles, A by LDS-DMA)
against plain PyTorch fp32 references: the store epilogue at every tile width and at row counts
that do and do not fill whole tiles / rounds, and the QKV epilogue (RoPE + KV-cache append) with
and without the fused RMSNorm row scale; plus the planner's dispatch from hip.gemm."""
import pytest
import torch

from llm_sharding_amd.ops import packing
from llm_sharding_amd.utils.numerics import rel_err  # global + per-16x16-tile + per-row

pytestmark = pytest.mark.gpu
DEV = "cuda"


def hip():
    from llm_sharding_amd.ops import hip as h
    h.lib()
    return h




def _rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(512, 12288, 4096), (300, 1536, 512), (1, 768, 256), (777, 1024, 1024),
                                   (129, 3072, 2816), (200, 768, 320), (64, 384, 64)])
@pytest.mark.parametrize("bn", [128, 192, 256])
@pytest.mark.parametrize("grid", [256, 37])
def test_gemm_wr_store(M, N, K, bn, grid):
    """K = 320 / 64 / 2816 leave a partial last group of K-steps (the ring holds 4). A width that
    does not tile N is refused on the host before anything launches (output left untouched)."""
    h = hip()
    a = _rnd(M, K)
    w = _rnd(N, K, scale=0.02)
    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
    if N % bn:
        with pytest.raises(ValueError, match="does not tile"):
            h.gemm_wr(a, packing.pack_b(w), M, N, K, h.EPI_STORE, h.make_epi(out=out, ldo=N), bn=bn, grid=grid)
        torch.cuda.synchronize()
        assert torch.isnan(out.float()).all()
        return
    h.gemm_wr(a, packing.pack_b(w), M, N, K, h.EPI_STORE, h.make_epi(out=out, ldo=N), bn=bn, grid=grid)
    assert rel_err(out, a.float() @ w.float().T) < 8e-3


def test_gemm_wr_strided_a():
    h = hip()
    M, N, K = 260, 768, 512
    big = _rnd(M, K + 64)
    a = big[:, 32:32 + K]
    w = _rnd(N, K, scale=0.02)
    out = torch.zeros(M, N + 8, dtype=torch.bfloat16, device=DEV)
    h.gemm_wr(a, packing.pack_b(w), M, N, K, h.EPI_STORE, h.make_epi(out=out, ldo=N + 8), bn=192)
    assert rel_err(out[:, :N], a.float() @ w.float().T) < 8e-3
    assert out[:, N:].abs().sum().item() == 0  # nothing written past N


def _rope_ref(t, pos, cos, sin):
    half = t.shape[-1] // 2
    c, s = cos[pos][:, None, :], sin[pos][:, None, :]
    t1, t2 = t[..., :half], t[..., half:]
    return torch.cat([t1 * c - t2 * s, t2 * c + t1 * s], dim=-1)


@pytest.mark.parametrize("nh,nkv,hd", [(32, 32, 128), (8, 2, 64), (24, 8, 128)])
@pytest.mark.parametrize("norm", [False, True])
@pytest.mark.parametrize("M", [300, 512])
@pytest.mark.parametrize("bn", [0, 256])
def test_gemm_wr_qkv_rope_kv_append(nh, nkv, hd, norm, M, bn):
    """bn 0: 192 where N tiles by it, else 128 (the routed widths); 256: the 13B route's width."""
    from llm_sharding_amd.config import tiny
    from llm_sharding_amd.models.rope import rope_table
    h = hip()
    H, slots, T, eps = 1024, 3, 512, 1e-5
    N = (nh + 2 * nkv) * hd
    bn = bn or (192 if N % 192 == 0 else 128)
    if N % bn:
        pytest.skip("N does not tile by bn")
    wq, wk, wv = _rnd(nh * hd, H, scale=0.05), _rnd(nkv * hd, H, scale=0.05), _rnd(nkv * hd, H, scale=0.05)
    x = _rnd(M, H)
    cos, sin = rope_table(tiny(head_dim=hd), T, DEV)
    slot = torch.randint(0, slots, (M,), device=DEV, dtype=torch.int32)
    pos = torch.randperm(T, device=DEV)[:M].to(torch.int32)
    q = torch.zeros(M, nh * hd, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(slots, nkv, T, hd, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    ss = None
    xf = x.float()
    if norm:  # per-64-column sums of squares of the raw residual stream (lsa_row_ss)
        ss = torch.empty(M, H // 64, device=DEV)
        h.row_ss(x, M, ss)
        xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    ep = h.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, cos=cos, sin=sin, ldo=nh * hd,
                    n_heads=nh, n_kv=nkv, head_dim=hd, t_max=T, ss_in=ss, ss_eps=eps)
    h.gemm_wr(x, packing.pack_b(packing.fuse_qkv(wq, wk, wv, nh, nkv, hd)), M, N, H, h.EPI_QKV, ep, bn=bn)
    pl, sl = pos.long(), slot.long()
    qr = _rope_ref((xf @ wq.float().T).view(M, nh, hd), pl, cos, sin).reshape(M, -1)
    kr = _rope_ref((xf @ wk.float().T).view(M, nkv, hd), pl, cos, sin)
    vr = (xf @ wv.float().T).view(M, nkv, hd)
    assert rel_err(q, qr) < 1e-2
    assert rel_err(kc[sl, :, pl], kr) < 1e-2
    assert rel_err(vc[sl, :, pl], vr) < 1e-2


@pytest.mark.parametrize("M,I,H", [(512, 8192, 3072), (300, 1024, 512), (129, 2048, 1024)])
@pytest.mark.parametrize("bn", [128, 256])
@pytest.mark.parametrize("norm", [False, True])
def test_gemm_wr_swiglu(M, I, H, bn, norm):
    """EPI_SWIGLU on gemm_wr (gate / up tiles interleaved by packing.fuse_gate_up), with and
    without the fused-RMSNorm row scale (ss_in), against fp32 silu(x W_g^T) * (x W_u^T)."""
    import torch.nn.functional as F
    h = hip()
    eps = 1e-5
    x = _rnd(M, H)
    wg, wu = _rnd(I, H, scale=0.05), _rnd(I, H, scale=0.05)
    xf = x.float()
    ss = None
    if norm:
        ss = torch.empty(M, H // 64, device=DEV)
        h.row_ss(x, M, ss)
        xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    out = torch.full((M, I), float("nan"), dtype=torch.bfloat16, device=DEV)
    ep = h.make_epi(out=out, ldo=I, ss_in=ss, ss_eps=eps)
    h.gemm_wr(x, packing.pack_b(packing.fuse_gate_up(wg, wu)), M, 2 * I, H, h.EPI_SWIGLU, ep, bn=bn)
    ref = F.silu(xf @ wg.float().T) * (xf @ wu.float().T)
    assert rel_err(out, ref) < 1e-2


def test_gemm_dispatches_wr_for_one_round_of_192_tiles(monkeypatch):
    """hip.gemm sends the 7B qkv shape at 384-512 rows to gemm_wr (one round of 192-256 whole tiles) and
    everything else to gemm_sk; LSA_GEMM_WR=0 turns it off."""
    h = hip()
    ep = h.make_epi(out=torch.empty(1, 1, device=DEV))
    assert h.gemm_wr_plan(512, 12288, 4096, h.EPI_QKV, ep) == 192
    assert h.gemm_wr_plan(384, 10240, 8192, h.EPI_QKV, ep) is None  # 70B qkv: measured a tie
    assert h.gemm_wr_plan(512, 12288, 4096, h.EPI_SWIGLU, ep) is None
    assert h.gemm_wr_plan(2048, 12288, 4096, h.EPI_QKV, ep) is None
    assert h.gemm_wr_plan(512, 4096, 4096, h.EPI_STORE, ep) is None
    monkeypatch.setenv("LSA_GEMM_WR", "0")
    assert h.gemm_wr_plan(512, 12288, 4096, h.EPI_QKV, ep) is None
    monkeypatch.delenv("LSA_GEMM_WR")
    calls = []
    real = h.gemm_wr
    monkeypatch.setattr(h, "gemm_wr", lambda *a, **k: (calls.append(a[1:5]), real(*a, **k)))
    M, N, K = 512, 12288, 4096
    a, w = _rnd(M, K), _rnd(N, K, scale=0.02)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    h.gemm(a, packing.pack_b(w), M, N, K, h.EPI_STORE, h.make_epi(out=out, ldo=N))
    assert calls and rel_err(out, a.float() @ w.float().T) < 8e-3
