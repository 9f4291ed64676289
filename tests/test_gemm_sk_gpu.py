"""gemm_sk.hip (LDS-DMA BM x BN tiles, BM = 256 / 128, BN = 256 / 192 / 128, data-parallel rounds + stream-K, fused epilogues)
against plain PyTorch fp32 references: every epilogue, both tile widths, grids that split tiles
between workgroups (stream-K partial slabs + last-arriver combine) and grids that do not."""
import pytest
import torch
import torch.nn.functional as F

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


@pytest.fixture(scope="module")
def ws():
    return hip().SkWorkspace(DEV, grid=1024, bn=256)


# (bn, grid, dp, split): planner default, whole-tile rounds + stream-K, pure stream-K, odd grids
# (bijective XCD remap), equal K splits of the remainder (2-, 3- and 8-way), 128-wide 2-buffer ring
# and 192-wide tiles (4 x 2 waves, uneven B-DMA split over the waves, partial last column tile)
CFGS = [(0, 0, 1, -1), (256, 256, 1, 0), (128, 256, 1, 0), (256, 37, 0, 0), (128, 13, 1, 0), (256, 1000, 0, 0),
        (256, 256, 1, 2), (128, 256, 0, 3), (256, 512, 1, 8), (128, 96, 1, 1), (192, 256, 1, 0), (192, 256, 1, 2),
        (192, 37, 0, 0)]


BMS = (256, 128)  # row tile heights (128: decode batches and odd M)


def _skip(bn, N):
    """bn = 192 takes any N % 16 == 0 (partial last tile); 128 / 256 need N % bn == 0."""
    return bn and N % (16 if bn == 192 else bn)


@pytest.mark.parametrize("M", [1, 64, 129, 256, 300, 512, 777])
@pytest.mark.parametrize("N,K", [(1024, 512), (512, 4096), (768, 1216)])
def test_gemm_sk_store_resid(M, N, K, ws):
    h = hip()
    a = _rnd(M, K)
    w = _rnd(N, K, scale=0.02)
    wp = packing.pack_b(w)
    ref = a.float() @ w.float().T
    r = _rnd(M, N)
    for bm in BMS:
        for (bn, grid, dp, split) in CFGS:
            if _skip(bn, N) or (bm == 128 and not bn):
                continue
            nb = 2 if (bn, grid) == (128, 96) else 0
            tiles = -(-M // bm) * -(-N // (bn or 256))
            if split > 0 and tiles * split > grid:
                continue
            out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
            h.gemm_sk(a, wp, M, N, K, h.EPI_STORE, h.make_epi(out=out, ldo=N), bn=bn, grid=grid, dp=dp, split=split,
                      nb=nb, ws=ws, bm=bm if bn else 0)
            assert rel_err(out, ref) < 8e-3, (bm, bn, grid, dp, split)
            o2 = r.clone()
            h.gemm_sk(a, wp, M, N, K, h.EPI_RESID, h.make_epi(out=o2, resid=o2, ldo=N, ldr=N), bn=bn, grid=grid, dp=dp,
                      split=split, nb=nb, ws=ws, bm=bm if bn else 0)
            assert rel_err(o2, r.float() + ref) < 8e-3, (bm, bn, grid, dp, split)
    assert int(ws.counters.abs().sum()) == 0  # every split tile's ticket was reset


def test_gemm_sk_strided_a_and_big_m(ws):
    """A with a row stride > K (a view into a wider buffer) and enough rows for several
    data-parallel rounds plus a stream-K tail."""
    h = hip()
    M, N, K = 4100, 1280, 320
    buf = _rnd(M, K + 64)
    a = buf[:, 32:32 + K]
    w = _rnd(N, K, scale=0.05)
    out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    h.gemm_sk(a, packing.pack_b(w), M, N, K, h.EPI_STORE, h.make_epi(out=out, ldo=N), bn=256, grid=16, ws=ws)
    assert rel_err(out, a.float() @ w.float().T) < 8e-3


@pytest.mark.parametrize("M", [96, 200, 512, 1030])
def test_gemm_sk_swiglu(M, ws):
    h = hip()
    I, H = 1024, 512
    x = _rnd(M, H)
    wg, wu = _rnd(I, H, scale=0.05), _rnd(I, H, scale=0.05)
    wp = packing.pack_b(packing.fuse_gate_up(wg, wu))
    ref = F.silu(x.float() @ wg.float().T) * (x.float() @ wu.float().T)
    for bm in BMS:
        for (bn, grid, dp, split) in CFGS:
            if bm == 128 and not bn:
                continue
            tiles = -(-M // bm) * -(-2 * I // (bn or 256))
            if split > 0 and tiles * split > grid:
                continue
            out = torch.zeros(M, I, dtype=torch.bfloat16, device=DEV)
            h.gemm_sk(x, wp, M, 2 * I, H, h.EPI_SWIGLU, h.make_epi(out=out, ldo=I), bn=bn, grid=grid, dp=dp,
                      split=split, ws=ws, bm=bm if bn else 0)
            assert rel_err(out, ref) < 1e-2, (bm, bn, grid, dp, split)


def _rope_ref(t, pos, cos, sin):
    half = t.shape[-1] // 2
    c, s = cos[pos][:, None, :], sin[pos][:, None, :]
    t1, t2 = t[..., :half], t[..., half:]
    return torch.cat([t1 * c - t2 * s, t2 * c + t1 * s], dim=-1)


@pytest.mark.parametrize("nh,nkv,hd", [(32, 32, 128), (8, 2, 64), (24, 8, 128)])
@pytest.mark.parametrize("cfg", [(0, 0, 1, -1), (128, 29, 0, 0), (256, 256, 1, 3), (192, 256, 1, 2),
                                 (128, 256, 1, 3, 128), (192, 256, 1, 2, 128), (256, 37, 0, 0, 128)])
def test_gemm_sk_qkv_rope_kv_append(nh, nkv, hd, cfg, ws):
    from llm_sharding_amd.config import tiny
    from llm_sharding_amd.models.rope import rope_table
    h = hip()
    H, M, slots, T = 512, 300, 3, 512
    wq, wk, wv = _rnd(nh * hd, H, scale=0.05), _rnd(nkv * hd, H, scale=0.05), _rnd(nkv * hd, H, scale=0.05)
    x = _rnd(M, H)
    cos, sin = rope_table(tiny(head_dim=hd), T, DEV)
    slot = torch.randint(0, slots, (M,), device=DEV, dtype=torch.int32)
    pos = torch.randperm(T, device=DEV)[:M].to(torch.int32)
    q = torch.zeros(M, nh * hd, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(slots, nkv, T, hd, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    wp = packing.pack_b(packing.fuse_qkv(wq, wk, wv, nh, nkv, hd))
    N = (nh + 2 * nkv) * hd
    ep = h.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, cos=cos, sin=sin, ldo=nh * hd,
                    n_heads=nh, n_kv=nkv, head_dim=hd, t_max=T)
    bn, grid, dp, split = cfg[:4]
    if _skip(bn, N):
        pytest.skip("N not a multiple of bn")
    h.gemm_sk(x, wp, M, N, H, h.EPI_QKV, ep, bn=bn, grid=grid, dp=dp, split=split, ws=ws,
              bm=cfg[4] if len(cfg) > 4 else 0)
    xf, pl, sl = x.float(), pos.long(), slot.long()
    qr = _rope_ref((xf @ wq.float().T).view(M, nh, hd), pl, cos, sin).reshape(M, -1)
    kr = _rope_ref((xf @ wk.float().T).view(M, nkv, hd), pl, cos, sin)
    vr = (xf @ wv.float().T).view(M, nkv, hd)
    assert rel_err(q, qr) < 1e-2
    assert rel_err(kc[sl, :, pl], kr) < 1e-2
    assert rel_err(vc[sl, :, pl], vr) < 1e-2


def test_gemm_sk_graph_replay(ws):
    """Captured in a hipGraph and replayed: the self-resetting tickets must leave every replay
    identical to the eager result."""
    h = hip()
    M, N, K = 512, 4096, 1024
    a = _rnd(M, K)
    w = _rnd(N, K, scale=0.02)
    wp = packing.pack_b(w)
    out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    ep = h.make_epi(out=out, ldo=N)
    h.gemm_sk(a, wp, M, N, K, h.EPI_STORE, ep, bn=128, grid=256, ws=ws)
    torch.cuda.synchronize()
    first = out.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        h.gemm_sk(a, wp, M, N, K, h.EPI_STORE, ep, bn=128, grid=256, ws=ws)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert rel_err(out, first) < 1e-6
    assert rel_err(first, a.float() @ w.float().T) < 8e-3


@pytest.mark.parametrize("M,N,K,bn,S", [(512, 4096, 4096, 128, 4), (300, 4096, 1216, 256, 3), (777, 2048, 640, 192, 2),
                                        (129, 8192, 512, 128, 1), (256, 4096, 11008, 128, 8)])
def test_gemm_sk_partials_resid_rmsnorm(M, N, K, bn, S, ws):
    """EPI_PARTIAL (each K range's fp32 partial stored, no in-GEMM fixup) + the fused residual
    add / RMSNorm kernel that sums them, against fp32 torch."""
    h = hip()
    a = _rnd(M, K)
    w = _rnd(N, K, scale=0.02)
    r = _rnd(M, N)
    ref = a.float() @ w.float().T
    P = torch.full((h.PARTIAL_MAX_SPLIT, M, N), float("nan"), device=DEV)
    with pytest.raises(ValueError, match="partial"):  # capacity is checked before anything is written
        h.gemm_sk(a, packing.pack_b(w), M, N, K, h.EPI_PARTIAL, h.make_epi(out=P, ldo=N), bn=bn, grid=256, dp=0,
                  split=S, ws=ws, out_numel=(S - 1) * M * N)
    h.gemm_sk(a, packing.pack_b(w), M, N, K, h.EPI_PARTIAL, h.make_epi(out=P, ldo=N), bn=bn, grid=256, dp=0, split=S,
              ws=ws, out_numel=P.numel())
    assert rel_err(P[:S].sum(0), ref) < 1e-5
    assert bool(torch.isnan(P[S:]).all())  # nothing beyond the S partials is written
    hb, xn = r.clone(), torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    h.resid_rmsnorm_partials(hb, P, S, M, 1e-5, out=xn)
    want_h = r.float() + ref
    assert rel_err(hb, want_h) < 8e-3
    hf = hb.float()
    want_xn = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5)
    assert rel_err(xn, want_xn) < 8e-3
    h2 = r.clone()
    h.resid_rmsnorm_partials(h2, P, S, M, 1e-5)  # residual only (stage output)
    assert torch.equal(h2, hb)


@pytest.mark.parametrize("M,N,bn,bm", [(300, 4096, 256, 0), (512, 32000 // 128 * 128, 0, 0), (777, 2048, 128, 0),
                                       (100, 4096, 256, 128), (300, 2048, 128, 128)])
def test_gemm_sk_argmax(M, N, bn, bm, ws):
    """EPI_ARGMAX (lm_head + greedy argmax keys, 64-bit atomics) against torch.argmax of the fp32
    logits, with a column offset and a -huge bias column, wherever the top-2 margin is clear."""
    h = hip()
    K = 1024
    a = _rnd(M, K)
    w = _rnd(N, K, scale=0.05)
    bias = torch.zeros(N, device=DEV)
    bias[7] = -3.0e38
    keys = torch.zeros(M, dtype=torch.int64, device=DEV)
    h.gemm_sk(a, packing.pack_b(w), M, N, K, h.EPI_ARGMAX, h.make_epi(keys=keys, col_offset=100, bias=bias), bn=bn,
              grid=256 if bn else 0, ws=ws, bm=bm)
    lg = a.float() @ w.float().T + bias
    top = lg.topk(2, dim=-1)
    clear = (top.values[:, 0] - top.values[:, 1]) > 1e-3 * top.values[:, 0].abs()
    got = 0xFFFFFFFF - (keys & 0xFFFFFFFF)
    assert bool((got[clear] == top.indices[clear, 0] + 100).all())


@pytest.mark.parametrize("M,bn,bm", [(300, 128, 0), (512, 256, 0), (129, 0, 0), (96, 128, 128), (200, 256, 128)])
def test_gemm_sk_fused_rmsnorm_across_gemms(M, bn, bm, ws):
    """RMSNorm fused across GEMMs: a residual GEMM writes per-64-column sums of squares of its
    rounded outputs (ss_out); a SwiGLU / QKV GEMM reading that raw residual stream as A scales
    each row by rsqrt(mean + eps) from them (ss_in) - against fp32 torch RMSNorm + projection."""
    from llm_sharding_amd.config import tiny
    from llm_sharding_amd.models.rope import rope_table
    h = hip()
    H, K0, I, eps = 1024, 512, 768, 1e-5
    x, r = _rnd(M, K0), _rnd(M, H)
    wo = _rnd(H, K0, scale=0.03)
    hb = r.clone()
    ss = torch.full((M, H // 64), float("nan"), device=DEV)
    h.gemm_sk(x, packing.pack_b(wo), M, H, K0, h.EPI_RESID, h.make_epi(out=hb, resid=hb, ldo=H, ldr=H, ss_out=ss),
              bn=bn, grid=256 if bn else 0, ws=ws, bm=bm)
    assert rel_err(hb, r.float() + x.float() @ wo.float().T) < 8e-3
    assert rel_err(ss, hb.float().pow(2).view(M, H // 64, 64).sum(-1)) < 1e-5
    hf = hb.float()
    xn = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps)
    # SwiGLU consumer
    wg, wu = _rnd(I, H, scale=0.03), _rnd(I, H, scale=0.03)
    out = torch.zeros(M, I, dtype=torch.bfloat16, device=DEV)
    h.gemm_sk(hb, packing.pack_b(packing.fuse_gate_up(wg, wu)), M, 2 * I, H, h.EPI_SWIGLU,
              h.make_epi(out=out, ldo=I, ss_in=ss, ss_eps=eps), ws=ws, bn=bn, grid=256 if bn else 0, bm=bm)
    assert rel_err(out, F.silu(xn @ wg.float().T) * (xn @ wu.float().T)) < 1e-2
    # QKV consumer (RoPE + KV append after the norm scale)
    nh, nkv, hd, T = 8, 2, 128, 512
    wq, wk, wv = _rnd(nh * hd, H, scale=0.03), _rnd(nkv * hd, H, scale=0.03), _rnd(nkv * hd, H, scale=0.03)
    cos, sin = rope_table(tiny(head_dim=hd), T, DEV)
    slot = torch.zeros(M, dtype=torch.int32, device=DEV)
    pos = torch.randperm(T, device=DEV)[:M].to(torch.int32)
    q = torch.zeros(M, nh * hd, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(1, nkv, T, hd, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    h.gemm_sk(hb, packing.pack_b(packing.fuse_qkv(wq, wk, wv, nh, nkv, hd)), M, (nh + 2 * nkv) * hd, H, h.EPI_QKV,
              h.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, cos=cos, sin=sin, ldo=nh * hd, n_heads=nh,
                         n_kv=nkv, head_dim=hd, t_max=T, ss_in=ss, ss_eps=eps), ws=ws, bn=bn, grid=256 if bn else 0,
              bm=bm)
    pl = pos.long()
    assert rel_err(q, _rope_ref((xn @ wq.float().T).view(M, nh, hd), pl, cos, sin).reshape(M, -1)) < 1e-2
    assert rel_err(vc[0, :, pl].transpose(0, 1), (xn @ wv.float().T).view(M, nkv, hd)) < 1e-2


@pytest.mark.parametrize("name,N,K,epi", [("qkv", 10240, 8192, "store"), ("o", 8192, 8192, "resid"),
                                          ("gate_up", 57344, 8192, "swiglu"), ("down", 8192, 28672, "resid")])
def test_gemm_llama70b_projections_at_512_rows(name, N, K, epi):
    """The four Llama-2-70B projections at the 512-row micro-batch of the 70B stage bench, through
    hip.gemm's tuned plan (profiles/r4_gemm_vs_hipblaslt_70b.jsonl), against fp32 PyTorch."""
    h = hip()
    M = 512
    a = _rnd(M, K)
    w = _rnd(N, K, scale=0.02)
    ref = a.float() @ w.float().T
    wp = packing.pack_b(w)
    del w
    sk_ws = h.SkWorkspace(DEV)
    if epi == "store":
        out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
        h.gemm(a, wp, M, N, K, h.EPI_STORE, h.make_epi(out=out, ldo=N), sk_ws=sk_ws)
        want = ref
    elif epi == "resid":
        resid = _rnd(M, N)
        out = resid.clone()
        h.gemm(a, wp, M, N, K, h.EPI_RESID, h.make_epi(out=out, resid=out, ldo=N, ldr=N), sk_ws=sk_ws)
        want = resid.float() + ref
    else:
        out = torch.full((M, N // 2), float("nan"), dtype=torch.bfloat16, device=DEV)
        h.gemm(a, wp, M, N, K, h.EPI_SWIGLU, h.make_epi(out=out, ldo=N // 2), sk_ws=sk_ws)
        g, u = ref.view(M, N // 32, 2, 16)[:, :, 0].reshape(M, -1), ref.view(M, N // 32, 2, 16)[:, :, 1].reshape(M, -1)
        want = F.silu(g) * u
    torch.cuda.synchronize()
    assert rel_err(out, want) < 1e-2, name
