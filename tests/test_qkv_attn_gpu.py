"""Fused QKV projection + attention (csrc/kernels/qkv_attn.hip) for small decode batches.

The kernel runs the same GEMV body (fused RMSNorm, RoPE, KV append) and the same attention body
as the two-launch path, so against `gemv(EPI_QKV) + attn(nsplit=1)` every output must be
bit-identical; against the fp32 PyTorch composition of RMSNorm -> q/k/v -> RoPE -> causal
softmax attention it must agree to bf16 rounding. The engine-level test checks that a decode
graph with the fused launch produces the tokens of the graph without it."""
import pytest
import torch

from llm_sharding_amd.config import LlamaConfig
from llm_sharding_amd.runtime.engine import DecodeGraph, RandomSource, StageEngine

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _hip():
    from llm_sharding_amd.ops import hip
    return hip


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _packed_qkv(g, nh, nkv, hd, H):
    """Random q/k/v weights fused, norm-folded and packed as StageEngine._prepare_layer does;
    also returns the fp32 pieces for the reference."""
    from llm_sharding_amd.ops import packing
    wq = torch.randn(nh * hd, H, generator=g) * 0.02
    wk = torch.randn(nkv * hd, H, generator=g) * 0.02
    wv = torch.randn(nkv * hd, H, generator=g) * 0.02
    gn = 1.0 + 0.1 * torch.randn(H, generator=g)
    fused = packing.fuse_qkv(wq, wk, wv, nh, nkv, hd)
    wp = packing.pack_b(packing.fold_norm(fused, gn).to(DEV).to(torch.bfloat16))
    return wp, (wq, wk, wv, gn)


@pytest.mark.parametrize("nh,nkv", [(4, 4), (8, 4), (12, 4), (8, 2), (16, 2)])
@pytest.mark.parametrize("rows", [1, 3, 16])
@pytest.mark.parametrize("cfg", [(1, 4, 4), (2, 4, 4), (1, 4, 8)])
def test_qkv_attn_bit_equal_to_two_launches(nh, nkv, rows, cfg):
    hip = _hip()
    H, hd = 1024, 128
    if (H // 32) % cfg[2]:
        pytest.skip("K does not tile")
    g = torch.Generator().manual_seed(nh * 100 + rows)
    N = (nh + 2 * nkv) * hd
    t_max = 256
    wpk, ref_w = _packed_qkv(g, nh, nkv, hd, H)
    x = torch.randn(rows, H, generator=g).to(DEV).to(torch.bfloat16)
    slots = torch.arange(rows, dtype=torch.int32, device=DEV)
    pos = torch.tensor([37 + 5 * r for r in range(rows)], dtype=torch.int32, device=DEV)
    from llm_sharding_amd.models.rope import rope_table
    lc = LlamaConfig(hidden_size=H, num_attention_heads=nh, num_key_value_heads=nkv, head_dim=hd,
                     max_position_embeddings=512)
    cos, sin = rope_table(lc, t_max, DEV)
    base_k = torch.randn(rows, nkv, t_max, hd, generator=g).to(torch.bfloat16).to(DEV)
    base_v = torch.randn(rows, nkv, t_max, hd, generator=g).to(torch.bfloat16).to(DEV)
    outs = []
    for fused in (False, True):
        kc, vc = base_k.clone(), base_v.clone()
        q = torch.full((rows, nh * hd), float("nan"), device=DEV).to(torch.bfloat16)
        ao = torch.full((rows, nh * hd), float("nan"), device=DEV).to(torch.bfloat16)
        ep = hip.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slots, pos=pos, cos=cos, sin=sin, ldo=q.stride(0),
                          n_heads=nh, n_kv=nkv, head_dim=hd, t_max=t_max)
        if fused:
            sync = torch.zeros(2 * nkv, dtype=torch.int32, device=DEV)
            err = torch.zeros(1, dtype=torch.int32, device=DEV)
            for _ in range(2):  # twice: the counters must come back zeroed
                hip.qkv_attn(x, wpk, rows, N, H, 1e-5, ep, ao, sync, err, cfg)
            torch.cuda.synchronize()
            assert int(err.item()) == 0 and int(sync.abs().sum()) == 0
        else:
            tn, nw, u = cfg
            hip.gemv(x, wpk, rows, N, H, hip.EPI_QKV, ep, norm=True, eps=1e-5, tn=tn, nw=nw, u=u)
            po = torch.empty(rows * nh * hd, device=DEV)
            pl = torch.empty(rows * nh, device=DEV)
            hip.attn(q, kc, vc, slots, pos, rows, nh, nkv, hd, 1, po, pl, ao, min_chunk=1)
            torch.cuda.synchronize()
        outs.append((q, kc, vc, ao))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    # fp32 reference: RMSNorm -> q/k/v -> half-split RoPE at pos -> softmax over keys [0, pos]
    wq, wk, wv, gn = ref_w
    xf = x.float().cpu()
    xn = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * gn
    qf, kf, vf = xn @ wq.T, xn @ wk.T, xn @ wv.T
    G = nh // nkv
    cs, sn = cos.float().cpu(), sin.float().cpu()
    kref, vref = base_k.float().cpu(), base_v.float().cpu()

    def rope(t, p):  # t [heads, hd]
        c, s_ = cs[p], sn[p]
        t1, t2 = t[:, :hd // 2], t[:, hd // 2:]
        return torch.cat([t1 * c - t2 * s_, t2 * c + t1 * s_], -1)
    want = torch.empty(rows, nh * hd)
    for r in range(rows):
        p = int(pos[r])
        qh = rope(qf[r].view(nh, hd), p)
        kh = rope(kf[r].view(nkv, hd), p)
        kr, vr = kref[r].clone(), vref[r].clone()
        kr[:, p] = kh
        vr[:, p] = vf[r].view(nkv, hd)
        for h in range(nh):
            sc = (kr[h // G, :p + 1] @ qh[h]) * hd ** -0.5
            want[r, h * hd:(h + 1) * hd] = torch.softmax(sc, -1) @ vr[h // G, :p + 1]
    assert rel_err(outs[1][3].cpu(), want) < 2e-2


def _engine(cfg, rows, fused, monkeypatch):
    monkeypatch.setattr(StageEngine, "QKV_ATTN", fused)
    return StageEngine(cfg, 0, cfg.num_hidden_layers, DEV, torch.bfloat16, has_embed=True, has_head=True,
                       source=RandomSource(cfg, 9), max_slots=rows, max_seq=128)


@pytest.mark.parametrize("rows", [1, 4])
@pytest.mark.parametrize("shape", ["7b", "gqa"])
def test_decode_graph_fused_matches_unfused(monkeypatch, rows, shape):
    hip = _hip()
    if shape == "7b":
        cfg = LlamaConfig(num_hidden_layers=2, vocab_size=2048, max_position_embeddings=1024, name="7b-2L")
    else:  # Llama-3.2-3B heads (24 q / 8 kv, G = 3)
        cfg = LlamaConfig(hidden_size=3072, intermediate_size=8192, num_attention_heads=24, num_key_value_heads=8,
                          head_dim=128, num_hidden_layers=2, vocab_size=2048, max_position_embeddings=1024,
                          name="3b-2L")
    if hip.qkv_attn_config(rows, cfg.qkv_size, cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                           cfg.head_dim) is None:
        pytest.skip("the tuned qkv config is not a streaming-GEMV config at this shape")
    calls = []
    real = hip.qkv_attn
    monkeypatch.setattr(hip, "qkv_attn", lambda *a, **k: (calls.append(a[2]), real(*a, **k)))
    hist = []
    for fused in (False, True):
        e = _engine(cfg, rows, fused, monkeypatch)
        toks = []
        for s in range(rows):
            p = torch.tensor([1, 17 + s, 99, 5 + 2 * s, 61])
            sl, po = e.prefill_rows([s], [p.numel()])
            h = e.forward(e.embed(p.to(DEV)), sl, po)
            e.advance([s], [p.numel()])
            toks.append(int(e.head(h, [p.numel() - 1])[0]))
        dg = DecodeGraph(e, rows, "full", history_len=8)
        dg.tokens.copy_(torch.tensor(toks, dtype=torch.int32))
        dg.capture()
        for _ in range(8):
            dg.replay()
        torch.cuda.synchronize()
        e.check_errors()
        hist.append(dg.history.cpu().tolist())
    assert rows in calls  # (the 5-token prompts also take it: short prefills run the decode path)
    assert hist[0] == hist[1]
