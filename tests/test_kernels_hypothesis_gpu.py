"""Hypothesis shape sweeps of the HIP kernels against plain PyTorch fp32 references (GPU):
decode/coop projections with the auto-selected configs, the prefill GEMM with its auto
split-K, split-KV decode attention and flash prefill attention over random sequence
layouts. Every drawn shape passes the host-side checks of ops/hip.py first."""
import math

import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from llm_sharding_amd.ops import packing
from llm_sharding_amd.utils.numerics import rel_err  # global + per-16x16-tile + per-row

pytestmark = pytest.mark.gpu
DEV = "cuda"
SET = settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])


def hip():
    from llm_sharding_amd.ops import hip as h
    h.lib()
    return h




@SET
@given(M=st.integers(1, 128), nt=st.integers(1, 24), kc=st.integers(1, 48), norm=st.booleans(),
       resid=st.booleans())
def test_projection_random_shapes(M, nt, kc, norm, resid):
    h = hip()
    N, K = nt * 64, kc * 64
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    g = (1 + 0.1 * torch.randn(K, device=DEV)).to(torch.bfloat16)
    r = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    out = r.clone() if resid else torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    xf = x.float()
    if norm:
        xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * g.float()
    ref = xf @ w.float().T + (r.float() if resid else 0)
    wp = packing.pack_b(packing.fold_norm(w, g) if norm else w)
    ep = h.make_epi(out=out, resid=out if resid else None, ldo=N, ldr=N)
    h.gemv(x, wp, M, N, K, h.EPI_RESID if resid else h.EPI_STORE, ep, norm=norm)
    assert rel_err(out, ref) < 1e-2


@SET
@given(M=st.integers(1, 700), nt=st.integers(1, 12), kc=st.integers(1, 40))
def test_gemm_random_shapes(M, nt, kc):
    h = hip()
    N, K = nt * 128, kc * 64
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    h.gemm(a, packing.pack_b(w), M, N, K, h.EPI_STORE, h.make_epi(out=out, ldo=N))
    assert rel_err(out, a.float() @ w.float().T) < 1e-2


@SET
@given(rows=st.integers(1, 6), heads=st.sampled_from([(8, 8, 128), (8, 2, 64), (16, 4, 128)]),
       T=st.integers(1, 700), nsplit=st.sampled_from([1, 2, 5, 8]))
def test_decode_attention_random(rows, heads, T, nsplit):
    h = hip()
    nh, nkv, hd = heads
    kc = torch.randn(rows, nkv, T, hd, device=DEV).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(rows, nh * hd, device=DEV).to(torch.bfloat16)
    slot = torch.arange(rows, dtype=torch.int32, device=DEV)
    pos = torch.randint(0, T, (rows,), dtype=torch.int32, device=DEV)
    po = torch.zeros(rows * nh * nsplit * hd, device=DEV)
    pl = torch.zeros(rows * nh * nsplit, device=DEV)
    out = torch.zeros(rows, nh * hd, dtype=torch.bfloat16, device=DEV)
    h.attn(q, kc, vc, slot, pos, rows, nh, nkv, hd, nsplit, po, pl, out)
    g = nh // nkv
    ref = torch.zeros(rows, nh * hd, device=DEV)
    for r in range(rows):
        t = int(pos[r]) + 1
        Kr = kc[r, :, :t].float().repeat_interleave(g, 0)
        Vr = vc[r, :, :t].float().repeat_interleave(g, 0)
        p = torch.softmax(q[r].float().view(nh, 1, hd) @ Kr.transpose(1, 2) / math.sqrt(hd), -1)
        ref[r] = (p @ Vr).reshape(-1)
    assert rel_err(out, ref) < 1e-2


@SET
@given(segs=st.lists(st.tuples(st.integers(0, 90), st.integers(1, 140)), min_size=1, max_size=4),
       heads=st.sampled_from([(8, 8, 128), (8, 2, 64), (16, 2, 128)]), causal=st.booleans())
def test_flash_prefill_random(segs, heads, causal):
    h = hip()
    nh, nkv, hd = heads
    T = 256
    slots = len(segs)
    kc = torch.randn(slots, nkv, T, hd, device=DEV).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    slot = sum([[i] * n for i, (p0, n) in enumerate(segs)], [])
    pos = sum([list(range(p0, p0 + n)) for p0, n in segs], [])
    kvl = None if causal else sum([[p0 + n] * n for p0, n in segs], [])
    rows = len(slot)
    q = torch.randn(rows, nh * hd, device=DEV).to(torch.bfloat16)
    out = torch.zeros(rows, nh * hd, dtype=torch.bfloat16, device=DEV)
    h.attn_prefill(q, kc, vc, h.build_prefill_tiles(slot, pos, kvl, device=DEV, tile_rows=h.prefill_tile_rows(nh, nkv)), nh, nkv, hd, out, causal=causal)
    g = nh // nkv
    ref = torch.zeros(rows, nh * hd, device=DEV)
    for r in range(rows):
        t = pos[r] + 1 if causal else kvl[r]
        Kr = kc[slot[r], :, :t].float().repeat_interleave(g, 0)
        Vr = vc[slot[r], :, :t].float().repeat_interleave(g, 0)
        p = torch.softmax(q[r].float().view(nh, 1, hd) @ Kr.transpose(1, 2) / math.sqrt(hd), -1)
        ref[r] = (p @ Vr).reshape(-1)
    assert rel_err(out, ref) < 1e-2
