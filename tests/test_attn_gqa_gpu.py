"""GQA decode attention on MFMA (attn_prefill.hip gqa_decode_kernel, lsa_attn_decode_mfma): rows
of one query position each against their own cache slots, G = 2 / 3 / 4 / 8 / 16 query heads per
KV head (3: Llama-3.2-3B, the reference's configured model; 8: Llama-2-70B), head dims 64 / 128,
2 or 4 waves splitting the keys, per-row lengths (causal pos + 1, or explicit kv_len) - against
an fp32 torch reference, and the hip.attn dispatch (which picks this kernel for GQA batches that
fill the GPU)."""
import pytest
import torch
from llm_sharding_amd.utils.numerics import rel_err  # global + per-16x16-tile + per-row

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(q, kc, vc, slot, lens, nh, nkv, hd):
    rows = q.shape[0]
    g = nh // nkv
    out = torch.zeros(rows, nh * hd)
    for r in range(rows):
        T = int(lens[r])
        k = kc[int(slot[r]), :, :T].float()          # [nkv, T, hd]
        v = vc[int(slot[r]), :, :T].float()
        qr = q[r].float().view(nh, hd)
        for h in range(nh):
            s = (k[h // g] @ qr[h]) * hd ** -0.5
            out[r, h * hd:(h + 1) * hd] = torch.softmax(s, -1) @ v[h // g]
    return out


@pytest.mark.parametrize("nh,nkv,hd", [(64, 8, 128), (24, 8, 128), (32, 8, 128), (16, 2, 64), (32, 16, 128),
                                       (32, 2, 128), (12, 4, 64)])
@pytest.mark.parametrize("explicit_len", [False, True])
@pytest.mark.parametrize("nw", [1, 2, 4])
def test_attn_decode_mfma_vs_fp32(nh, nkv, hd, explicit_len, nw):
    from llm_sharding_amd.ops import hip
    torch.manual_seed(0)
    rows, slots, tmax = 40, 48, 320
    kc = torch.randn(slots, nkv, tmax, hd, device=DEV).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(rows, nh * hd, device=DEV).to(torch.bfloat16)
    slot = torch.randperm(slots, device=DEV)[:rows].to(torch.int32)
    pos = torch.randint(0, tmax, (rows,), device=DEV, dtype=torch.int32)
    pos[0], pos[1], pos[2] = 0, 63, tmax - 1  # one key, one full block, the whole cache
    kv_len = torch.randint(1, tmax + 1, (rows,), device=DEV, dtype=torch.int32) if explicit_len else None
    out = torch.zeros(rows, nh * hd, dtype=torch.bfloat16, device=DEV)
    rc = hip.lib().lsa_attn_decode_mfma(hip._p(q), q.stride(0), hip._p(kc), hip._p(vc), hip._p(slot), hip._p(pos),
                                        hip._p(kv_len), rows, nh, nkv, hd, tmax, float(hd ** -0.5), hip._p(out),
                                        out.stride(0), nw, hip._stream())
    assert rc == 0
    torch.cuda.synchronize()
    lens = (kv_len if explicit_len else pos + 1).cpu()
    ref = _ref(q.cpu(), kc.cpu(), vc.cpu(), slot.cpu(), lens, nh, nkv, hd)
    err = rel_err(out.cpu(), ref)
    assert err < 1e-2, err


@pytest.mark.parametrize("nh,nkv", [(64, 8), (24, 8)])
def test_attn_dispatch_uses_mfma_for_big_gqa_batches(nh, nkv):
    """hip.attn: a 70B-shaped (64 / 8 heads) or 3B-shaped (24 / 8) batch of 128 rows goes to the
    MFMA kernel and agrees with the split-KV kernel it replaces (LSA_ATTN_MFMA switch), within
    bf16 rounding."""
    from llm_sharding_amd.ops import hip
    torch.manual_seed(1)
    rows, hd, tmax = 128, 128, 256
    kc = torch.randn(rows, nkv, tmax, hd, device=DEV).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(rows, nh * hd, device=DEV).to(torch.bfloat16)
    slot = torch.arange(rows, device=DEV, dtype=torch.int32)
    pos = torch.randint(0, tmax, (rows,), device=DEV, dtype=torch.int32)
    po = torch.empty(rows * nh * 4 * hd, device=DEV)
    pl = torch.empty(rows * nh * 4, device=DEV)
    cnt = torch.zeros(rows * nkv, dtype=torch.int32, device=DEV)
    outs = []
    for mfma in (True, False):
        prev = hip.ATTN_MFMA
        hip.ATTN_MFMA = mfma
        try:
            o = torch.zeros(rows, nh * hd, dtype=torch.bfloat16, device=DEV)
            hip.attn(q, kc, vc, slot, pos, rows, nh, nkv, hd, 2, po, pl, o, counters=cnt)
            outs.append(o)
        finally:
            hip.ATTN_MFMA = prev
    torch.cuda.synchronize()
    err = rel_err(outs[0], outs[1])
    assert rows * nkv >= hip.ATTN_MFMA_MIN_ITEMS
    assert err < 1e-2, err
