"""LlamaShardPart (reference C4, utils/shard_loader.py:8-78): a contiguous layer range as a
module with the reference constructor, optional final norm and a KV-cache handle, against the
fp32 golden model - on CPU, and on an MI355X (HIP kernels, HIP RMSNorm for the final norm)."""
import pytest
import torch

from llm_sharding_amd.models import weights as W
from llm_sharding_amd.models.reference import ReferenceLlama, rmsnorm
from llm_sharding_amd.utils.shard_loader import LlamaShardPart
from llm_sharding_amd.utils.numerics import rel_err  # global + per-16x16-tile + per-row




def _check(shards, device, dtype, tol):
    cfg, emb, layers, fn, lm = W.load_full_model(shards)
    L = cfg.num_hidden_layers
    ref = ReferenceLlama(cfg, emb, layers, fn, lm)
    ids = torch.tensor([[1, 33, 44, 55, 66, 7]])
    x = ref.embed[ids]
    want_mid = ref.forward_hidden(x.clone(), 0, 2)
    ref.reset()
    want_all = rmsnorm(ref.forward_hidden(x.clone()), fn, cfg.rms_norm_eps)
    a = LlamaShardPart(shards, [f"block_{i}.pth" for i in range(0, 2)], 0, 2, device=device, dtype=dtype)
    b = LlamaShardPart(shards, [f"block_{i}.pth" for i in range(2, L)], 2, L, device=device, dtype=dtype,
                       add_final_norm=True, final_norm_weight="final_norm.pth")
    h = a(x.to(device, dtype))
    assert rel_err(h, want_mid) < tol
    out = b(h)
    assert out.shape == (1, 6, cfg.hidden_size)
    assert rel_err(out, want_all) < tol
    # incremental decode through the KV-cache handles: prefill 5 tokens, then the 6th alone
    ca, cb = a.new_cache(1), b.new_cache(1)
    ha = a(x[:, :5].to(device, dtype), past_key_value=ca)
    b(ha, past_key_value=cb)
    assert ca.get_seq_length() == 5 and cb.get_seq_length() == 5
    last = b(a(x[:, 5:].to(device, dtype), past_key_value=ca), past_key_value=cb)
    assert rel_err(last[0, -1], want_all[0, -1]) < tol


def test_shard_part_cpu(tiny_shards):
    _check(tiny_shards, "cpu", torch.float32, 1e-4)


@pytest.mark.gpu
def test_shard_part_gpu(tiny_shards_bf16):
    _check(tiny_shards_bf16, "cuda", torch.bfloat16, 3e-2)
