"""Golden fp32 torch implementation of the Llama decoder.

SURVEY.md Q16: the local transformers (5.x) silently drops the reference's
``past_key_value=`` kwarg, so it cannot serve as an oracle. This module re-implements the
math of HF ``LlamaDecoderLayer`` (transformers 4.53, the reference's pin,
``/root/reference/requirements.txt:8``) in plain torch:

* RMSNorm: fp32 upcast, ``x * rsqrt(mean(x^2) + eps)``, times weight
* q/k/v projection, half-split RoPE, GQA by ``repeat_kv``
* softmax in fp32 with ``1/sqrt(head_dim)`` scaling; causal by default, the reference's
  unmasked prefill (Q1, ``shard_loader.py:57,69``) via ``causal=False``
* o projection + residual, RMSNorm, SwiGLU MLP + residual
* final RMSNorm, lm_head, greedy argmax of the last position
  (``node_worker.py:260-265``)

Everything here is computed in float32 regardless of the weight dtype; it is the oracle
that every HIP kernel and the engine are tested against.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from ..config import LlamaConfig
from .rope import apply_rope, full_cos_sin, rope_table

LAYER_KEYS = (
    "self_attn.q_proj.weight",
    "self_attn.k_proj.weight",
    "self_attn.v_proj.weight",
    "self_attn.o_proj.weight",
    "mlp.gate_proj.weight",
    "mlp.up_proj.weight",
    "mlp.down_proj.weight",
    "input_layernorm.weight",
    "post_attention_layernorm.weight",
)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    return xf * torch.rsqrt(var + eps) * w.float()


def repeat_kv(x: torch.Tensor, n: int) -> torch.Tensor:
    if n == 1:
        return x
    b, h, t, d = x.shape
    return x[:, :, None].expand(b, h, n, t, d).reshape(b, h * n, t, d)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, past_len: int,
              causal: bool = True) -> torch.Tensor:
    """q: [B, nH, S, d]; k, v: [B, nH, T, d] (T = past_len + S). Returns [B, nH, S, d]."""
    d = q.shape[-1]
    scores = torch.matmul(q, k.transpose(-1, -2)) * (d ** -0.5)
    if causal:
        S, T = q.shape[2], k.shape[2]
        qpos = torch.arange(S, device=q.device)[:, None] + past_len
        kpos = torch.arange(T, device=q.device)[None, :]
        scores = scores.masked_fill(kpos > qpos, float("-inf"))
    p = torch.softmax(scores.float(), dim=-1)
    return torch.matmul(p, v)


class RefKVCache:
    """Per-layer list of fp32 (k, v) tensors [B, nKV, T, d]."""

    def __init__(self, n_layers: int):
        self.k = [None] * n_layers
        self.v = [None] * n_layers

    def get_seq_length(self, layer: int = 0) -> int:
        return 0 if self.k[layer] is None else int(self.k[layer].shape[2])

    def update(self, layer: int, k: torch.Tensor, v: torch.Tensor):
        if self.k[layer] is None:
            self.k[layer], self.v[layer] = k, v
        else:
            self.k[layer] = torch.cat([self.k[layer], k], dim=2)
            self.v[layer] = torch.cat([self.v[layer], v], dim=2)
        return self.k[layer], self.v[layer]


def decoder_layer(cfg: LlamaConfig, w: dict, h: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor,
                  cache: RefKVCache, layer: int, causal: bool = True) -> torch.Tensor:
    """One HF-equivalent ``LlamaDecoderLayer`` forward in fp32. h: [B, S, H]."""
    B, S, _ = h.shape
    nh, nkv, d = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    past = cache.get_seq_length(layer)
    x = rmsnorm(h, w["input_layernorm.weight"], cfg.rms_norm_eps)
    q = F.linear(x, w["self_attn.q_proj.weight"].float()).view(B, S, nh, d).transpose(1, 2)
    k = F.linear(x, w["self_attn.k_proj.weight"].float()).view(B, S, nkv, d).transpose(1, 2)
    v = F.linear(x, w["self_attn.v_proj.weight"].float()).view(B, S, nkv, d).transpose(1, 2)
    q = apply_rope(q, cos, sin)
    k = apply_rope(k, cos, sin)
    k, v = cache.update(layer, k, v)
    g = nh // nkv
    o = attention(q, repeat_kv(k, g), repeat_kv(v, g), past, causal)
    o = o.transpose(1, 2).reshape(B, S, nh * d)
    h = h.float() + F.linear(o, w["self_attn.o_proj.weight"].float())
    x = rmsnorm(h, w["post_attention_layernorm.weight"], cfg.rms_norm_eps)
    a = F.silu(F.linear(x, w["mlp.gate_proj.weight"].float())) * F.linear(x, w["mlp.up_proj.weight"].float())
    return h + F.linear(a, w["mlp.down_proj.weight"].float())


class ReferenceLlama:
    """Whole-model fp32 oracle (embedding -> layers -> final norm -> lm_head -> argmax).

    ``layers`` is a list of per-layer state dicts with the reference block keys
    (``/root/reference/utils/model_sharder.py:77-80``).
    """

    def __init__(self, cfg: LlamaConfig, embed: torch.Tensor, layers: list, final_norm: torch.Tensor,
                 lm_head: torch.Tensor, causal: bool = True, max_pos: Optional[int] = None):
        self.cfg = cfg
        self.embed = embed.float()
        self.layers = [{k: t.float() for k, t in lw.items()} for lw in layers]
        self.final_norm = final_norm.float()
        self.lm_head = lm_head.float()
        self.causal = causal
        self.cos, self.sin = rope_table(cfg, max_pos or min(cfg.max_position_embeddings, 8192))
        self.cache = RefKVCache(len(layers))

    def reset(self):
        self.cache = RefKVCache(len(self.layers))

    def forward_hidden(self, h: torch.Tensor, first: int = 0, last: Optional[int] = None) -> torch.Tensor:
        last = len(self.layers) if last is None else last
        B, S, _ = h.shape
        past = self.cache.get_seq_length(first)
        pos = torch.arange(past, past + S)[None].expand(B, S)
        cos, sin = full_cos_sin(self.cos, self.sin, pos)
        h = h.float()
        for i in range(first, last):
            h = decoder_layer(self.cfg, self.layers[i], h, cos, sin, self.cache, i, self.causal)
        return h

    def logits(self, h: torch.Tensor) -> torch.Tensor:
        return F.linear(rmsnorm(h, self.final_norm, self.cfg.rms_norm_eps), self.lm_head)

    def step(self, input_ids: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """Run ids [B, S] through the model; return (next_token [B], last logits [B, V])."""
        h = self.embed[input_ids]
        h = self.forward_hidden(h)
        lg = self.logits(h[:, -1])
        return torch.argmax(lg, dim=-1), lg

    def generate(self, input_ids: torch.Tensor, max_new_tokens: int) -> torch.Tensor:
        self.reset()
        out = []
        tok, _ = self.step(input_ids)
        out.append(tok)
        for _ in range(max_new_tokens - 1):
            tok, _ = self.step(tok[:, None])
            out.append(tok)
        return torch.stack(out, dim=1)
