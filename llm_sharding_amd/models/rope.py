"""Rotary position embedding tables.

The reference builds HF ``LlamaRotaryEmbedding`` on the head stage only and ships the
resulting ``cos``/``sin`` tensors ([B, S, head_dim]) down the chain
(``/root/reference/utils/node_worker.py:149-153,239-241,267-271``).  Here the table is a
precomputed ``[max_pos, head_dim/2]`` fp32 array resident on every stage, indexed by a
device-side position counter, so nothing but the hidden state travels between stages.

Math matches HF (default and ``llama3`` rope types): ``inv_freq = base^(-2i/d)``,
``emb = cat(freqs, freqs)``, half-split ``rotate_half``.
"""
from __future__ import annotations

import math

import torch

from ..config import LlamaConfig


def inv_freq(cfg: LlamaConfig) -> torch.Tensor:
    d = cfg.head_dim
    base = float(cfg.rope_theta)
    inv = 1.0 / (base ** (torch.arange(0, d, 2, dtype=torch.int64).float() / d))
    rs = cfg.rope_scaling or {}
    rtype = rs.get("rope_type", rs.get("type", "default"))
    if rtype in (None, "default"):
        return inv
    if rtype == "linear":
        return inv / float(rs["factor"])
    if rtype == "llama3":
        factor = float(rs["factor"])
        low = float(rs["low_freq_factor"])
        high = float(rs["high_freq_factor"])
        old_ctx = float(rs["original_max_position_embeddings"])
        low_wl = old_ctx / low
        high_wl = old_ctx / high
        wavelen = 2 * math.pi / inv
        inv_l = torch.where(wavelen > low_wl, inv / factor, inv)
        smooth = (old_ctx / wavelen - low) / (high - low)
        smoothed = (1 - smooth) * inv_l / factor + smooth * inv_l
        is_med = ~(wavelen < high_wl) * ~(wavelen > low_wl)
        return torch.where(is_med, smoothed, inv_l)
    raise NotImplementedError(f"rope_type {rtype!r} not supported")


def rope_table(cfg: LlamaConfig, max_pos: int | None = None, device=None) -> tuple[torch.Tensor, torch.Tensor]:
    """Return ``(cos, sin)`` each ``[max_pos, head_dim/2]`` fp32."""
    n = int(max_pos or cfg.max_position_embeddings)
    inv = inv_freq(cfg)
    pos = torch.arange(n, dtype=torch.float32)
    freqs = torch.outer(pos, inv.float())
    cos, sin = freqs.cos(), freqs.sin()
    if device is not None:
        cos, sin = cos.to(device), sin.to(device)
    return cos.contiguous(), sin.contiguous()


def full_cos_sin(cos_half: torch.Tensor, sin_half: torch.Tensor, position_ids: torch.Tensor,
                 dtype=None) -> tuple[torch.Tensor, torch.Tensor]:
    """HF-shaped ``[B, S, head_dim]`` cos/sin for the wire protocol (``next_state_info``)."""
    c = cos_half[position_ids]
    s = sin_half[position_ids]
    c = torch.cat([c, c], dim=-1)
    s = torch.cat([s, s], dim=-1)
    if dtype is not None:
        c, s = c.to(dtype), s.to(dtype)
    return c, s


def rotate_half(x: torch.Tensor) -> torch.Tensor:
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), dim=-1)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """``x``: [B, nh, S, d]; ``cos``/``sin``: [B, S, d] (full, HF layout)."""
    return x * cos.unsqueeze(1) + rotate_half(x) * sin.unsqueeze(1)
