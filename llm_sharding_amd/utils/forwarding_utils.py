"""``build_position_ids`` (reference ``utils/forwarding_utils.py:4-26``).

Accepts the same ``past_key_value`` forms: anything with ``get_seq_length()`` (our static
KV handles, HF caches), a ``(k, v)`` tuple with k ``[B, n_kv, past, Hd]``, or ``None``.
"""
from __future__ import annotations

import torch


def build_position_ids(past_key_value, seq_len: int, device, batch_size: int = 1) -> torch.Tensor:
    if past_key_value is None:
        past_len = 0
    elif hasattr(past_key_value, "get_seq_length"):
        past_len = int(past_key_value.get_seq_length())
    elif isinstance(past_key_value, tuple) and len(past_key_value) == 2:
        past_len = int(past_key_value[0].shape[-2])
    else:
        raise ValueError("[ERROR] Unsupported past_key_value structure")
    pos = torch.arange(past_len, past_len + seq_len, device=device, dtype=torch.long)
    return pos.unsqueeze(0).expand(batch_size, -1).contiguous()
