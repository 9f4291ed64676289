"""``LlamaShardPart`` - a contiguous range of decoder layers as one module
(reference C4, ``utils/shard_loader.py:8-78``).

Same constructor (``shards_path, shard_weights, start, end, device, dtype, add_final_norm,
final_norm_weight``) and ``forward(hidden_states, attention_mask=None, past_key_value=None,
rotary_emb=None)``. Underneath it is a :class:`StageEngine`: on a ROCm device the layers run
as the fused HIP kernels with packed weights and a static KV cache; on CPU as torch ops.

Differences from the reference, by design:
* ``past_key_value`` is a :class:`StageKVCache` handle (``get_seq_length()``), created with
  :meth:`LlamaShardPart.new_cache`; passing ``None`` runs a stateless forward from position 0.
  Layer indices stay relative to the shard (reference Q15) - the cache belongs to the shard.
* ``rotary_emb`` is accepted for API compatibility; positions come from the cache length and
  RoPE is applied inside the fused QKV kernel from a precomputed table (so cos/sin never need
  to travel between stages).
* attention is causal unless ``causal=False`` (the reference's unmasked prefill, Q1).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from ..config import LlamaConfig
from ..models import weights as W
from ..runtime.engine import ShardFolderSource, StageEngine


class StageKVCache:
    """Handle on a shard's static KV cache (per-batch-row sequence length)."""

    def __init__(self, shard: "LlamaShardPart", batch_size: int = 1):
        self.shard = shard
        self.batch_size = batch_size
        self.shard.engine.reset(range(batch_size))

    def get_seq_length(self, layer_idx: int = 0) -> int:
        return int(self.shard.engine.seq_len[0])

    def reset(self) -> None:
        self.shard.engine.reset(range(self.batch_size))


class _ListSource(ShardFolderSource):
    """Shard-folder source restricted to an explicit list of block files."""

    def __init__(self, path: str, cfg: LlamaConfig, files: list, start: int):
        super().__init__(path, cfg)
        self.files, self.start = files, start

    def layer(self, i, device, dtype):
        d = W.load_tensor_dict(os.path.join(self.path, self.files[i - self.start]), device)
        return {k: v.to(dtype) for k, v in d.items()}


class LlamaShardPart(torch.nn.Module):
    def __init__(self, shards_path: str, shard_weights: list, start: int, end: int,
                 device="cpu", dtype=torch.float32, add_final_norm: bool = False,
                 final_norm_weight: Optional[str] = None, max_batch: int = 1, max_seq: int = 2048,
                 causal: bool = True):
        super().__init__()
        self.shards_path, self.shard_weights = shards_path, list(shard_weights)
        self.start, self.end = start, end
        self.device = torch.device(device)
        self.dtype = dtype
        self.config = LlamaConfig.from_pretrained(shards_path)
        if len(self.shard_weights) != end - start:
            raise ValueError("[ERROR] String list: shard_weights length must be equal to (end - start)")
        if add_final_norm and final_norm_weight is None:
            raise ValueError("[ERROR] final_norm_weight is required when add_final_norm is True")
        eng_dtype = torch.bfloat16 if self.device.type == "cuda" else dtype
        self.engine = StageEngine(self.config, start, end, self.device, eng_dtype,
                                  source=_ListSource(shards_path, self.config, self.shard_weights, start),
                                  max_slots=max_batch, max_seq=max_seq, causal=causal)
        self.final_norm = None
        if add_final_norm:
            self.final_norm_weight = final_norm_weight
            self.final_norm = W.load_single(shards_path, final_norm_weight, self.device, eng_dtype)
        self.causal = causal

    def new_cache(self, batch_size: int = 1) -> StageKVCache:
        return StageKVCache(self, batch_size)

    @torch.inference_mode()
    def forward(self, hidden_states: torch.Tensor, attention_mask=None, past_key_value=None,
                rotary_emb=None) -> torch.Tensor:
        B, S, H = hidden_states.shape
        eng = self.engine
        if past_key_value is None:
            eng.reset(range(B))
        slots = list(range(B))
        slot, pos = eng.prefill_rows(slots, [S] * B)
        kv_len = None if self.causal else [eng.seq_len[0] + S] * (B * S)
        out = eng.forward(hidden_states.reshape(B * S, H).to(self.device, eng.dtype), slot, pos, kv_len=kv_len)
        if past_key_value is None:
            eng.reset(range(B))
        else:
            eng.advance(slots, [S] * B)
        if self.final_norm is not None:
            if eng.gpu:  # the HIP RMSNorm kernel (elementwise.hip), weight applied in-kernel
                from ..ops import hip
                normed = torch.empty((B * S, H), dtype=torch.bfloat16, device=self.device)
                hip.rmsnorm(out.contiguous(), self.final_norm, normed, B * S, self.config.rms_norm_eps)
                out = normed
            else:
                from ..models.reference import rmsnorm
                out = rmsnorm(out, self.final_norm, self.config.rms_norm_eps).to(eng.dtype)
        out = out.reshape(B, S, H)
        return out.to(self.dtype) if self.device.type == "cpu" else out
