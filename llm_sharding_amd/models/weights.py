"""On-disk shard format and weight generation.

Layout (kept byte-compatible with the reference, SURVEY.md §2.7,
``/root/reference/utils/model_sharder.py:50-94``)::

    shards/<Model>_<dtype>/
        config.json, generation_config.json, tokenizer files   (copied verbatim)
        embedding.pth     {"weight": [V, H]}
        block_{i}.pth     LlamaDecoderLayer.state_dict() keys (LAYER_KEYS)
        final_norm.pth    {"weight": [H]}
        lm_head.pth       {"weight": [V, H]}

Every ``.pth`` is a plain ``torch.save`` of a ``dict[str, Tensor]``; we always read them with
``torch.load(..., weights_only=True)`` (no unpickling of arbitrary objects). Optionally a
``<name>.safetensors`` twin is read when present (mmap, zero-copy).

Random-init shards (no checkpoints are available offline) follow HF's init
(normal(0, initializer_range=0.02) for matrices, ones for norms) and are generated
deterministically per layer from ``seed`` so any stage can regenerate exactly its own layers
on its own device without touching disk (``random_layer``), which is how the 70B
benchmarks avoid writing 138 GB.
"""
from __future__ import annotations

import json
import os
from typing import Iterable, Optional

import torch

from ..config import LlamaConfig, dtype_suffix
from .reference import LAYER_KEYS

INIT_STD = 0.02


def block_file(i: int) -> str:
    return f"block_{i}.pth"


def layer_shapes(cfg: LlamaConfig) -> dict:
    H, I = cfg.hidden_size, cfg.intermediate_size
    return {
        "self_attn.q_proj.weight": (cfg.q_size, H),
        "self_attn.k_proj.weight": (cfg.kv_size, H),
        "self_attn.v_proj.weight": (cfg.kv_size, H),
        "self_attn.o_proj.weight": (H, cfg.q_size),
        "mlp.gate_proj.weight": (I, H),
        "mlp.up_proj.weight": (I, H),
        "mlp.down_proj.weight": (H, I),
        "input_layernorm.weight": (H,),
        "post_attention_layernorm.weight": (H,),
    }


def _gen(device, seed: int) -> torch.Generator:
    g = torch.Generator(device=device if torch.device(device).type != "cpu" else "cpu")
    g.manual_seed(seed)
    return g


def _randn(shape, std, dtype, device, gen) -> torch.Tensor:
    t = torch.empty(shape, dtype=torch.float32, device=device)
    t.normal_(0.0, std, generator=gen)
    return t.to(dtype)


def _norm_weight(shape, dtype, device, gen, jitter: float) -> torch.Tensor:
    if jitter == 0.0:
        return torch.ones(shape, dtype=dtype, device=device)
    t = torch.empty(shape, dtype=torch.float32, device=device)
    t.uniform_(1.0 - jitter, 1.0 + jitter, generator=gen)
    return t.to(dtype)


def random_layer(cfg: LlamaConfig, i: int, dtype=torch.bfloat16, device="cpu", seed: int = 0,
                 std: float = INIT_STD, norm_jitter: float = 0.1) -> dict:
    """Deterministic random weights for layer ``i`` (same on every device for a given seed)."""
    gen = _gen(device, seed * 100003 + 17 * i + 1)
    out = {}
    for k, shp in layer_shapes(cfg).items():
        if len(shp) == 1:
            out[k] = _norm_weight(shp, dtype, device, gen, norm_jitter)
        else:
            out[k] = _randn(shp, std, dtype, device, gen)
    return out


def random_embedding(cfg: LlamaConfig, dtype=torch.bfloat16, device="cpu", seed: int = 0,
                     std: float = 1.0) -> torch.Tensor:
    # HF inits embeddings with std=initializer_range; a larger std keeps hidden-state
    # magnitudes (and therefore greedy decisions) well-conditioned for random models.
    gen = _gen(device, seed * 100003 + 7)
    return _randn((cfg.vocab_size, cfg.hidden_size), std, dtype, device, gen)


def random_final_norm(cfg: LlamaConfig, dtype=torch.bfloat16, device="cpu", seed: int = 0,
                      norm_jitter: float = 0.1) -> torch.Tensor:
    gen = _gen(device, seed * 100003 + 11)
    return _norm_weight((cfg.hidden_size,), dtype, device, gen, norm_jitter)


def random_lm_head(cfg: LlamaConfig, dtype=torch.bfloat16, device="cpu", seed: int = 0,
                   std: float = INIT_STD) -> torch.Tensor:
    gen = _gen(device, seed * 100003 + 13)
    return _randn((cfg.vocab_size, cfg.hidden_size), std, dtype, device, gen)


# ---------------------------------------------------------------------------- IO
def save_tensor_dict(d: dict, path: str) -> None:
    torch.save({k: v.contiguous() for k, v in d.items()}, path)


def dequantize(d: dict) -> dict:
    """Quantised shards (utils/model_sharder.py) -> bf16: fp8 / int8 with per-channel scales
    (``q * scale[:, None]``), int4 packed two per byte with group-wise scales."""
    out = {}
    for k, v in d.items():
        if k.endswith("_scale"):
            continue
        s = d.get(k + "_scale")
        if s is not None:
            s = s.to(v.device)
            if v.dtype == torch.uint8 and s.dim() == 2:
                from ..utils.model_sharder import dequantize_int4
                v = dequantize_int4(v, s).to(torch.bfloat16)
            else:
                v = (v.float() * s.float()[:, None]).to(torch.bfloat16)
        out[k] = v
    return out


def load_tensor_dict(path: str, device="cpu") -> dict:
    st = os.path.splitext(path)[0] + ".safetensors"
    if os.path.exists(st):
        from safetensors.torch import load_file
        return dequantize(load_file(st, device=str(device)))
    return dequantize(torch.load(path, map_location=device, weights_only=True))


def load_block(shards_path: str, i: int, device="cpu", dtype=None) -> dict:
    d = load_tensor_dict(os.path.join(shards_path, block_file(i)), device)
    missing = [k for k in LAYER_KEYS if k not in d]
    if missing:
        raise KeyError(f"block_{i}.pth is missing keys {missing}")
    if dtype is not None:
        d = {k: v.to(dtype) for k, v in d.items()}
    return d


def load_single(shards_path: str, name: str, device="cpu", dtype=None) -> torch.Tensor:
    d = load_tensor_dict(os.path.join(shards_path, name), device)
    w = d["weight"]
    return w.to(dtype) if dtype is not None else w


def load_lm_head(shards_path: str, cfg: LlamaConfig, device="cpu", dtype=None) -> torch.Tensor:
    p = os.path.join(shards_path, "lm_head.pth")
    if os.path.exists(p) or os.path.exists(p.replace(".pth", ".safetensors")):
        return load_single(shards_path, "lm_head.pth", device, dtype)
    if cfg.tie_word_embeddings:
        return load_single(shards_path, "embedding.pth", device, dtype)
    raise FileNotFoundError(p)


def write_random_shards(cfg: LlamaConfig, folder: str, dtype=torch.bfloat16, seed: int = 0,
                        append_dtype_suffix: bool = True, tokenizer: bool = True,
                        layers: Optional[Iterable[int]] = None) -> str:
    """Write a complete random-init shard folder in the reference format. Returns its path."""
    from .tokenizer import SyntheticByteTokenizer
    out = folder + "_" + dtype_suffix(dtype) if append_dtype_suffix else folder
    os.makedirs(out, exist_ok=True)
    cfg.save_pretrained(out)
    with open(os.path.join(out, "generation_config.json"), "w") as f:
        json.dump({"bos_token_id": cfg.bos_token_id, "eos_token_id": cfg.eos_token_id,
                   "do_sample": False}, f, indent=2)
    if tokenizer:
        SyntheticByteTokenizer(cfg.vocab_size, cfg.bos_token_id, cfg.eos_ids[0] if cfg.eos_ids else 2
                               ).save_pretrained(out)
    save_tensor_dict({"weight": random_embedding(cfg, dtype, seed=seed)}, os.path.join(out, "embedding.pth"))
    for i in (range(cfg.num_hidden_layers) if layers is None else layers):
        save_tensor_dict(random_layer(cfg, i, dtype, seed=seed), os.path.join(out, block_file(i)))
    save_tensor_dict({"weight": random_final_norm(cfg, dtype, seed=seed)}, os.path.join(out, "final_norm.pth"))
    save_tensor_dict({"weight": random_lm_head(cfg, dtype, seed=seed)}, os.path.join(out, "lm_head.pth"))
    return out


def load_full_model(shards_path: str, device="cpu", dtype=None):
    """Load every file of a shard folder: (cfg, embed, [layers], final_norm, lm_head)."""
    cfg = LlamaConfig.from_pretrained(shards_path)
    embed = load_single(shards_path, "embedding.pth", device, dtype)
    layers = [load_block(shards_path, i, device, dtype) for i in range(cfg.num_hidden_layers)]
    fn = load_single(shards_path, "final_norm.pth", device, dtype)
    lm = load_lm_head(shards_path, cfg, device, dtype)
    return cfg, embed, layers, fn, lm
