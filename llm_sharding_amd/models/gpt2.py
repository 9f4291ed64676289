"""GPT-2 family: on-disk shard format, random init and the fp32 golden forward.

Shard layout written by the reference sharder (``/root/reference/utils/model_sharder.py:96-132``)
and by ours (``utils/model_sharder.py::_save_gpt``)::

    embedding.pth   {"wte": {"weight": [V, H]}, "wpe": {"weight": [P, H]}, "drop": {}}
    block_{i}.pth   GPT2Block.state_dict(): ln_1.{weight,bias}, attn.c_attn.{weight [H,3H], bias},
                    attn.c_proj.{weight [H,H], bias}, ln_2.{weight,bias},
                    mlp.c_fc.{weight [H,I], bias}, mlp.c_proj.{weight [I,H], bias}
    ln_f.pth        {"weight", "bias"}
    lm_head.pth     {"weight": [V, H]}  (tied to wte)

HF's ``Conv1D`` stores weights as [in, out]; :func:`to_linear` turns a block into the engine's
[out, in] ``nn.Linear`` orientation. The reference has no GPT-2 loader, so
parity is pinned against transformers' ``GPT2LMHeadModel`` (tests/test_gpt2.py).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

from ..config import LlamaConfig

GPT2_LAYER_KEYS = (
    "ln_1.weight", "ln_1.bias",
    "attn.c_attn.weight", "attn.c_attn.bias",
    "attn.c_proj.weight", "attn.c_proj.bias",
    "ln_2.weight", "ln_2.bias",
    "mlp.c_fc.weight", "mlp.c_fc.bias",
    "mlp.c_proj.weight", "mlp.c_proj.bias",
)

INIT_STD = 0.02


def layer_shapes(cfg: LlamaConfig) -> dict:
    H, I, Q = cfg.hidden_size, cfg.intermediate_size, cfg.qkv_size
    return {"ln_1.weight": (H,), "ln_1.bias": (H,), "attn.c_attn.weight": (H, Q), "attn.c_attn.bias": (Q,),
            "attn.c_proj.weight": (H, H), "attn.c_proj.bias": (H,), "ln_2.weight": (H,), "ln_2.bias": (H,),
            "mlp.c_fc.weight": (H, I), "mlp.c_fc.bias": (I,), "mlp.c_proj.weight": (I, H), "mlp.c_proj.bias": (H,)}


def _gen(device, seed: int) -> torch.Generator:
    g = torch.Generator(device=device if torch.device(device).type != "cpu" else "cpu")
    g.manual_seed(seed)
    return g


def _randn(shape, std, dtype, device, gen, mean: float = 0.0) -> torch.Tensor:
    t = torch.empty(shape, dtype=torch.float32, device=device)
    t.normal_(mean, std, generator=gen)
    return t.to(dtype)


def random_layer(cfg: LlamaConfig, i: int, dtype=torch.bfloat16, device="cpu", seed: int = 0) -> dict:
    """HF GPT-2 init (normal(0, 0.02), residual projections scaled by 1/sqrt(2 L)) plus small
    random biases and LayerNorm affine jitter so every term of the forward is exercised."""
    gen = _gen(device, seed * 100019 + 29 * i + 3)
    out = {}
    for k, shp in layer_shapes(cfg).items():
        if k.startswith("ln_"):
            out[k] = _randn(shp, 0.1, dtype, device, gen, mean=1.0 if k.endswith("weight") else 0.0)
        elif k.endswith("bias"):
            out[k] = _randn(shp, 0.02, dtype, device, gen)
        else:
            std = INIT_STD / (2 * cfg.num_hidden_layers) ** 0.5 if k.endswith("c_proj.weight") else INIT_STD
            out[k] = _randn(shp, std, dtype, device, gen)
    return out


def random_wte(cfg: LlamaConfig, dtype=torch.bfloat16, device="cpu", seed: int = 0) -> torch.Tensor:
    # larger than HF's 0.02 so random models make well-separated greedy decisions
    return _randn((cfg.vocab_size, cfg.hidden_size), 0.5, dtype, device, _gen(device, seed * 100019 + 7))


def random_wpe(cfg: LlamaConfig, dtype=torch.bfloat16, device="cpu", seed: int = 0) -> torch.Tensor:
    return _randn((cfg.max_position_embeddings, cfg.hidden_size), 0.1, dtype, device, _gen(device, seed * 100019 + 8))


def random_ln_f(cfg: LlamaConfig, dtype=torch.bfloat16, device="cpu", seed: int = 0) -> tuple:
    gen = _gen(device, seed * 100019 + 11)
    return (_randn((cfg.hidden_size,), 0.1, dtype, device, gen, mean=1.0),
            _randn((cfg.hidden_size,), 0.1, dtype, device, gen))


def to_linear(lw: dict) -> dict:
    """GPT-2 block state dict -> engine layout: [out, in] weights, fused q|k|v kept in HF order."""
    return {
        "qkv_w": lw["attn.c_attn.weight"].t().contiguous(), "qkv_b": lw["attn.c_attn.bias"],
        "o_w": lw["attn.c_proj.weight"].t().contiguous(), "o_b": lw["attn.c_proj.bias"],
        "fc_w": lw["mlp.c_fc.weight"].t().contiguous(), "fc_b": lw["mlp.c_fc.bias"],
        "proj_w": lw["mlp.c_proj.weight"].t().contiguous(), "proj_b": lw["mlp.c_proj.bias"],
        "ln1_w": lw["ln_1.weight"], "ln1_b": lw["ln_1.bias"], "ln2_w": lw["ln_2.weight"], "ln2_b": lw["ln_2.bias"],
    }


# ---------------------------------------------------------------------------- shard IO
def load_embedding(shards_path: str, device="cpu", dtype=None) -> tuple:
    """(wte, wpe) from the reference's nested ``embedding.pth``."""
    d = torch.load(os.path.join(shards_path, "embedding.pth"), map_location=device, weights_only=True)
    wte, wpe = d["wte"]["weight"], d["wpe"]["weight"]
    if dtype is not None:
        wte, wpe = wte.to(dtype), wpe.to(dtype)
    return wte, wpe


def load_ln_f(shards_path: str, device="cpu", dtype=None) -> tuple:
    d = torch.load(os.path.join(shards_path, "ln_f.pth"), map_location=device, weights_only=True)
    w, b = d["weight"], d["bias"]
    return (w.to(dtype), b.to(dtype)) if dtype is not None else (w, b)


def load_block(shards_path: str, i: int, device="cpu", dtype=None) -> dict:
    d = torch.load(os.path.join(shards_path, f"block_{i}.pth"), map_location=device, weights_only=True)
    missing = [k for k in GPT2_LAYER_KEYS if k not in d]
    if missing:
        raise KeyError(f"block_{i}.pth is missing GPT-2 keys {missing}")
    # older transformers also persisted the causal-mask buffers attn.bias / attn.masked_bias
    return {k: (d[k].to(dtype) if dtype is not None else d[k]) for k in GPT2_LAYER_KEYS}


def load_lm_head(shards_path: str, device="cpu", dtype=None) -> torch.Tensor:
    p = os.path.join(shards_path, "lm_head.pth")
    if os.path.exists(p):
        w = torch.load(p, map_location=device, weights_only=True)["weight"]
        return w.to(dtype) if dtype is not None else w
    return load_embedding(shards_path, device, dtype)[0]


def write_random_shards(cfg: LlamaConfig, folder: str, dtype=torch.bfloat16, seed: int = 0) -> str:
    """A complete random-init GPT-2 shard folder in the reference format."""
    os.makedirs(folder, exist_ok=True)
    cfg.save_pretrained(folder)
    wte = random_wte(cfg, dtype, seed=seed)
    torch.save({"wte": {"weight": wte}, "wpe": {"weight": random_wpe(cfg, dtype, seed=seed)}, "drop": {}},
               os.path.join(folder, "embedding.pth"))
    for i in range(cfg.num_hidden_layers):
        torch.save(random_layer(cfg, i, dtype, seed=seed), os.path.join(folder, f"block_{i}.pth"))
    w, b = random_ln_f(cfg, dtype, seed=seed)
    torch.save({"weight": w, "bias": b}, os.path.join(folder, "ln_f.pth"))
    torch.save({"weight": wte.clone()}, os.path.join(folder, "lm_head.pth"))
    return folder


# ---------------------------------------------------------------------------- golden forward
def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps)


def gelu_new(x: torch.Tensor) -> torch.Tensor:
    return 0.5 * x * (1.0 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x.pow(3))))


def forward_full(cfg: LlamaConfig, wte: torch.Tensor, wpe: torch.Tensor, layers: list, ln_f: tuple,
                 ids: torch.Tensor, lm_head: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 causal forward of a whole sequence ``ids`` [S] -> logits [S, V] (no KV cache)."""
    S = ids.numel()
    nh, hd = cfg.num_attention_heads, cfg.head_dim
    h = wte[ids].float() + wpe[:S].float()
    mask = torch.ones(S, S, dtype=torch.bool).tril()
    for lw in layers:
        x = layer_norm(h, lw["ln_1.weight"], lw["ln_1.bias"], cfg.rms_norm_eps)
        qkv = x @ lw["attn.c_attn.weight"].float() + lw["attn.c_attn.bias"].float()
        q, k, v = qkv.split(cfg.hidden_size, dim=-1)
        q, k, v = (t.view(S, nh, hd).transpose(0, 1) for t in (q, k, v))
        sc = (q @ k.transpose(-1, -2)) * hd ** -0.5
        p = torch.softmax(sc.masked_fill(~mask, float("-inf")), -1)
        o = (p @ v).transpose(0, 1).reshape(S, cfg.hidden_size)
        h = h + o @ lw["attn.c_proj.weight"].float() + lw["attn.c_proj.bias"].float()
        x = layer_norm(h, lw["ln_2.weight"], lw["ln_2.bias"], cfg.rms_norm_eps)
        a = gelu_new(x @ lw["mlp.c_fc.weight"].float() + lw["mlp.c_fc.bias"].float())
        h = h + a @ lw["mlp.c_proj.weight"].float() + lw["mlp.c_proj.bias"].float()
    x = layer_norm(h, ln_f[0], ln_f[1], cfg.rms_norm_eps)
    return x @ (wte if lm_head is None else lm_head).float().t()


def greedy_generate(cfg: LlamaConfig, wte, wpe, layers, ln_f, prompt: list, n_new: int) -> list:
    """Greedy decode by full recompute (oracle for the cached engine)."""
    ids = list(prompt)
    out = []
    for _ in range(n_new):
        t = int(forward_full(cfg, wte, wpe, layers, ln_f, torch.tensor(ids))[-1].argmax())
        out.append(t)
        ids.append(t)
    return out


__all__ = ["GPT2_LAYER_KEYS", "layer_shapes", "random_layer", "random_wte", "random_wpe", "random_ln_f",
           "to_linear", "load_embedding", "load_ln_f", "load_block", "load_lm_head", "write_random_shards",
           "layer_norm", "gelu_new", "forward_full", "greedy_generate"]
