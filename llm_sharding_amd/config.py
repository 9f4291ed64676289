"""Model configuration for the Llama decoder family served by this engine.

The reference reads hyper-parameters from the HF ``config.json`` stored inside the shard
folder (``/root/reference/utils/node_worker.py:88`` -> ``LlamaConfig.from_pretrained``).
We parse the same file ourselves (no transformers dependency on the hot path) and provide
presets for the models the reference is configured with:

* Llama-2-7B  (``/root/reference/utils/node_worker.py:564``, ``inference.py:11``)
* Llama-3.2-3B-Instruct (``/root/reference/start_node.py:14``, 28 layers: ``node_profiler.py:1207``)
* Llama-2-70B (BASELINE.json config 4)

plus tiny configs used by the CPU test-suite.

The same dataclass also describes **GPT-2** (``model_type == "gpt2"``): the reference's
sharder writes GPT-2 shards (``/root/reference/utils/model_sharder.py:96-132``) but nothing in
the reference can load or run them. Here GPT-2 is a served family: pre-LN
LayerNorm with bias, learned absolute positions (no RoPE), Conv1D projections with biases,
tanh-GELU MLP, tied lm_head. HF GPT-2 ``config.json`` keys (``n_embd``, ``n_layer``,
``n_head``, ``n_positions``, ``n_inner``, ``layer_norm_epsilon``) are mapped on load.
"""
from __future__ import annotations

import dataclasses
import json
import math
import os
from typing import Any, Optional


@dataclasses.dataclass
class LlamaConfig:
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 32
    head_dim: int = 128
    vocab_size: int = 32000
    max_position_embeddings: int = 4096
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    rope_scaling: Optional[dict] = None
    tie_word_embeddings: bool = False
    bos_token_id: int = 1
    eos_token_id: Any = 2
    model_type: str = "llama"
    name: str = "llama"

    # ------------------------------------------------------------------ derived
    @property
    def q_size(self) -> int:
        return self.num_attention_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_key_value_heads * self.head_dim

    @property
    def qkv_size(self) -> int:
        return self.q_size + 2 * self.kv_size

    @property
    def is_gpt2(self) -> bool:
        return self.model_type == "gpt2"

    @property
    def mlp_in_size(self) -> int:
        """Output width of the fused MLP input projection (gate|up for SwiGLU, c_fc for GPT-2)."""
        return self.intermediate_size if self.is_gpt2 else 2 * self.intermediate_size

    @property
    def head_rows(self) -> int:
        """lm_head rows as served: the vocabulary padded to whole 128-column groups (8 MFMA
        tiles, so every GEMV / coop tiling applies; GPT-2's 50257 -> 50304; Llama vocabularies
        are already multiples). Padding rows copy row 0, so they never win the argmax tie-break."""
        return -(-self.vocab_size // 128) * 128

    @property
    def gqa_group(self) -> int:
        return self.num_attention_heads // self.num_key_value_heads

    @property
    def eos_ids(self) -> list:
        e = self.eos_token_id
        if e is None:
            return []
        return list(e) if isinstance(e, (list, tuple)) else [int(e)]

    def layer_param_count(self) -> int:
        H, I = self.hidden_size, self.intermediate_size
        if self.is_gpt2:  # c_attn, c_proj, c_fc, mlp.c_proj (+ biases), ln_1, ln_2 (+ biases)
            return H * self.qkv_size + self.qkv_size + H * H + H + 2 * H * I + I + H + 4 * H
        return H * self.qkv_size + self.q_size * H + 3 * H * I + 2 * H

    def layer_bytes(self, elem_bytes: int = 2) -> int:
        return self.layer_param_count() * elem_bytes

    def kv_bytes_per_token_per_layer(self, elem_bytes: int = 2) -> int:
        return 2 * self.kv_size * elem_bytes

    def validate(self) -> None:
        if self.num_attention_heads % self.num_key_value_heads:
            raise ValueError("num_attention_heads must be a multiple of num_key_value_heads")
        if self.head_dim % 16 or self.head_dim & (self.head_dim - 1):
            raise ValueError("head_dim must be a power of two >= 16")

    # ------------------------------------------------------------------ IO
    @classmethod
    def from_dict(cls, d: dict) -> "LlamaConfig":
        if d.get("model_type") == "gpt2" and "n_embd" in d:  # HF GPT2Config keys
            H = int(d["n_embd"])
            m = {"hidden_size": H, "num_hidden_layers": d.get("n_layer", 12),
                 "num_attention_heads": d.get("n_head", 12), "num_key_value_heads": d.get("n_head", 12),
                 "head_dim": H // int(d.get("n_head", 12)),
                 "intermediate_size": d.get("n_inner") or 4 * H,
                 "max_position_embeddings": d.get("n_positions", 1024),
                 "rms_norm_eps": d.get("layer_norm_epsilon", 1e-5), "tie_word_embeddings": True}
            if d.get("activation_function", "gelu_new") not in ("gelu_new", "gelu_pytorch_tanh"):
                raise ValueError(f"unsupported GPT-2 activation {d.get('activation_function')!r}")
            d = {**{k: v for k, v in d.items() if k not in ("n_embd", "n_layer", "n_head", "n_inner",
                                                              "n_positions", "layer_norm_epsilon")}, **m}
        rp = d.get("rope_parameters")
        if isinstance(rp, dict):  # transformers >= 5 writes theta + scaling as one "rope_parameters" dict
            d = dict(d)
            d.setdefault("rope_theta", rp.get("rope_theta", cls.rope_theta))
            if rp.get("rope_type", "default") != "default" and not d.get("rope_scaling"):
                d["rope_scaling"] = {k: v for k, v in rp.items() if k != "rope_theta"}
        fields = {f.name for f in dataclasses.fields(cls)}
        kw = {k: v for k, v in d.items() if k in fields}
        if "num_key_value_heads" not in d or d.get("num_key_value_heads") is None:
            kw["num_key_value_heads"] = d.get("num_attention_heads", cls.num_attention_heads)
        if "head_dim" not in d or d.get("head_dim") is None:
            kw["head_dim"] = d.get("hidden_size", cls.hidden_size) // d.get(
                "num_attention_heads", cls.num_attention_heads)
        if "_name_or_path" in d and "name" not in d:
            kw["name"] = os.path.basename(str(d["_name_or_path"]).rstrip("/")) or "llama"
        cfg = cls(**kw)
        cfg.validate()
        return cfg

    @classmethod
    def from_pretrained(cls, path: str) -> "LlamaConfig":
        """Same entry point name as HF's ``LlamaConfig.from_pretrained`` (reads ``config.json``)."""
        p = os.path.join(path, "config.json") if os.path.isdir(path) else path
        with open(p, "r") as f:
            d = json.load(f)
        if "name" not in d:
            d["name"] = os.path.basename(os.path.dirname(os.path.abspath(p)))
        return cls.from_dict(d)

    def to_dict(self) -> dict:
        d = dataclasses.asdict(self)
        d["torch_dtype"] = "bfloat16"
        if self.is_gpt2:  # HF GPT2Config layout (readable by transformers as well)
            for k in ("hidden_size", "num_hidden_layers", "num_attention_heads", "num_key_value_heads",
                      "head_dim", "intermediate_size", "max_position_embeddings", "rms_norm_eps",
                      "rope_theta", "rope_scaling"):
                d.pop(k)
            d.update({"architectures": ["GPT2LMHeadModel"], "n_embd": self.hidden_size,
                      "n_layer": self.num_hidden_layers, "n_head": self.num_attention_heads,
                      "n_inner": self.intermediate_size, "n_positions": self.max_position_embeddings,
                      "layer_norm_epsilon": self.rms_norm_eps, "activation_function": "gelu_new"})
            return d
        d["architectures"] = ["LlamaForCausalLM"]
        return d

    def save_pretrained(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "config.json"), "w") as f:
            json.dump(self.to_dict(), f, indent=2)


# ---------------------------------------------------------------------- presets
def llama2_7b() -> LlamaConfig:
    return LlamaConfig(name="Llama-2-7b-chat-hf")


def llama2_13b() -> LlamaConfig:
    return LlamaConfig(hidden_size=5120, intermediate_size=13824, num_hidden_layers=40,
                       num_attention_heads=40, num_key_value_heads=40, name="Llama-2-13b-chat-hf")


def llama2_70b() -> LlamaConfig:
    return LlamaConfig(hidden_size=8192, intermediate_size=28672, num_hidden_layers=80,
                       num_attention_heads=64, num_key_value_heads=8, name="Llama-2-70b-chat-hf")


def llama32_3b() -> LlamaConfig:
    return LlamaConfig(hidden_size=3072, intermediate_size=8192, num_hidden_layers=28,
                       num_attention_heads=24, num_key_value_heads=8, head_dim=128,
                       vocab_size=128256, max_position_embeddings=131072, rms_norm_eps=1e-5,
                       rope_theta=500000.0,
                       rope_scaling={"rope_type": "llama3", "factor": 32.0,
                                     "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                     "original_max_position_embeddings": 8192},
                       tie_word_embeddings=True, bos_token_id=128000,
                       eos_token_id=[128001, 128008, 128009], name="Llama-3___2-3B-Instruct")


def tiny(layers: int = 4, hidden: int = 256, heads: int = 4, kv_heads: int = 2,
         head_dim: int = 64, inter: int = 512, vocab: int = 512, llama3: bool = False) -> LlamaConfig:
    """Small config for CPU tests (shapes respect every kernel's tiling constraints)."""
    cfg = LlamaConfig(hidden_size=hidden, intermediate_size=inter, num_hidden_layers=layers,
                      num_attention_heads=heads, num_key_value_heads=kv_heads, head_dim=head_dim,
                      vocab_size=vocab, max_position_embeddings=2048, name="tiny-llama",
                      bos_token_id=1, eos_token_id=2)
    if llama3:
        cfg.rope_theta = 500000.0
        cfg.rope_scaling = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                            "high_freq_factor": 4.0, "original_max_position_embeddings": 256}
    return cfg


def gpt2(size: str = "small") -> LlamaConfig:
    """GPT-2 124M / medium 355M / large 774M / xl 1.5B (HF ``gpt2*`` configs)."""
    H, L, nh = {"small": (768, 12, 12), "medium": (1024, 24, 16), "large": (1280, 36, 20),
                "xl": (1600, 48, 25)}[size]
    return LlamaConfig(hidden_size=H, intermediate_size=4 * H, num_hidden_layers=L, num_attention_heads=nh,
                       num_key_value_heads=nh, head_dim=H // nh, vocab_size=50257, max_position_embeddings=1024,
                       rms_norm_eps=1e-5, tie_word_embeddings=True, bos_token_id=50256, eos_token_id=50256,
                       model_type="gpt2", name="gpt2" if size == "small" else f"gpt2-{size}")


def tiny_gpt2(layers: int = 4, hidden: int = 256, heads: int = 4, vocab: int = 500) -> LlamaConfig:
    """Small GPT-2 for CPU tests (vocab deliberately not a multiple of 16)."""
    return LlamaConfig(hidden_size=hidden, intermediate_size=4 * hidden, num_hidden_layers=layers,
                       num_attention_heads=heads, num_key_value_heads=heads, head_dim=hidden // heads,
                       vocab_size=vocab, max_position_embeddings=512, tie_word_embeddings=True,
                       bos_token_id=vocab - 1, eos_token_id=vocab - 1, model_type="gpt2", name="tiny-gpt2")


PRESETS = {
    "llama2-7b": llama2_7b,
    "llama2-13b": llama2_13b,
    "llama2-70b": llama2_70b,
    "llama3.2-3b": llama32_3b,
    "tiny": tiny,
    "tiny8": lambda: tiny(layers=8),  # one layer per stage on 8 ranks (N=8 schedule rehearsal)
    "gpt2": gpt2,
    "gpt2-medium": lambda: gpt2("medium"),
    "gpt2-large": lambda: gpt2("large"),
    "gpt2-xl": lambda: gpt2("xl"),
    "tiny-gpt2": tiny_gpt2,
}


def get_preset(name: str) -> LlamaConfig:
    key = name.lower().replace("_", "-")
    if key not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; known: {sorted(PRESETS)}")
    return PRESETS[key]()


def dtype_suffix(dtype) -> str:
    """Shard-folder suffix: ``str(dtype).split('.')[-1]`` (reference ``model_sharder.py:24``)."""
    return str(dtype).split(".")[-1]


def ceil_div(a: int, b: int) -> int:
    return -(-a // b)


def round_up(a: int, b: int) -> int:
    return ceil_div(a, b) * b


def human_bytes(n: float) -> str:
    for unit in ("B", "KiB", "MiB", "GiB", "TiB"):
        if abs(n) < 1024 or unit == "TiB":
            return f"{n:.2f} {unit}"
        n /= 1024
    return f"{n:.2f} TiB"


__all__ = ["LlamaConfig", "llama2_7b", "llama2_13b", "llama2_70b", "llama32_3b", "tiny", "gpt2", "tiny_gpt2",
           "get_preset", "dtype_suffix", "ceil_div", "round_up", "human_bytes", "math"]
