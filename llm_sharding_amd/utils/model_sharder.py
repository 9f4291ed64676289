"""Offline weight splitter (reference C6, ``utils/model_sharder.py:7-134``).

``ModelSharder(model_path, model_type, shard_save_folder, device="cpu", dtype=torch.float32)``
and ``save_shards()`` write the reference on-disk format into
``<shard_save_folder>_<dtype>``: every non-weight file copied, then

* llama: ``embedding.pth {"weight"}``, ``block_{i}.pth`` (``LlamaDecoderLayer`` keys),
  ``final_norm.pth {"weight"}``, ``lm_head.pth {"weight"}``
* gpt (GPT-2): ``embedding.pth {"wte": {...}, "wpe": {...}, "drop": {}}``, ``block_{i}.pth``,
  ``ln_f.pth``, ``lm_head.pth``

Unlike the reference (``AutoModelForCausalLM.from_pretrained`` of the whole model, which
needs a device able to hold it), the checkpoint is streamed tensor by tensor from its
``*.safetensors`` shards (zero-copy mmap) or ``pytorch_model*.bin`` files (read with
``torch.load(weights_only=True, mmap=True)``), so a 70B model shards on a small host.

Quantised shards. The reference's ``dtype=torch.int8 / torch.int4`` branch
(``/root/reference/utils/model_sharder.py:28-39``) hands the model to bitsandbytes
(CUDA-only) and has no loader for the result (Q12). Here every 2-D projection / head
matrix is quantised by the sharder itself and the loader (models/weights.py) dequantises
it to bf16; norms and the embedding stay bf16 (suffixes as in the reference:
``_int8``, ``_int4``, ``_float8_e4m3fn``):

* ``torch.float8_e4m3fn`` - OCP FP8 (MI355X-native, decodes on the W8A16 fp8 kernels with
  ``weight_dtype="fp8"``): ``<name>`` e4m3 [N, K] + ``<name>_scale`` fp32 [N];
* ``torch.int8`` - symmetric per-output-channel int8: ``<name>`` int8 [N, K] +
  ``<name>_scale`` fp32 [N] (w ~= q * scale, |q| <= 127);
* ``torch.int4`` - symmetric group-wise int4 (``INT4_GROUP`` = 128 input channels per
  scale), two values per byte, even k in the low nibble: ``<name>`` uint8 [N, K/2] +
  ``<name>_scale`` fp32 [N, K/128] (|q| <= 7).
"""
from __future__ import annotations

import glob
import json
import math
import os
import re
import shutil
from typing import Iterator

import torch

from ..config import dtype_suffix

FP8 = getattr(torch, "float8_e4m3fn", None)


def _iter_checkpoint(model_path: str) -> Iterator[tuple]:
    """Yield (name, tensor) for every tensor of an HF checkpoint directory, lazily."""
    st = sorted(glob.glob(os.path.join(model_path, "*.safetensors")))
    if st:
        from safetensors import safe_open
        for f in st:
            with safe_open(f, framework="pt", device="cpu") as fh:
                for k in fh.keys():
                    yield k, fh.get_tensor(k)
        return
    bins = sorted(glob.glob(os.path.join(model_path, "pytorch_model*.bin")) +
                  glob.glob(os.path.join(model_path, "*.pth")))
    if not bins:
        raise FileNotFoundError(f"no *.safetensors / pytorch_model*.bin in {model_path}")
    for f in bins:
        sd = torch.load(f, map_location="cpu", weights_only=True, mmap=True)
        for k, v in sd.items():
            yield k, v


INT4_GROUP = 128


def quantize_int8(w: torch.Tensor) -> tuple:
    """Per-output-channel symmetric int8: w ~= q * scale[:, None], q in [-127, 127]."""
    scale = w.float().abs().amax(dim=1).clamp(min=1e-12) / 127.0
    q = torch.round(w.float() / scale[:, None]).clamp(-127, 127).to(torch.int8)
    return q, scale


def quantize_int4(w: torch.Tensor, group: int = INT4_GROUP) -> tuple:
    """Group-wise symmetric int4 packed two per byte (even k -> low nibble):
    w[n, k] ~= q[n, k] * scale[n, k // group], q in [-7, 7]."""
    N, K = w.shape
    group = math.gcd(K, group)  # narrow matrices (K not a multiple of 128): the largest divisor
    if group % 2:
        raise ValueError(f"int4 needs an even input dimension, got K={K}")
    wg = w.float().reshape(N, K // group, group)
    scale = wg.abs().amax(dim=2).clamp(min=1e-12) / 7.0
    q = torch.round(wg / scale[:, :, None]).clamp(-7, 7).to(torch.int8).reshape(N, K)
    u = (q & 0xF).to(torch.uint8)
    return (u[:, 0::2] | (u[:, 1::2] << 4)).contiguous(), scale


def dequantize_int4(packed: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    """Inverse of :func:`quantize_int4` -> fp32 [N, K]."""
    N = packed.shape[0]
    lo = (packed & 0xF).to(torch.int8)
    hi = (packed >> 4).to(torch.int8)
    q = torch.stack((lo, hi), dim=2).reshape(N, -1)
    q = torch.where(q > 7, q - 16, q).float()
    G = q.shape[1] // scale.shape[1]
    return (q.reshape(N, scale.shape[1], G) * scale.float()[:, :, None]).reshape(N, -1)


QUANT_DTYPES = tuple(d for d in (FP8, torch.int8, getattr(torch, "int4", None)) if d is not None)


def quantize_fp8(w: torch.Tensor) -> tuple:
    """Per-output-channel symmetric OCP e4m3 quantisation: w ~= q * scale[:, None]."""
    amax = w.float().abs().amax(dim=1).clamp(min=1e-12)
    scale = amax / 448.0
    q = (w.float() / scale[:, None]).clamp(-448.0, 448.0).to(FP8)
    return q, scale


class ModelSharder:
    LLAMA_LAYER = re.compile(r"^model\.layers\.(\d+)\.(.+)$")
    GPT_LAYER = re.compile(r"^(?:transformer\.)?h\.(\d+)\.(.+)$")

    def __init__(self, model_path: str, model_type: str, shard_save_folder: str, device="cpu",
                 dtype=torch.float32, verbose: bool = True):
        self.model_path = model_path
        self.model_type = model_type
        self.device = torch.device(device)
        self.dtype = dtype
        self.verbose = verbose
        self.shard_save_folder = shard_save_folder + "_" + dtype_suffix(dtype)
        os.makedirs(self.shard_save_folder, exist_ok=True)

    def _log(self, m: str) -> None:
        if self.verbose:
            print(m, flush=True)

    def _cast(self, name: str, t: torch.Tensor) -> dict:
        """Return {name: tensor} (and a scale for quantised matrices)."""
        if not t.is_floating_point():
            return {name: t}
        if self.dtype in QUANT_DTYPES:
            if t.dim() == 2 and name.endswith("weight"):
                if self.dtype == torch.int8:
                    q, s = quantize_int8(t)
                elif self.dtype == FP8:
                    q, s = quantize_fp8(t)
                else:
                    q, s = quantize_int4(t)
                return {name: q, name + "_scale": s}
            return {name: t.to(torch.bfloat16)}
        return {name: t.to(self.dtype)}

    def _copy_non_weight_files(self) -> None:
        for fn in os.listdir(self.model_path):
            if fn.endswith((".bin", ".safetensors", ".pth")) or fn == "original":
                continue
            src = os.path.join(self.model_path, fn)
            if os.path.isfile(src):
                shutil.copyfile(src, os.path.join(self.shard_save_folder, fn))
                self._log(f"Copied {fn} -> {self.shard_save_folder}")

    def _save(self, d: dict, name: str) -> None:
        torch.save({k: v.contiguous() for k, v in d.items()}, os.path.join(self.shard_save_folder, name))

    def save_shards(self) -> str:
        self._copy_non_weight_files()
        if self.model_type == "llama":
            self._save_llama()
        elif self.model_type in ("gpt", "gpt2"):
            self._save_gpt()
        else:
            raise ValueError(f"[ERROR] Unsupported model type: {self.model_type}")
        self._log("Sharding complete.")
        return self.shard_save_folder

    # Layers are flushed as soon as the next layer index appears (HF checkpoints are ordered by
    # layer), so peak host memory is about one layer plus one checkpoint file's mmap.
    def _save_llama(self) -> None:
        blocks: dict = {}
        embed = final = head = None
        done = set()
        for name, t in _iter_checkpoint(self.model_path):
            m = self.LLAMA_LAYER.match(name)
            if m:
                i = int(m.group(1))
                blocks.setdefault(i, {}).update(self._cast(m.group(2), t))
                for j in [j for j in blocks if j < i - 1]:
                    self._save(blocks.pop(j), f"block_{j}.pth")
                    done.add(j)
                    self._log(f"Saved block {j}")
            elif name == "model.embed_tokens.weight":
                embed = t
            elif name == "model.norm.weight":
                final = t
            elif name == "lm_head.weight":
                head = t
        for j in sorted(blocks):
            self._save(blocks[j], f"block_{j}.pth")
            done.add(j)
            self._log(f"Saved block {j}")
        if embed is None or final is None:
            raise KeyError("checkpoint lacks model.embed_tokens.weight / model.norm.weight")
        emb = {"weight": embed.to(torch.bfloat16 if self.dtype in QUANT_DTYPES else self.dtype)}
        self._save(emb, "embedding.pth")
        self._save({"weight": final.to(emb["weight"].dtype)}, "final_norm.pth")
        self._save(self._cast("weight", head if head is not None else embed), "lm_head.pth")
        self._log(f"Saved embedding, {len(done)} blocks, final normalization and lm_head.")

    def _save_gpt(self) -> None:
        blocks: dict = {}
        wte = wpe = None
        lnf: dict = {}
        head = None
        for name, t in _iter_checkpoint(self.model_path):
            m = self.GPT_LAYER.match(name)
            if m:
                blocks.setdefault(int(m.group(1)), {}).update(self._cast(m.group(2), t))
            elif name.endswith("wte.weight"):
                wte = t
            elif name.endswith("wpe.weight"):
                wpe = t
            elif ".ln_f." in name or name.startswith("ln_f."):
                lnf[name.split("ln_f.")[-1]] = t
            elif name == "lm_head.weight":
                head = t
        dt = torch.bfloat16 if self.dtype in QUANT_DTYPES else self.dtype
        # nested dict layout of the reference (model_sharder.py:109-113)
        torch.save({"wte": {"weight": wte.to(dt)}, "wpe": {"weight": wpe.to(dt)}, "drop": {}},
                   os.path.join(self.shard_save_folder, "embedding.pth"))
        for j in sorted(blocks):
            self._save(blocks[j], f"block_{j}.pth")
        self._save({k: v.to(dt) for k, v in lnf.items()}, "ln_f.pth")
        self._save({"weight": (head if head is not None else wte).to(dt)}, "lm_head.pth")


def write_hf_llama_checkpoint(cfg, path: str, embed: torch.Tensor, layers: list, final_norm: torch.Tensor,
                              lm_head: torch.Tensor, n_files: int = 2) -> None:
    """Write an HF-format Llama checkpoint (config + sharded safetensors + index). Used to
    exercise ModelSharder offline (no real checkpoints are available)."""
    from safetensors.torch import save_file
    os.makedirs(path, exist_ok=True)
    d = cfg.to_dict()
    d.update({"model_type": "llama", "architectures": ["LlamaForCausalLM"]})
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(d, f, indent=1)
    names = {"model.embed_tokens.weight": embed, "model.norm.weight": final_norm, "lm_head.weight": lm_head}
    for i, lw in enumerate(layers):
        for k, v in lw.items():
            names[f"model.layers.{i}.{k}"] = v
    keys = list(names)
    per = -(-len(keys) // n_files)
    index = {"metadata": {}, "weight_map": {}}
    for fi in range(n_files):
        chunk = keys[fi * per:(fi + 1) * per]
        fn = f"model-{fi + 1:05d}-of-{n_files:05d}.safetensors"
        save_file({k: names[k].contiguous() for k in chunk}, os.path.join(path, fn))
        for k in chunk:
            index["weight_map"][k] = fn
    with open(os.path.join(path, "model.safetensors.index.json"), "w") as f:
        json.dump(index, f)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser(description="split an HF checkpoint into per-layer shards")
    ap.add_argument("model_path")
    ap.add_argument("shard_save_folder")
    ap.add_argument("--model-type", default="llama")
    ap.add_argument("--dtype", default="bfloat16")
    a = ap.parse_args()
    ModelSharder(a.model_path, a.model_type, a.shard_save_folder, dtype=getattr(torch, a.dtype)).save_shards()
