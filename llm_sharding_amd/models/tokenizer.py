"""Tokenizers.

The reference loads ``AutoTokenizer.from_pretrained(shards_path)``
(``/root/reference/utils/node_worker.py:118``). No tokenizer files exist offline, so a
shard folder written by :func:`write_random_shards` carries a tiny deterministic byte-level
tokenizer instead. When real tokenizer files are present, transformers' ``AutoTokenizer`` is
used (it is importable here), so real checkpoints keep their real tokenizer.

The synthetic tokenizer exposes the subset of the HF API the reference touches:
``tok(text, return_tensors="pt")["input_ids"]``, ``decode(ids)``, ``eos_token``,
``eos_token_id``.
"""
from __future__ import annotations

import json
import os

import torch

SYNTH_CLASS = "SyntheticByteTokenizer"


class SyntheticByteTokenizer:
    """ids: 0=<pad>, bos, eos, then byte b -> ``offset + b``; ids beyond the byte range decode
    to ``<tok{id}>`` (random models emit arbitrary ids)."""

    def __init__(self, vocab_size: int = 32000, bos_token_id: int = 1, eos_token_id: int = 2):
        self.vocab_size = int(vocab_size)
        self.bos_token_id = int(bos_token_id)
        self.eos_token_id = int(eos_token_id)
        self.offset = 3
        self.eos_token = "</s>"
        self.bos_token = "<s>"
        self.pad_token_id = 0

    # HF-like call
    def __call__(self, text, return_tensors=None, add_special_tokens: bool = True):
        texts = [text] if isinstance(text, str) else list(text)
        rows = [self.encode(t, add_special_tokens) for t in texts]
        if return_tensors == "pt":
            L = max(len(r) for r in rows)
            ids = torch.full((len(rows), L), self.pad_token_id, dtype=torch.long)
            mask = torch.zeros((len(rows), L), dtype=torch.long)
            for i, r in enumerate(rows):
                ids[i, :len(r)] = torch.tensor(r)
                mask[i, :len(r)] = 1
            return _BatchEncoding(input_ids=ids, attention_mask=mask)
        return {"input_ids": rows if len(rows) > 1 else rows[0]}

    def encode(self, text: str, add_special_tokens: bool = True) -> list:
        ids = [self.bos_token_id] if add_special_tokens else []
        for b in text.encode("utf-8"):
            t = self.offset + b
            ids.append(t if t < self.vocab_size else self.offset + (b % max(1, self.vocab_size - self.offset)))
        return ids

    def _piece(self, i: int) -> str:
        if i == self.eos_token_id:
            return self.eos_token
        if i == self.bos_token_id:
            return self.bos_token
        if i == self.pad_token_id:
            return ""
        b = i - self.offset
        if 0 <= b < 256:
            return bytes([b]).decode("latin-1")
        return f"<tok{i}>"

    def decode(self, ids, skip_special_tokens: bool = False) -> str:
        if isinstance(ids, torch.Tensor):
            ids = ids.reshape(-1).tolist()
        elif isinstance(ids, int):
            ids = [ids]
        out = []
        for i in ids:
            i = int(i)
            if skip_special_tokens and i in (self.eos_token_id, self.bos_token_id, self.pad_token_id):
                continue
            out.append(self._piece(i))
        return "".join(out)

    def save_pretrained(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "tokenizer_config.json"), "w") as f:
            json.dump({"tokenizer_class": SYNTH_CLASS, "vocab_size": self.vocab_size,
                       "bos_token_id": self.bos_token_id, "eos_token_id": self.eos_token_id,
                       "eos_token": self.eos_token, "bos_token": self.bos_token}, f, indent=2)

    @classmethod
    def from_pretrained(cls, path: str) -> "SyntheticByteTokenizer":
        with open(os.path.join(path, "tokenizer_config.json")) as f:
            d = json.load(f)
        return cls(d.get("vocab_size", 32000), d.get("bos_token_id", 1), d.get("eos_token_id", 2))


class _BatchEncoding(dict):
    def __init__(self, **kw):
        super().__init__(**kw)

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def to(self, device):
        return _BatchEncoding(**{k: v.to(device) for k, v in self.items()})


def load_tokenizer(path: str):
    """AutoTokenizer-equivalent: synthetic tokenizer for random shards, HF otherwise."""
    cfg_p = os.path.join(path, "tokenizer_config.json")
    if os.path.exists(cfg_p):
        with open(cfg_p) as f:
            d = json.load(f)
        if d.get("tokenizer_class") == SYNTH_CLASS:
            return SyntheticByteTokenizer.from_pretrained(path)
    has_real = any(os.path.exists(os.path.join(path, n)) for n in
                   ("tokenizer.json", "tokenizer.model", "vocab.json"))
    if has_real:
        from transformers import AutoTokenizer  # real checkpoints only
        return AutoTokenizer.from_pretrained(path)
    # No tokenizer at all: fall back to the synthetic one sized from config.json.
    vocab = 32000
    cp = os.path.join(path, "config.json")
    if os.path.exists(cp):
        with open(cp) as f:
            vocab = json.load(f).get("vocab_size", vocab)
    return SyntheticByteTokenizer(vocab)
