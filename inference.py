#!/usr/bin/env python3
"""Single-process greedy generation (reference inference.py, which calls HF generate): the
whole model on one device through the MI355X engine (hipGraph decode on GPU).

    python inference.py --shards DIR [--prompt "..."] [--max-new-tokens 128]
    python inference.py --random llama2-7b --max-new-tokens 64     # random-init weights
    python inference.py --shards DIR --hf-compare HF_DIR           # + the reference's own path

``--hf-compare HF_DIR`` also runs what the reference's inference.py runs
(/root/reference/inference.py:16-45: transformers' AutoModelForCausalLM + greedy generate) on the
HF checkpoint the shards were cut from, in fp32 on the CPU, and reports where the two greedy
decodes agree (tests/test_llama_hf_parity.py pins the same parity in the test suite).
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from llm_sharding_amd.config import LlamaConfig, get_preset  # noqa: E402
from llm_sharding_amd.models.tokenizer import SyntheticByteTokenizer, load_tokenizer  # noqa: E402
from llm_sharding_amd.runtime.engine import DecodeGraph, RandomSource, ShardFolderSource, StageEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", default="")
    ap.add_argument("--random", default="", help="preset name for random-init weights (no checkpoint)")
    ap.add_argument("--prompt", default="Write a poem about the blue sky.")
    ap.add_argument("--max-new-tokens", type=int, default=128)
    ap.add_argument("--device", default="cuda:0" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--hf-compare", default="", help="HF checkpoint dir: also run transformers' greedy generate "
                                                     "(the reference inference.py's path, fp32 CPU) and compare tokens")
    a = ap.parse_args()
    if a.shards:
        cfg = LlamaConfig.from_pretrained(a.shards)
        src, tok = ShardFolderSource(a.shards, cfg), load_tokenizer(a.shards)
    else:
        cfg = get_preset(a.random or "tiny")
        src, tok = RandomSource(cfg), SyntheticByteTokenizer(cfg.vocab_size)
    dt = torch.bfloat16 if a.device.startswith("cuda") else torch.float32
    t0 = time.perf_counter()
    eng = StageEngine(cfg, 0, cfg.num_hidden_layers, a.device, dt, has_embed=True, has_head=True, source=src,
                      max_seq=min(cfg.max_position_embeddings, 4096))
    ids = tok(a.prompt, return_tensors="pt")["input_ids"][0]
    print(f"[INFO] loaded in {time.perf_counter() - t0:.1f}s; prompt tokens {ids.numel()}")
    slot, pos = eng.prefill_rows([0], [ids.numel()])
    h = eng.forward(eng.embed(ids.to(a.device)), slot, pos)
    eng.advance([0], [ids.numel()])
    first = eng.head(h, [ids.numel() - 1])
    out = [int(first[0])]
    t1 = time.perf_counter()
    if eng.gpu:
        g = DecodeGraph(eng, 1, "full", history_len=a.max_new_tokens)
        g.tokens.copy_(first.to(torch.int32))
        g.capture()
        for _ in range(a.max_new_tokens - 1):
            g.replay()
        torch.cuda.synchronize()
        out += g.history[:a.max_new_tokens - 1, 0].tolist()
    else:
        cur = first
        for _ in range(a.max_new_tokens - 1):
            slot, pos = eng.prefill_rows([0], [1])
            h = eng.forward(eng.embed(cur), slot, pos)
            eng.advance([0], [1])
            cur = eng.head(h)
            out.append(int(cur[0]))
    dt_s = time.perf_counter() - t1
    eos = [i for i, t in enumerate(out) if t in cfg.eos_ids]
    if eos:
        out = out[:eos[0] + 1]
    print(tok.decode(ids.tolist() + out, skip_special_tokens=True))
    print(f"[INFO] {len(out)} new tokens, {max(1, len(out) - 1) / max(dt_s, 1e-9):.1f} tok/s decode")
    if a.hf_compare:
        hf = hf_greedy(a.hf_compare, ids, len(out))
        same = next((i for i, (x, y) in enumerate(zip(out, hf)) if x != y), len(out))
        print(f"[INFO] HF greedy (transformers, fp32 CPU) agrees on the first {same}/{len(out)} tokens"
              + ("" if same == len(out) else f"; first divergence at token {same}: ours {out[same]}, HF {hf[same]}"))
    return out


def hf_greedy(hf_dir: str, ids: torch.Tensor, n_new: int) -> list:
    """The reference's single-process path: AutoModelForCausalLM.from_pretrained + greedy
    generate (/root/reference/inference.py:16-45), here fp32 on the CPU as the oracle."""
    from transformers import AutoModelForCausalLM
    m = AutoModelForCausalLM.from_pretrained(hf_dir, dtype=torch.float32).eval()
    with torch.no_grad():
        g = m.generate(ids[None].cpu(), max_new_tokens=n_new, min_new_tokens=n_new, do_sample=False)
    return g[0, ids.numel():].tolist()


if __name__ == "__main__":
    main()
