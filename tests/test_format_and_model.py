"""CPU tests: config, on-disk shard format, tokenizer, packing, golden model, CPU engine."""
import json
import os

import torch

from llm_sharding_amd.config import LlamaConfig, get_preset, llama2_7b, llama32_3b, tiny
from llm_sharding_amd.models import weights as W
from llm_sharding_amd.models.reference import LAYER_KEYS, ReferenceLlama
from llm_sharding_amd.models.rope import inv_freq, rope_table
from llm_sharding_amd.models.tokenizer import SyntheticByteTokenizer, load_tokenizer
from llm_sharding_amd.ops import packing
from llm_sharding_amd.runtime.engine import RandomSource, ShardFolderSource, StageEngine


def test_presets():
    c = llama2_7b()
    assert c.qkv_size == 3 * 4096 and c.gqa_group == 1 and c.head_dim == 128
    c3 = llama32_3b()
    assert c3.gqa_group == 3 and c3.tie_word_embeddings and c3.num_hidden_layers == 28
    c70 = get_preset("llama2-70b")
    assert c70.kv_size == 1024 and c70.num_hidden_layers == 80
    # 7B layer weight bytes in bf16 ~ 404 MB
    assert abs(c.layer_bytes() / 1e6 - 404.8) < 1.0


def test_config_roundtrip(tmp_path):
    c = tiny(llama3=True)
    c.save_pretrained(str(tmp_path))
    c2 = LlamaConfig.from_pretrained(str(tmp_path))
    assert c2.rope_scaling == c.rope_scaling and c2.hidden_size == c.hidden_size
    # HF-style config without head_dim / num_key_value_heads
    d = {"hidden_size": 512, "num_attention_heads": 8, "num_hidden_layers": 2, "intermediate_size": 1024,
         "vocab_size": 100}
    c3 = LlamaConfig.from_dict(d)
    assert c3.head_dim == 64 and c3.num_key_value_heads == 8


def test_shard_folder_format(tiny_shards):
    files = set(os.listdir(tiny_shards))
    cfg = LlamaConfig.from_pretrained(tiny_shards)
    assert tiny_shards.endswith("_float32")
    for f in ["config.json", "generation_config.json", "embedding.pth", "final_norm.pth", "lm_head.pth",
              "tokenizer_config.json"] + [f"block_{i}.pth" for i in range(cfg.num_hidden_layers)]:
        assert f in files, f
    blk = torch.load(os.path.join(tiny_shards, "block_0.pth"), weights_only=True)
    assert set(blk) == set(LAYER_KEYS)
    assert blk["self_attn.k_proj.weight"].shape == (cfg.kv_size, cfg.hidden_size)
    emb = torch.load(os.path.join(tiny_shards, "embedding.pth"), weights_only=True)
    assert list(emb) == ["weight"] and emb["weight"].shape == (cfg.vocab_size, cfg.hidden_size)


def test_random_weights_deterministic():
    c = tiny()
    a = W.random_layer(c, 2, torch.float32, seed=1)
    b = W.random_layer(c, 2, torch.float32, seed=1)
    d = W.random_layer(c, 3, torch.float32, seed=1)
    assert all(torch.equal(a[k], b[k]) for k in a)
    assert not torch.equal(a["mlp.up_proj.weight"], d["mlp.up_proj.weight"])


def test_tokenizer(tiny_shards):
    tok = load_tokenizer(tiny_shards)
    assert isinstance(tok, SyntheticByteTokenizer)
    enc = tok("Write a poem about the blue sky.", return_tensors="pt")
    ids = enc["input_ids"]
    assert ids.shape[0] == 1 and ids[0, 0].item() == tok.bos_token_id
    assert tok.decode(ids[0], skip_special_tokens=True) == "Write a poem about the blue sky."
    assert tok.decode(tok.eos_token_id) == tok.eos_token


def test_rope_llama3_scaling():
    c = llama32_3b()
    inv = inv_freq(c)
    base = 1.0 / (c.rope_theta ** (torch.arange(0, 128, 2).float() / 128))
    # high-frequency dims unchanged, low-frequency dims divided by factor
    assert torch.allclose(inv[0], base[0])
    assert torch.allclose(inv[-1], base[-1] / 32.0)
    cos, sin = rope_table(tiny(), 16)
    assert cos.shape == (16, 32) and torch.allclose(cos[0], torch.ones(32))


def test_pack_roundtrip_and_layout():
    w = torch.randn(64, 96)
    wp = packing.pack_b(w)
    assert wp.shape == (4, 3, 64, 8)
    assert torch.equal(packing.unpack_b(wp), w)
    # fragment (nt=1, kt=2): lane 17 -> row 16+1, k = 64 + 8*1 .. +8
    assert torch.equal(wp[1, 2, 17], w[17, 72:80])


def test_rope_perm_pairs():
    hd = 128
    p = packing.rope_head_perm(hd)
    assert sorted(p) == list(range(hd))
    for c in range(hd):
        partner = p[c ^ 8]
        assert abs(p[c] - partner) == hd // 2


def test_gate_up_interleave():
    g = torch.arange(32 * 4).float().view(32, 4)
    u = -g
    gu = packing.fuse_gate_up(g, u)
    assert torch.equal(gu[:16], g[:16]) and torch.equal(gu[16:32], u[:16]) and torch.equal(gu[32:48], g[16:])


def _ref_from_folder(path, causal=True):
    cfg, emb, layers, fn, lm = W.load_full_model(path)
    return cfg, ReferenceLlama(cfg, emb, layers, fn, lm, causal=causal)


def _engine_generate(engines, prompt, n_new):
    """Greedy generation through a chain of CPU StageEngines (single sequence)."""
    first, last = engines[0], engines[-1]
    out = []
    ids = prompt
    for step in range(n_new):
        S = ids.numel()
        h = first.embed(ids)
        for e in engines:
            slot, pos = e.prefill_rows([0], [S])
            h = e.forward(h, slot, pos)
            e.advance([0], [S])
        tok = last.head(h, [S - 1])
        out.append(int(tok[0]))
        ids = tok
    return out


def test_cpu_engine_matches_golden(tiny_shards):
    cfg, ref = _ref_from_folder(tiny_shards)
    prompt = torch.tensor([[1, 50, 60, 70, 80, 90, 33]])
    want = ref.generate(prompt, 12)[0].tolist()
    src = ShardFolderSource(tiny_shards)
    eng = StageEngine(cfg, 0, cfg.num_hidden_layers, "cpu", torch.float32, has_embed=True, has_head=True,
                      source=src, max_seq=128)
    got = _engine_generate([eng], prompt[0], 12)
    assert got == want


def test_cpu_engine_two_stage_split_equals_single(tiny_shards):
    cfg, ref = _ref_from_folder(tiny_shards)
    prompt = torch.tensor([[1, 5, 9, 13, 200, 17]])
    want = ref.generate(prompt, 10)[0].tolist()
    src = ShardFolderSource(tiny_shards)
    a = StageEngine(cfg, 0, 2, "cpu", torch.float32, has_embed=True, source=src, max_seq=64)
    b = StageEngine(cfg, 2, cfg.num_hidden_layers, "cpu", torch.float32, has_head=True, source=src, max_seq=64)
    assert _engine_generate([a, b], prompt[0], 10) == want


def test_cpu_engine_noncausal_flag(tiny_shards):
    """Reference quirk Q1: unmasked prefill. kv_len override reproduces it."""
    cfg, ref = _ref_from_folder(tiny_shards, causal=False)
    prompt = torch.tensor([[1, 5, 9, 13, 200, 17]])
    tok_ref, _ = ref.step(prompt)
    eng = StageEngine(cfg, 0, cfg.num_hidden_layers, "cpu", torch.float32, has_embed=True, has_head=True,
                      source=ShardFolderSource(tiny_shards), max_seq=64)
    S = prompt.shape[1]
    slot, pos = eng.prefill_rows([0], [S])
    h = eng.forward(eng.embed(prompt[0]), slot, pos, kv_len=[S] * S)
    assert int(eng.head(h, [S - 1])[0]) == int(tok_ref[0])


def test_cpu_engine_batched_rows_multi_slot():
    """Two sequences of different lengths in one row batch == each run alone."""
    cfg = tiny()
    src = RandomSource(cfg, seed=9)
    eng = StageEngine(cfg, 0, cfg.num_hidden_layers, "cpu", torch.float32, has_embed=True, has_head=True,
                      source=src, max_slots=2, max_seq=64)
    p0 = torch.tensor([1, 4, 8, 15, 16])
    p1 = torch.tensor([1, 23, 42])
    slot, pos = eng.prefill_rows([0, 1], [5, 3])
    h = eng.forward(eng.embed(torch.cat([p0, p1])), slot, pos)
    eng.advance([0, 1], [5, 3])
    toks = eng.head(h, [4, 7]).tolist()
    solo = []
    for p in (p0, p1):
        e = StageEngine(cfg, 0, cfg.num_hidden_layers, "cpu", torch.float32, has_embed=True, has_head=True,
                        source=src, max_seq=64)
        sl, po = e.prefill_rows([0], [p.numel()])
        hh = e.forward(e.embed(p), sl, po)
        solo.append(int(e.head(hh, [p.numel() - 1])[0]))
    assert toks == solo
