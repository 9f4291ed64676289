"""ModelSharder: HF checkpoint (sharded safetensors) -> reference shard format, round-trip
through the engine, FP8 shards, GPT-2 layout."""
import os

import pytest
import torch

from llm_sharding_amd.config import tiny
from llm_sharding_amd.models import weights as W
from llm_sharding_amd.models.reference import LAYER_KEYS, ReferenceLlama
from llm_sharding_amd.runtime.engine import ShardFolderSource, StageEngine
from llm_sharding_amd.utils.model_sharder import ModelSharder, write_hf_llama_checkpoint


@pytest.fixture(scope="module")
def hf_ckpt(tmp_path_factory):
    cfg = tiny()
    d = str(tmp_path_factory.mktemp("hf") / "tiny-hf")
    layers = [W.random_layer(cfg, i, torch.float32, seed=2) for i in range(cfg.num_hidden_layers)]
    write_hf_llama_checkpoint(cfg, d, W.random_embedding(cfg, torch.float32, seed=2), layers,
                              W.random_final_norm(cfg, torch.float32, seed=2), W.random_lm_head(cfg, torch.float32, seed=2))
    with open(os.path.join(d, "tokenizer_config.json"), "w") as f:
        f.write('{"tokenizer_class": "SyntheticByteTokenizer", "vocab_size": 512}')
    return cfg, d, layers


def test_sharder_llama_layout_and_values(hf_ckpt, tmp_path):
    cfg, d, layers = hf_ckpt
    out = ModelSharder(d, "llama", str(tmp_path / "tiny"), dtype=torch.bfloat16, verbose=False).save_shards()
    assert out.endswith("_bfloat16")
    files = set(os.listdir(out))
    assert {"config.json", "tokenizer_config.json", "embedding.pth", "final_norm.pth", "lm_head.pth"} <= files
    assert not any(f.endswith(".safetensors") for f in files)
    for i in range(cfg.num_hidden_layers):
        blk = torch.load(os.path.join(out, f"block_{i}.pth"), weights_only=True)
        assert set(blk) == set(LAYER_KEYS)
        assert torch.equal(blk["mlp.down_proj.weight"], layers[i]["mlp.down_proj.weight"].to(torch.bfloat16))
    # the shards run through the engine exactly like the golden model of the same weights
    c2, emb, lays, fn, lm = W.load_full_model(out)
    ref = ReferenceLlama(c2, emb, lays, fn, lm)
    prompt = torch.tensor([[1, 11, 22, 33]])
    want = ref.generate(prompt, 5)[0].tolist()
    eng = StageEngine(c2, 0, c2.num_hidden_layers, "cpu", torch.float32, has_embed=True, has_head=True,
                      source=ShardFolderSource(out), max_seq=64)
    ids, got = prompt[0], []
    for _ in range(5):
        sl, po = eng.prefill_rows([0], [ids.numel()])
        h = eng.forward(eng.embed(ids), sl, po)
        eng.advance([0], [ids.numel()])
        ids = eng.head(h, [ids.numel() - 1])
        got.append(int(ids[0]))
    assert got == want


@pytest.mark.skipif(not hasattr(torch, "float8_e4m3fn"), reason="no fp8 dtype")
def test_sharder_fp8(hf_ckpt, tmp_path):
    cfg, d, layers = hf_ckpt
    out = ModelSharder(d, "llama", str(tmp_path / "tiny"), dtype=torch.float8_e4m3fn, verbose=False).save_shards()
    raw = torch.load(os.path.join(out, "block_0.pth"), weights_only=True)
    assert raw["self_attn.q_proj.weight"].dtype == torch.float8_e4m3fn and "self_attn.q_proj.weight_scale" in raw
    blk = W.load_block(out, 0)
    w = layers[0]["self_attn.q_proj.weight"]
    rel = (blk["self_attn.q_proj.weight"].float() - w).norm() / w.norm()
    assert rel < 0.05


def test_sharder_gpt2_layout(tmp_path):
    from safetensors.torch import save_file
    d = tmp_path / "gpt2"
    d.mkdir()
    t = {"wte.weight": torch.randn(50, 16), "wpe.weight": torch.randn(32, 16), "ln_f.weight": torch.ones(16),
         "ln_f.bias": torch.zeros(16)}
    for i in range(2):
        t[f"h.{i}.attn.c_attn.weight"] = torch.randn(16, 48)
        t[f"h.{i}.ln_1.weight"] = torch.ones(16)
    save_file(t, str(d / "model.safetensors"))
    (d / "config.json").write_text('{"model_type": "gpt2"}')
    out = ModelSharder(str(d), "gpt", str(tmp_path / "g"), dtype=torch.float16, verbose=False).save_shards()
    emb = torch.load(os.path.join(out, "embedding.pth"), weights_only=True)
    assert set(emb) == {"wte", "wpe", "drop"} and emb["wte"]["weight"].dtype == torch.float16
    assert set(torch.load(os.path.join(out, "block_1.pth"), weights_only=True)) == {"attn.c_attn.weight", "ln_1.weight"}
    assert set(torch.load(os.path.join(out, "ln_f.pth"), weights_only=True)) == {"weight", "bias"}
    assert torch.equal(torch.load(os.path.join(out, "lm_head.pth"), weights_only=True)["weight"], t["wte.weight"].half())


@pytest.mark.parametrize("dtype,tol", [(torch.int8, 0.01), (getattr(torch, "int4", None), 0.12)])
def test_sharder_int8_int4(hf_ckpt, tmp_path, dtype, tol):
    """The reference's int8 / int4 sharding options (bitsandbytes there): self-contained
    symmetric quantisation here, loaded back as bf16 by the engine."""
    if dtype is None:
        pytest.skip("no torch.int4")
    cfg, d, layers = hf_ckpt
    out = ModelSharder(d, "llama", str(tmp_path / "tiny"), dtype=dtype, verbose=False).save_shards()
    assert out.endswith("_" + str(dtype).split(".")[-1])
    raw = torch.load(os.path.join(out, "block_0.pth"), weights_only=True)
    q, s = raw["mlp.down_proj.weight"], raw["mlp.down_proj.weight_scale"]
    w = layers[0]["mlp.down_proj.weight"]
    if dtype == torch.int8:
        assert q.dtype == torch.int8 and q.shape == w.shape and s.shape == (w.shape[0],)
    else:
        assert q.dtype == torch.uint8 and q.shape == (w.shape[0], w.shape[1] // 2) and s.dim() == 2
    assert raw["input_layernorm.weight"].dtype == torch.bfloat16
    blk = W.load_block(out, 0)
    for k in ("self_attn.q_proj.weight", "mlp.down_proj.weight"):
        ref = layers[0][k]
        assert blk[k].dtype == torch.bfloat16 and blk[k].shape == ref.shape
        assert (blk[k].float() - ref).norm() / ref.norm() < tol
    # the engine on the quantised shards == the golden model on the same (dequantised) weights
    c2, emb, lays, fn, lm = W.load_full_model(out)
    prompt = torch.tensor([[1, 11, 22, 33]])
    want = ReferenceLlama(c2, emb, lays, fn, lm).generate(prompt, 4)[0].tolist()
    eng = StageEngine(c2, 0, c2.num_hidden_layers, "cpu", torch.float32, has_embed=True, has_head=True,
                      source=ShardFolderSource(out), max_seq=64)
    ids, got = prompt[0], []
    for _ in range(4):
        sl, po = eng.prefill_rows([0], [ids.numel()])
        h = eng.forward(eng.embed(ids), sl, po)
        eng.advance([0], [ids.numel()])
        ids = eng.head(h, [ids.numel() - 1])
        got.append(int(ids[0]))
    assert got == want


def test_int4_pack_roundtrip():
    from llm_sharding_amd.utils.model_sharder import dequantize_int4, quantize_int4
    w = torch.randn(8, 256)
    q, s = quantize_int4(w)
    assert q.shape == (8, 128) and s.shape == (8, 2)
    # on-grid values come back exactly
    grid = (torch.randint(-7, 8, (8, 256)).float() * s.repeat_interleave(128, dim=1))
    q2, s2 = quantize_int4(grid)
    assert torch.allclose(dequantize_int4(q2, s2), grid, atol=1e-6)
    # narrow K: group = gcd(K, 128)
    q3, s3 = quantize_int4(torch.randn(4, 96))
    assert s3.shape == (4, 3)
