"""GPT-2 family on the CPU path (the reference shards GPT-2 but cannot load or
run it, so parity is pinned against transformers' GPT2LMHeadModel instead).

HF checkpoint (random init, non-trivial biases / LayerNorm affine) -> our ModelSharder
(model_type "gpt") -> reference-format shard folder -> StageEngine(s) with a KV cache, greedy
decode -> must equal HF's greedy decode by full recompute, in fp32."""
import pytest
import torch

from llm_sharding_amd.config import LlamaConfig, tiny_gpt2
from llm_sharding_amd.models import gpt2 as G2
from llm_sharding_amd.runtime.engine import RandomSource, ShardFolderSource, StageEngine
from llm_sharding_amd.utils.model_sharder import ModelSharder

transformers = pytest.importorskip("transformers")

NEW = 12


def _hf_model(tmp_path):
    from transformers import GPT2Config, GPT2LMHeadModel
    torch.manual_seed(0)
    c = GPT2Config(n_embd=128, n_layer=3, n_head=4, n_positions=128, vocab_size=300, bos_token_id=299,
                   eos_token_id=299, resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)
    m = GPT2LMHeadModel(c).eval()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("bias") or ".ln_" in n:
                p.add_(torch.randn_like(p) * 0.1)
            elif "h." in n and p.dim() == 2:
                p.mul_(10.0)  # layers that matter + well-separated greedy decisions
        m.transformer.wte.weight.mul_(5.0)
    d = tmp_path / "hf_gpt2"
    m.save_pretrained(str(d))
    return m, str(d)


def _engine_generate(cfg, src, prompt, n_new, cuts=None):
    """Greedy decode through StageEngines covering [0, L) split at ``cuts`` (CPU, fp32)."""
    L = cfg.num_hidden_layers
    bounds = [0] + list(cuts or []) + [L]
    engs = [StageEngine(cfg, a, b, "cpu", torch.float32, has_embed=(a == 0), has_head=(b == L), source=src,
                        max_slots=1, max_seq=64) for a, b in zip(bounds, bounds[1:])]
    ids = torch.tensor(prompt)
    out = []
    h = engs[0].embed(ids)
    for step in range(n_new):
        n = h.shape[0]
        for e in engs:
            slot, pos = e.prefill_rows([0], [n])
            h = e.forward(h, slot, pos)
            e.advance([0], [n])
        t = int(engs[-1].head(h, [n - 1])[0])
        out.append(t)
        h = engs[0].embed(torch.tensor([t]))
    return out


@pytest.fixture(scope="module")
def hf(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("gpt2")
    m, d = _hf_model(tmp)
    shards = ModelSharder(d, "gpt", str(tmp / "shards"), dtype=torch.float32, verbose=False).save_shards()
    return m, shards


def _hf_greedy(m, prompt, n_new):
    ids = list(prompt)
    out = []
    with torch.no_grad():
        for _ in range(n_new):
            t = int(m(torch.tensor([ids])).logits[0, -1].argmax())
            out.append(t)
            ids.append(t)
    return out


def test_config_maps_hf_keys(hf):
    _, shards = hf
    cfg = LlamaConfig.from_pretrained(shards)
    assert cfg.is_gpt2 and cfg.hidden_size == 128 and cfg.num_hidden_layers == 3 and cfg.head_dim == 32
    assert cfg.intermediate_size == 512 and cfg.vocab_size == 300 and cfg.head_rows == 384


def test_shard_format_matches_reference_layout(hf):
    _, shards = hf
    emb = torch.load(f"{shards}/embedding.pth", weights_only=True)
    assert set(emb) == {"wte", "wpe", "drop"} and emb["drop"] == {}
    assert set(torch.load(f"{shards}/block_0.pth", weights_only=True)) >= set(G2.GPT2_LAYER_KEYS)
    assert set(torch.load(f"{shards}/ln_f.pth", weights_only=True)) == {"weight", "bias"}


@pytest.mark.parametrize("cuts", [None, [1], [1, 2]])
def test_engine_matches_hf_greedy(hf, cuts):
    m, shards = hf
    cfg = LlamaConfig.from_pretrained(shards)
    prompt = [5, 17, 250, 3, 99, 42, 7]
    ref = _hf_greedy(m, prompt, NEW)
    assert len(set(ref)) > 2
    assert _engine_generate(cfg, ShardFolderSource(shards, cfg), prompt, NEW, cuts) == ref


def test_golden_forward_matches_hf(hf):
    m, shards = hf
    cfg = LlamaConfig.from_pretrained(shards)
    wte, wpe = G2.load_embedding(shards)
    layers = [G2.load_block(shards, i) for i in range(cfg.num_hidden_layers)]
    ids = torch.tensor([1, 2, 3, 250, 7])
    ours = G2.forward_full(cfg, wte, wpe, layers, G2.load_ln_f(shards), ids)
    with torch.no_grad():
        theirs = m(ids[None]).logits[0]
    torch.testing.assert_close(ours, theirs, rtol=1e-4, atol=1e-4)


def test_random_source_matches_written_shards(tmp_path):
    cfg = tiny_gpt2(layers=2, hidden=64, heads=2, vocab=100)
    folder = G2.write_random_shards(cfg, str(tmp_path / "g"), dtype=torch.float32, seed=3)
    prompt = [4, 8, 15, 16]
    a = _engine_generate(cfg, RandomSource(cfg, seed=3), prompt, 6)
    b = _engine_generate(LlamaConfig.from_pretrained(folder), ShardFolderSource(folder), prompt, 6)
    assert a == b
