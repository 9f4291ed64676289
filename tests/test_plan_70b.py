"""Stage memory at the bench defaults: the scheduler's plan for Llama-2-70B
on eight MI355X stages fits 288 GB per GPU with weights, the static KV cache of every
micro-batch AND the engine's scratch counted, and the memory model the plan uses
(:func:`stage_memory` / :func:`scratch_bytes`) is the one the engine actually allocates -
exactly on CPU for weights + KV, and against torch's allocator on an MI355X for a
70B-shaped stage (``test_stage_memory_model_on_gpu``)."""
import pytest
import torch

from llm_sharding_amd.config import get_preset
from llm_sharding_amd.parallel.scheduler import DeviceSpec, plan_stages, scratch_bytes, stage_memory

HBM = 288e9


def _bench_geometry(pp, steps=64, warmup=8, batch=512, prompt_len=128, lat=32, lat_warm=4):
    """What run_decode_benchmark sizes for its defaults (pipeline.py)."""
    need = prompt_len + max(warmup + steps, lat_warm + lat) + 1
    return batch, pp, -(-need // 64) * 64, prompt_len


def _stage_tables(model, pp, **kw):
    cfg = get_preset(model)
    B, M, max_seq, P = _bench_geometry(pp, **kw)
    plan = plan_stages(cfg, pp, kv_tokens=max_seq * B * M, head_split=pp > 1,
                       scratch=scratch_bytes(cfg, B * P, 1, max_seq))
    V = cfg.head_rows
    v1 = (V // 2) // 128 * 128 if pp > 1 else V
    out = []
    for st in plan.stages:
        hr = (v1 if st.has_head else 0) + (V - v1 if (pp > 1 and st.has_embed) else 0)
        out.append((st, stage_memory(cfg, st.n_layers, slots=B * M, max_seq=max_seq, prefill_rows=B * P,
                                     has_embed=st.has_embed, head_rows=hr, io_rows=B * M)))
    return cfg, plan, out


@pytest.mark.parametrize("steps,warmup", [(64, 8), (20, 5)])  # bench defaults, driver's call
def test_llama2_70b_eight_stage_plan_fits(steps, warmup):
    cfg, plan, tables = _stage_tables("llama2-70b", 8, steps=steps, warmup=warmup)
    assert [st.n_layers for st in plan.stages] == [10] * 8
    assert plan.stages[0].has_embed and plan.stages[-1].has_head
    for st, m in tables:
        assert m["total"] <= HBM - DeviceSpec().reserve_bytes, (st.index, m)
        # 10 layers x 1.71 GB of bf16 weights; KV for 8 micro-batches x 512 sequences
        assert 17.0e9 < m["weights"] < 18.5e9
        assert m["kv"] == 10 * cfg.kv_bytes_per_token_per_layer() * 512 * 8 * _bench_geometry(8, steps, warmup)[2]
    # the whole 70B model (138 GB of weights) does NOT fit one GPU next to the KV cache of the
    # same 4096 sequences, which is why the plan needs several stages
    with pytest.raises(ValueError):
        plan_stages(cfg, 1, kv_tokens=256 * 512 * 8, scratch=scratch_bytes(cfg, 512 * 128))


def test_llama2_7b_stage_tables_fit():
    for pp in (1, 2, 4, 8):
        _, plan, tables = _stage_tables("llama2-7b", pp)
        assert sum(st.n_layers for st in plan.stages) == 32
        assert all(m["total"] < HBM - 8e9 for _, m in tables)


def test_plan_counts_scratch_against_memory():
    cfg = get_preset("llama2-70b")
    dev = [DeviceSpec(mem_bytes=60e9, reserve_bytes=0) for _ in range(8)]
    plan_stages(cfg, dev, kv_tokens=0)                     # 17 GB weights per stage: fits
    with pytest.raises(ValueError):                        # + 45 GB of scratch: does not
        plan_stages(cfg, dev, kv_tokens=0, scratch=45e9)


def test_stage_memory_matches_cpu_engine():
    """Weights + KV of the model are the engine's own tensors (CPU engine: no scratch)."""
    from llm_sharding_amd.runtime.engine import RandomSource, StageEngine
    cfg = get_preset("tiny")
    eng = StageEngine(cfg, 0, 2, "cpu", torch.bfloat16, has_embed=True, has_head=True,
                      source=RandomSource(cfg, 0), max_slots=6, max_seq=64)
    m = stage_memory(cfg, 2, slots=6, max_seq=64, prefill_rows=0, has_embed=True, head_rows=cfg.head_rows)
    assert eng.memory_bytes() == m["weights"] + m["kv"]


@pytest.mark.gpu
def test_stage_memory_model_on_gpu():
    """A 70B-shaped stage (two Llama-2-70B layers, split-head part, 8 x 64 sequences of 256
    tokens, 8192-row prefill) on an MI355X: the model's prediction within 2% of what torch's
    allocator holds for the engine, and its 1.1 prefill + decode run inside that."""
    from llm_sharding_amd.parallel.pipeline import PipelineStage
    from llm_sharding_amd.runtime.engine import RandomSource
    cfg = get_preset("llama2-70b")
    dev = torch.device("cuda", 0)
    torch.cuda.empty_cache()
    base = torch.cuda.memory_allocated(dev)
    B, M, S, P = 64, 8, 256, 128
    stage = PipelineStage(cfg, 0, 1, 0, 2, dev, B, M, S, RandomSource(cfg, 0), use_graph=False,
                          max_prefill_rows=B * P)
    torch.cuda.synchronize()
    held = torch.cuda.memory_allocated(dev) - base
    m = stage_memory(cfg, 2, slots=B * M, max_seq=S, prefill_rows=B * P, has_embed=True,
                     head_rows=cfg.head_rows, io_rows=B * M)
    assert abs(held - m["total"]) <= 0.02 * m["total"], (held / 1e9, {k: v / 1e9 for k, v in m.items()})
    del stage
    torch.cuda.empty_cache()
