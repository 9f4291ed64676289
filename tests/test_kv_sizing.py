"""KV cache sizing from device memory (the static cache is sized from the
288 GB of HBM per MI355X, not a fixed guess)."""
import pytest

from llm_sharding_amd.config import get_preset
from llm_sharding_amd.parallel.scheduler import kv_slots_for_memory, plan_stages


def test_llama2_7b_one_gpu_fills_hbm_up_to_graph_cap():
    cfg = get_preset("llama2-7b")
    plan = plan_stages(cfg, 1)
    st = plan.stages[0]
    # 32 layers x 2 x 4096 x 2 B = 512 KiB per token; 4096 tokens -> 2 GiB per slot
    n = kv_slots_for_memory(cfg, st.n_layers, 4096, 288e9, st.weight_bytes, max_per_microbatch=10_000)
    per_slot = 32 * 2 * 4096 * 2 * 4096
    assert n == int((288e9 - 8e9 - st.weight_bytes) // per_slot)
    assert 100 < n < 128
    assert kv_slots_for_memory(cfg, st.n_layers, 1024, 288e9, st.weight_bytes) == 128  # graph cap


def test_70b_pipeline_stage_and_microbatches():
    cfg = get_preset("llama2-70b")
    plan = plan_stages(cfg, 8, head_split=True)
    worst = min(kv_slots_for_memory(cfg, s.n_layers, 8192, 288e9, s.weight_bytes, microbatches=8,
                                    max_per_microbatch=10_000) for s in plan.stages)
    # GQA 8:1 -> 4 KiB per token per layer; 10 layers x 8192 tokens = 320 MiB per slot
    assert 60 < worst < 120


def test_too_small_device_raises():
    cfg = get_preset("llama2-70b")
    plan = plan_stages(cfg, 1)
    with pytest.raises(ValueError):
        kv_slots_for_memory(cfg, 80, 4096, 100e9, plan.stages[0].weight_bytes)
