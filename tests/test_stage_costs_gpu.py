"""Planner inputs measured on the DEPLOYED engine: the stage-cost profile
(hipGraph decode replays of StageEngine/DecodeGraph on 1 and n layers, hipEvents) prices a
4-stage Llama-2-7B plan, and every planned stage's own captured decode step - built exactly as
a pipeline rank builds it - measures within 15 % of the planner's predicted time.
Reference: c_k of /root/reference/utils/node_profiler.py:822-979 feeds the master scheduler
(/root/reference/README.md:7-8)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("batch", [1, 256])
def test_planner_predicts_deployed_stage_times(batch):
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_profiler import _measure_stage
    from llm_sharding_amd.config import get_preset
    from llm_sharding_amd.parallel.scheduler import DeviceSpec
    from llm_sharding_amd.runtime.engine import RandomSource
    from llm_sharding_amd.utils.master_node import MasterNode
    from llm_sharding_amd.utils.node_profiler import profile_stage_costs
    cfg = get_preset("llama2-7b")
    src = RandomSource(cfg, 3)
    prof = profile_stage_costs(cfg, src, "cuda", batch=batch, context=128, n_layers=3, prefill_len=256, replays=20)
    print(f"[stage-costs] batch {batch}: " + ", ".join(f"{k} {v:.4f}" for k, v in prof.items()
                                                       if isinstance(v, float)))
    m = MasterNode(cfg, [DeviceSpec() for _ in range(4)])
    plan = m.plan_from_profiles([prof] * 4, kv_tokens=batch * 512)
    for st in plan.stages:
        got = _measure_stage(cfg, src, st.start, st.end, st.has_embed, st.has_head, batch, 128, device="cuda",
                             dtype=torch.bfloat16, reps=20)
        print(f"[stage-costs] batch {batch} stage [{st.start},{st.end}) predicted {st.est_time:.3f} ms "
              f"measured {got:.3f} ms")
        assert abs(st.est_time - got) / got < 0.15, (st.start, st.end, st.est_time, got)
        torch.cuda.empty_cache()
