"""Property-based tests (hypothesis), CPU: the scheduler's exact min-max partition against a
brute-force search over every cut, and the in-memory wire protocol round-trip (SURVEY.md §4:
'sweeping shapes with hypothesis')."""
import itertools

import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from llm_sharding_amd.config import tiny
from llm_sharding_amd.parallel import protocol
from llm_sharding_amd.parallel.scheduler import DeviceSpec, plan_stages


def _brute(costs, speeds, head, embed):
    L, n = len(costs), len(speeds)
    best = float("inf")
    for cuts in itertools.combinations(range(1, L), n - 1):
        b = (0,) + cuts + (L,)
        worst = 0.0
        for k in range(n):
            t = sum(costs[b[k]:b[k + 1]]) + (embed if k == 0 else 0.0) + (head if k == n - 1 else 0.0)
            worst = max(worst, t * speeds[k])
        best = min(best, worst)
    return best


@settings(max_examples=60, deadline=None)
@given(L=st.integers(2, 9), data=st.data())
def test_plan_is_optimal(L, data):
    n = data.draw(st.integers(1, min(L, 4)))
    costs = data.draw(st.lists(st.floats(0.1, 5.0), min_size=L, max_size=L))
    speeds = data.draw(st.lists(st.floats(0.5, 3.0), min_size=n, max_size=n))
    head = data.draw(st.floats(0.0, 3.0))
    cfg = tiny(layers=L)
    devs = [DeviceSpec(speed=s) for s in speeds]
    plan = plan_stages(cfg, devs, layer_costs=costs, head_cost=head, embed_cost=0.0)
    assert [s.start for s in plan.stages][0] == 0 and plan.stages[-1].end == L
    assert all(s.end > s.start for s in plan.stages)
    assert abs(plan.bottleneck - _brute(costs, speeds, head, 0.0)) < 1e-6 * max(1.0, plan.bottleneck)


@settings(max_examples=60, deadline=None)
@given(shape=st.lists(st.integers(0, 5), min_size=0, max_size=4),
       dtype=st.sampled_from([torch.float32, torch.bfloat16, torch.float16, torch.int64, torch.int32]),
       extra=st.dictionaries(st.text(min_size=1, max_size=8), st.one_of(st.integers(-2**40, 2**40), st.text(max_size=10),
                                                                      st.booleans(), st.none()), max_size=4))
def test_protocol_roundtrip(shape, dtype, extra):
    t = (torch.randn(shape) * 100).to(dtype)
    msg = {"hidden_states": t, "meta": extra, "list": [t.clone(), 3, "x"], "nested": {"k": (1, 2)}}
    out = protocol.decode(protocol.encode(msg))
    assert torch.equal(out["hidden_states"], t) and out["hidden_states"].dtype == t.dtype
    assert out["meta"] == extra and out["list"][1:] == [3, "x"] and torch.equal(out["list"][0], t)
    assert tuple(out["nested"]["k"]) == (1, 2)
