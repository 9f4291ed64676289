"""Timeline tracer: spans -> Chrome trace JSON, per-rank merge, env activation in the
server (CPU; the GPU path records hipEvents and is exercised by bench.py --trace)."""
import json
import os

import torch

from llm_sharding_amd.config import tiny
from llm_sharding_amd.parallel.server import PipelineServer
from llm_sharding_amd.runtime.engine import RandomSource
from llm_sharding_amd.utils.tracing import Timeline, merge_traces


def test_spans_export_and_merge(tmp_path):
    tls = []
    for r in range(2):
        tl = Timeline(rank=r, device="cpu")
        tl.start()
        for i in range(3):
            with tl.span("work", i=i):
                sum(range(10000))
        tls.append(tl.export(str(tmp_path / f"t{r}.json")))
    out = merge_traces(tls, str(tmp_path / "all.json"))
    evs = json.load(open(out))["traceEvents"]
    xs = [e for e in evs if e["ph"] == "X"]
    assert len(xs) == 6 and {e["pid"] for e in xs} == {0, 1}
    assert all(e["dur"] >= 0 and e["ts"] >= 0 for e in xs)
    s = Timeline(device="cpu")
    with s.span("a"):
        pass
    assert s.summary()["a"]["n"] == 1


def test_server_trace_from_env(tmp_path, monkeypatch):
    monkeypatch.setenv("LSA_TRACE", str(tmp_path))
    cfg = tiny(layers=2)
    srv = PipelineServer(cfg, RandomSource(cfg, 1), device="cpu", batch=2, microbatches=1, max_seq=64,
                         dtype=torch.float32)
    srv.generate([[1, 2, 3], [4, 5]], 3, eos_ids=())
    path = tmp_path / "trace_rank0.json"
    assert path.exists()
    names = {e["name"] for e in json.load(open(path))["traceEvents"] if e["ph"] == "X"}
    assert {"prefill", "decode"} <= names
