"""Per-rank execution timelines (the reference has no tracer - only
``perf_counter`` around ``cuda.synchronize``, ``/root/reference/utils/node_profiler.py:300-308``).

:class:`Timeline` records named spans. On a GPU each span is bracketed by two
``torch.cuda.Event``s on the current stream, so the recorded interval is the DEVICE execution
window of the work enqueued inside the span (no host synchronisation while tracing); the host
enqueue time is recorded as well. On CPU spans are host ``perf_counter`` intervals.
:meth:`Timeline.export` writes Chrome trace-event JSON (open in chrome://tracing or
Perfetto): one process per rank, a "gpu" and a "host" thread. :func:`merge_traces` combines
the per-rank files of a multi-GPU run into one timeline (ranks are aligned on a
barrier-synchronised reference event, see :meth:`Timeline.start`).

    tl = Timeline(rank, enabled=True)
    tl.start()                     # after a barrier on every rank
    with tl.span("decode", mb=0):  # enqueue GPU work
        graph.replay()
    tl.export("trace_rank0.json")
"""
from __future__ import annotations

import json
import os
import statistics
import time
from contextlib import contextmanager
from typing import Dict, List, Optional

import torch


class Timeline:
    def __init__(self, rank: int = 0, enabled: bool = True, device=None, max_spans: int = 1_000_000):
        self.rank = rank
        self.enabled = enabled
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.gpu = self.device.type == "cuda"
        self.max_spans = max_spans
        self.spans: List[tuple] = []  # (name, args, host_t0, host_t1, ev0, ev1)
        self._ref_ev = None
        self._ref_host = None

    def start(self) -> None:
        """Reference point of this rank's timeline (call right after a cross-rank barrier)."""
        if not self.enabled:
            return
        self._ref_host = time.perf_counter()
        if self.gpu:
            self._ref_ev = torch.cuda.Event(enable_timing=True)
            self._ref_ev.record()

    @contextmanager
    def span(self, name: str, **args):
        if not self.enabled or len(self.spans) >= self.max_spans:
            yield
            return
        if self._ref_host is None:
            self.start()
        e0 = e1 = None
        if self.gpu:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        h0 = time.perf_counter()
        try:
            yield
        finally:
            h1 = time.perf_counter()
            if self.gpu:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
            self.spans.append((name, args, h0, h1, e0, e1))

    def events(self) -> List[dict]:
        """Chrome trace events (microseconds, relative to :meth:`start`). Synchronises."""
        if self.gpu:
            torch.cuda.synchronize(self.device)
        out = []
        pid = self.rank
        for name, args, h0, h1, e0, e1 in self.spans:
            out.append({"name": name, "ph": "X", "pid": pid, "tid": "host", "ts": (h0 - self._ref_host) * 1e6,
                        "dur": (h1 - h0) * 1e6, "args": args})
            if e0 is not None:
                t0 = self._ref_ev.elapsed_time(e0) * 1e3
                t1 = self._ref_ev.elapsed_time(e1) * 1e3
                out.append({"name": name, "ph": "X", "pid": pid, "tid": "gpu", "ts": t0, "dur": max(0.0, t1 - t0),
                            "args": args})
        out.append({"name": "process_name", "ph": "M", "pid": pid, "args": {"name": f"rank {pid}"}})
        return out

    def export(self, path: str) -> str:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump({"traceEvents": self.events(), "displayTimeUnit": "ms"}, f)
        return path

    def summary(self, thread: Optional[str] = None) -> Dict[str, dict]:
        """Per span name: count, mean / p50 / max duration (us) on the GPU thread if traced
        there, else on the host."""
        thread = thread or ("gpu" if self.gpu else "host")
        by: Dict[str, list] = {}
        for ev in self.events():
            if ev.get("ph") == "X" and ev["tid"] == thread:
                by.setdefault(ev["name"], []).append(ev["dur"])
        return {k: {"n": len(v), "mean_us": statistics.mean(v), "p50_us": statistics.median(v), "max_us": max(v)}
                for k, v in by.items()}


class _NullTimeline(Timeline):
    def __init__(self):
        super().__init__(enabled=False, device="cpu")


NULL = _NullTimeline()


def from_env(rank: int = 0, device=None) -> Timeline:
    """A live timeline if ``LSA_TRACE`` (an output directory) is set, else a no-op one."""
    return Timeline(rank, enabled=True, device=device) if os.environ.get("LSA_TRACE") else NULL


def export_env(tl: Timeline) -> Optional[str]:
    d = os.environ.get("LSA_TRACE")
    if not d or not tl.enabled:
        return None
    return tl.export(os.path.join(d, f"trace_rank{tl.rank}.json"))


def merge_traces(paths: List[str], out: str) -> str:
    evs = []
    for p in paths:
        with open(p) as f:
            evs += json.load(f)["traceEvents"]
    with open(out, "w") as f:
        json.dump({"traceEvents": evs, "displayTimeUnit": "ms"}, f)
    return out


__all__ = ["Timeline", "NULL", "from_env", "export_env", "merge_traces"]
