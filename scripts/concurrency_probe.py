#!/usr/bin/env python3
"""Does replaying decode graphs of different micro-batches CONCURRENTLY (one HIP stream each,
separate scratch sets) raise one GPU's decode throughput over running them back to back?
Llama-2-7B random init, sequences pre-positioned at 128 tokens. Prints JSON lines."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.config import get_preset  # noqa: E402
from llm_sharding_amd.runtime.engine import DecodeGraph, RandomSource, StageEngine  # noqa: E402


def timed(fn, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    cfg = get_preset("llama2-7b")
    dev = torch.device("cuda", 0)
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    nstreams = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    eng = StageEngine(cfg, 0, cfg.num_hidden_layers, dev, torch.bfloat16, has_embed=True, has_head=True,
                      source=RandomSource(cfg, 0), max_slots=rows * nstreams, max_seq=512, max_prefill_rows=rows)
    for s in range(rows * nstreams):
        eng.seq_len[s] = 128
    gs = [DecodeGraph(eng, rows, "full", slots=list(range(k * rows, (k + 1) * rows)), scratch=k).capture()
          for k in range(nstreams)]
    mode = sys.argv[3] if len(sys.argv) > 3 else "pool"
    if mode == "prio":      # high-priority pool (a different set of HW queues)
        streams = [torch.cuda.Stream(dev, priority=-1) for _ in range(nstreams)]
    elif mode == "skip":    # every other pool stream
        streams = [torch.cuda.Stream(dev) for _ in range(2 * nstreams)][::2]
    else:
        streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    reps = 12
    one = timed(lambda: gs[0].replay(), reps)
    serial = timed(lambda: [g.replay() for g in gs], reps)

    def conc():
        cur = torch.cuda.current_stream(dev)
        for st in streams:
            st.wait_stream(cur)
        for g, st in zip(gs, streams):
            with torch.cuda.stream(st):
                g.replay()
        for st in streams:
            cur.wait_stream(st)
    concurrent = timed(conc, reps)
    print(json.dumps({"rows_per_graph": rows, "graphs": nstreams, "stream_mode": mode, "one_graph_ms": round(one, 3),
                      "serial_ms": round(serial, 3), "concurrent_ms": round(concurrent, 3),
                      "tok_s_one": round(rows / one * 1e3), "tok_s_serial": round(rows * nstreams / serial * 1e3),
                      "tok_s_concurrent": round(rows * nstreams / concurrent * 1e3)}), flush=True)


if __name__ == "__main__":
    main()
