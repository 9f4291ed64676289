#!/usr/bin/env python3
"""Single-GPU latency sweep (BASELINE.md §2 'report ... TTFT at prompt lengths 8...512,
matching the reference profiler sweep'): for each prompt length, batch-1 time-to-first-token
(embed -> all layers -> fused norm/lm_head/argmax, eager prefill path), plus batch-1 decode
TPOT through the hipGraph step, on random-init weights of a preset (default Llama-2-7B)."""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.config import get_preset  # noqa: E402
from llm_sharding_amd.runtime.engine import DecodeGraph, RandomSource, StageEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--lengths", default="8,16,32,64,128,256,512,1024,2048")
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--decode-steps", type=int, default=64)
    ap.add_argument("--decode-batches", default="1,4,16")
    a = ap.parse_args()
    cfg = get_preset(a.model)
    dev = torch.device("cuda", 0)
    lens = [int(x) for x in a.lengths.split(",")]
    t0 = time.perf_counter()
    eng = StageEngine(cfg, 0, cfg.num_hidden_layers, dev, torch.bfloat16, has_embed=True, has_head=True,
                      source=RandomSource(cfg, 0), max_slots=max(int(x) for x in a.decode_batches.split(",")),
                      max_seq=max(lens) + a.decode_steps + 8,
                      max_prefill_rows=max(lens))
    torch.cuda.synchronize()
    print(f"[sweep] {cfg.name} loaded in {time.perf_counter() - t0:.1f}s", flush=True)
    g = torch.Generator().manual_seed(0)
    res = {"model": cfg.name, "ttft_ms": {}, "tpot_ms": {}}
    for P in lens:
        ts = []
        for r in range(a.repeats + 1):
            ids = torch.randint(3, cfg.vocab_size, (P,), generator=g).to(dev)
            eng.reset() if hasattr(eng, "reset") else None
            eng.seq_len[0] = 0
            torch.cuda.synchronize()
            t = time.perf_counter()
            sl, po = eng.prefill_rows([0], [P])
            h = eng.forward(eng.embed(ids), sl, po)
            tok = eng.head(h, [P - 1])
            int(tok[0])
            ts.append((time.perf_counter() - t) * 1e3)
        res["ttft_ms"][P] = round(statistics.median(ts[1:]), 3)
        print(f"[sweep] prompt {P:5d}: ttft {res['ttft_ms'][P]:.2f} ms", flush=True)
    for B in [int(x) for x in a.decode_batches.split(",")]:
        for s in range(B):
            eng.seq_len[s] = 128
        dg = DecodeGraph(eng, B, "full", slots=list(range(B))).capture()
        for _ in range(4):
            dg.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.decode_steps):
            dg.replay()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.decode_steps
        res["tpot_ms"][B] = round(ms, 3)
        print(f"[sweep] decode batch {B:3d}: {ms:.3f} ms/token/step ({B / ms * 1e3:.0f} tok/s)", flush=True)
    wbytes = sum(p.numel() * p.element_size() for lw in eng.layers for p in (lw.qkv, lw.o, lw.gate_up, lw.down))
    wbytes += eng.lm_head.numel() * 2
    res["weight_GB"] = round(wbytes / 1e9, 2)
    res["b1_roofline_ms_at_6.3TBps"] = round(wbytes / 6.3e9, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
