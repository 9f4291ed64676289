#!/usr/bin/env python3
"""Batch-1 decode projections streaming from HBM vs from the Infinity Cache (VERDICT r3 item 4:
"the tail workgroups of each projection prefetch the first panels of the next projection's
weights into the Infinity Cache").

Per 7B projection at 1 row, the engine's tuned GEMV:
  cold    weights rotated over > 600 MB of copies (every launch streams from HBM)
  warm    the same copy every launch (< 256 MB: served by the Infinity Cache)
  pf      chain "short kernel (4 us, attention-sized) -> GEMV", with lsa_mall_prefetch of the
          GEMV's weights on a side stream forked at the short kernel: does the prefetch overlap
          the short kernel and speed up the GEMV that follows?
One JSON line per projection. usage: mall_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import MODEL_SHAPES  # noqa: E402


def graph_time(body, reps=10, replays=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(0)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(reps):
            body(i)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(replays):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (reps * replays) * 1e3


def main():
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    spin_src = torch.randn(1 << 20, device="cuda").to(torch.bfloat16)  # 2 MB: a ~4 us stand-in kernel
    spin_dst = torch.empty(1 << 20, device="cuda", dtype=torch.float32)
    side = torch.cuda.Stream()
    for name, (N, K) in MODEL_SHAPES["llama2-7b"].items():
        if name == "lm_head":
            continue
        nbuf = max(2, (640 << 20) // (N * K * 2) + 1)
        wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        x = torch.randn(1, K, device="cuda").to(torch.bfloat16)
        out = torch.empty(1, N, dtype=torch.bfloat16, device="cuda")
        ep = hip.make_epi(out=out, ldo=N)

        def gemv(i):
            hip.gemv(x, wps[i % nbuf], 1, N, K, hip.EPI_STORE, ep)

        def short(_):
            torch.mul(spin_src, 1.0, out=spin_dst)

        t_cold = graph_time(gemv)
        t_warm = graph_time(lambda i: gemv(0))
        t_short = graph_time(short)
        t_chain = graph_time(lambda i: (short(i), gemv(i)))

        def chain_pf(i):
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                hip.mall_prefetch(wps[i % nbuf], sink)
            short(i)
            gemv(i)
            cur.wait_stream(side)

        t_pf = graph_time(chain_pf)
        t_pf_only = graph_time(lambda i: hip.mall_prefetch(wps[i % nbuf], sink))
        mb = N * K * 2 / 1e6
        print(json.dumps({"proj": name, "N": N, "K": K, "MB": round(mb, 1), "cold_us": round(t_cold, 2),
                          "cold_TBps": round(mb / t_cold, 2), "warm_us": round(t_warm, 2),
                          "warm_TBps": round(mb / t_warm, 2), "short_us": round(t_short, 2),
                          "chain_us": round(t_chain, 2), "chain_prefetch_us": round(t_pf, 2),
                          "prefetch_alone_us": round(t_pf_only, 2)}), flush=True)
        del wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
