#!/usr/bin/env python3
"""Batch-1..16 decode attention (Llama-2-7B heads, 32 x 128, MHA) at short / mid contexts: the
split-KV kernel's split count and minimum chunk swept, hipGraph-timed (20 launches per graph),
to set StageEngine.decode_nsplit for latency-bound decode. One JSON line per (rows, T).

usage: attn_b1_probe.py [rows,rows,...] [T,T,...] [t_max]   (defaults 1,4,16  150,600,2048  4096)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip  # noqa: E402
from scripts.bench_kernels import timeit  # noqa: E402

DEV = "cuda"
hip.lib()
nh = nkv = 32
hd = 128
ROWS = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 4, 16]
TS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [150, 600, 2048]
TMAX = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
for rows in ROWS:
    for T in TS:
        tmax = TMAX
        kc = torch.randn(rows, nkv, tmax, hd, device=DEV).to(torch.bfloat16)
        vc = torch.randn_like(kc)
        q = torch.randn(rows, nh * hd, device=DEV).to(torch.bfloat16)
        slot = torch.arange(rows, dtype=torch.int32, device=DEV)
        pos = torch.full((rows,), T - 1, dtype=torch.int32, device=DEV)
        out = torch.zeros(rows, nh * hd, dtype=torch.bfloat16, device=DEV)
        po = torch.zeros(rows * nh * 16 * hd, device=DEV)
        pl = torch.zeros(rows * nh * 16, device=DEV)
        cnt = torch.zeros(rows * nkv, dtype=torch.int32, device=DEV)
        ref = None
        res = []
        for ns in (1, 2, 4, 8, 16):
            for mc in (16, 32, 64, 128):
                if ns == 1 and mc != 64:
                    continue
                us = timeit(lambda i: hip.attn(q, kc, vc, slot, pos, rows, nh, nkv, hd, ns, po, pl, out, min_chunk=mc,
                                               counters=cnt))
                if ref is None:
                    ref = out.clone()
                err = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
                res.append((round(us, 2), ns, mc, round(err, 6)))
        res.sort()
        print(json.dumps({"rows": rows, "T": T, "best": res[0], "all(us,nsplit,min_chunk,relerr)": res}), flush=True)
