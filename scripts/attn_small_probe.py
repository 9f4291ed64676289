#!/usr/bin/env python3
"""Batch-1 decode attention (Llama-2-7B heads, 32 x 128, MHA, one split: the 8-wave small-grid
kernel, or the 4-wave split kernel with LSA_ATTN_SMALL_MAX_WGS=0) against the context length T,
hipGraph-timed back to back (each launch depends on the previous: the per-launch time includes
the kernel boundary, as inside a decode step), with a one-row embedding gather as the
trivial-kernel floor. One JSON line per T."""
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
tmax = 1024
kc = torch.randn(4, nkv, tmax, hd, device=DEV).to(torch.bfloat16)
vc = torch.randn_like(kc)
q = torch.randn(1, nh * hd, device=DEV).to(torch.bfloat16)
slot = torch.zeros(1, dtype=torch.int32, device=DEV)
out = torch.zeros(1, nh * hd, dtype=torch.bfloat16, device=DEV)
po = torch.zeros(nh * 16 * hd, device=DEV)
pl = torch.zeros(nh * 16, device=DEV)
cnt = torch.zeros(nkv, dtype=torch.int32, device=DEV)
ids = torch.zeros(1, dtype=torch.int32, device=DEV)
table = torch.randn(16, 4096, device=DEV).to(torch.bfloat16)
eo = torch.zeros(1, 4096, dtype=torch.bfloat16, device=DEV)
floor = timeit(lambda i: hip.embed(ids, table, eo))
print(json.dumps({"kernel": "embed 1 row (floor)", "us": round(floor, 2)}), flush=True)
for T in (1, 16, 64, 150, 256, 512):
    pos = torch.full((1,), T - 1, dtype=torch.int32, device=DEV)
    us = timeit(lambda i: hip.attn(q, kc, vc, slot, pos, 1, nh, nkv, hd, 1, po, pl, out, counters=cnt))
    kv_mb = T * nkv * hd * 2 * 2 / 1e6
    print(json.dumps({"T": T, "us": round(us, 2), "over_floor_us": round(us - floor, 2), "kv_MB": round(kv_mb, 2),
                      "small_max_wgs": os.environ.get("LSA_ATTN_SMALL_MAX_WGS", "default")}), flush=True)
