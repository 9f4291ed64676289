#!/usr/bin/env python3
"""Decode-attention bandwidth at the headline bench's shape (512 sequences x ~143 tokens of
context, Llama-2-7B heads) for loop variants of attn_split_kernel (probe knob
lsa_attn_set_variant) and split factors. Prints one JSON line per (variant, nsplit)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip  # noqa: E402

DEV = "cuda"


def main():
    rows_list = [int(r) for r in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["512"])]
    nh, nkv, hd, tmax = 32, 32, 128, 192
    L = hip.lib()
    L.lsa_attn_set_variant.argtypes = [ctypes.c_int]
    for rows, T in [(r, t) for r in rows_list for t in (143, 180)]:
        kcs = [torch.randn(rows, nkv, tmax, hd, device=DEV).to(torch.bfloat16) for _ in range(3)]
        vcs = [torch.randn_like(k) for k in kcs]
        q = torch.randn(rows, nh * hd, device=DEV).to(torch.bfloat16)
        slot = torch.arange(rows, dtype=torch.int32, device=DEV)
        pos = torch.full((rows,), T - 1, dtype=torch.int32, device=DEV)
        out = torch.zeros(rows, nh * hd, dtype=torch.bfloat16, device=DEV)
        po = torch.zeros(rows * nh * 4 * hd, device=DEV)
        pl = torch.zeros(rows * nh * 4, device=DEV)
        cnt = torch.zeros(rows * nkv, dtype=torch.int32, device=DEV)
        nbytes = rows * nkv * T * hd * 2 * 2
        ref = None
        for var in (0, 200, 201, 210, 211, 400, 410, 411, 800, 801, 810, 811):
            L.lsa_attn_set_variant(var)
            for ns in (1, 2, 4):
                def run(i):
                    hip.attn(q, kcs[i % 3], vcs[i % 3], slot, pos, rows, nh, nkv, hd, ns, po, pl, out, counters=cnt)
                run(0)
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                err = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
                for i in range(3):
                    run(i)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                n = 30
                s.record()
                for i in range(n):
                    run(i)
                e.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(e) * 1e3 / n
                print(json.dumps({"rows": rows, "T": T, "variant": var, "nsplit": ns, "us": round(us, 2),
                                  "TBps": round(nbytes / us / 1e6, 3), "relerr_vs_default": float(f"{err:.2e}")}),
                      flush=True)
        L.lsa_attn_set_variant(0)
        del kcs, vcs
        torch.cuda.empty_cache()
    # streaming-read reference: one pass over the same bytes (torch sum of a bf16 buffer)
    buf = torch.randn(512 * nkv * 143 * hd * 2, device=DEV).to(torch.bfloat16)
    for _ in range(3):
        buf.sum()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        buf.sum()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / 20
    print(json.dumps({"reference": "torch.sum bf16", "bytes": buf.numel() * 2, "us": round(us, 2),
                      "TBps": round(buf.numel() * 2 / us / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
