"""Split-K over the library GEMM for the under-filled N=4096 decode projections.

At 512 decode rows Llama-2-7B's o_proj (K=4096) and down_proj (K=11008) are 512 x 4096 outputs:
a 256x256 macro-tile grid is 32 tiles for 256 CUs, so hipBLASLt runs them at 0.6-0.8 PFLOP/s
(profiles/r1_tunableop_decode_gemms.txt). Splitting K into s slices as ONE strided-batched GEMM
(torch.bmm over [s, M, K/s] x [s, K/s, N] views, no copies) gives s x the tiles; the s partials
are then reduced into the residual. Prints one JSON line per (op, s): graph-timed us per call,
weights rotated through enough copies to exceed the 256 MiB MALL.

    python scripts/splitk_lib_probe.py [--rows 512]
"""
from __future__ import annotations

import argparse
import json

import torch


def timed(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g, stream=s):
        for _ in range(iters):
            fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=512)
    args = ap.parse_args()
    dev = "cuda:0"
    M, N = args.rows, 4096
    torch.manual_seed(0)
    for name, K in (("o", 4096), ("down", 11008)):
        ncopy = max(2, int(1.2 * 2 ** 30 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        h0 = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        ref = h0.float() + a.float() @ ws[0].float().t()
        h = h0.clone()
        it = [0]

        def base():
            w = ws[it[0] % ncopy]
            it[0] += 1
            h.addmm_(a, w.t())

        us = timed(base)
        h.copy_(h0)
        h.addmm_(a, ws[0].t())
        err = ((h.float() - ref).abs().max() / ref.abs().max()).item()
        flop = 2 * M * N * K
        print(json.dumps({"op": name, "M": M, "N": N, "K": K, "split": 1, "us": round(us, 2),
                          "tflops": round(flop / us / 1e6, 1), "rel_err": err}), flush=True)
        for sk in (2, 4, 8):
            if K % sk:
                continue
            ks = K // sk
            part = torch.empty(sk, M, N, device=dev, dtype=torch.bfloat16)
            av = a.view(M, sk, ks).transpose(0, 1)  # [sk, M, ks], strides (ks, K, 1)

            def split():
                w = ws[it[0] % ncopy]
                it[0] += 1
                torch.bmm(av, w.view(N, sk, ks).permute(1, 2, 0), out=part)  # [sk, ks, N]
                h.add_(part.sum(0))

            us = timed(split)
            h.copy_(h0)
            torch.bmm(av, ws[0].view(N, sk, ks).permute(1, 2, 0), out=part)
            h.add_(part.sum(0))
            err = ((h.float() - ref).abs().max() / ref.abs().max()).item()
            print(json.dumps({"op": name, "M": M, "N": N, "K": K, "split": sk, "us": round(us, 2),
                              "tflops": round(flop / us / 1e6, 1), "rel_err": err}), flush=True)
        del ws


if __name__ == "__main__":
    main()
