#!/usr/bin/env python3
"""PMC probe of the four Llama-2-7B projection GEMMs at decode-batch rows: the engine's dispatch
(hip.gemm: gemm_wr where routed, gemm_sk elsewhere; plain-store epilogue) and torch.matmul
(hipBLASLt) on the same operands, eager launches with cold weights (rotating copies > 600 MB, as
in a decode step). Run under ``rocprofv3 --pmc ...`` (one pass per counter group) or
``--kernel-trace``; scripts/gemm_pmc_summary.py attributes every dispatch to its (impl, shape)
through the 1-element fill kernel launched before each block.

usage: gemm_pmc_probe.py [--rows 512] [--launches 6] [--impls ours,coop,blas] [--model llama2-7b]
Prints the block order as one JSON line (the summary reads it from the log)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import MODEL_SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=512)
    ap.add_argument("--launches", type=int, default=6)
    ap.add_argument("--impls", default="ours,blas")
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    a = ap.parse_args()
    M = a.rows
    sk_ws = hip.SkWorkspace("cuda")
    marker = torch.empty(1, device="cuda")
    blocks = []
    for name in a.shapes.split(","):
        N, K = MODEL_SHAPES[a.model][name]
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        ws_ = [torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16) for _ in range(nbuf)]
        wps = [packing.pack_b(w) for w in ws_]
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        ep = hip.make_epi(out=out, ldo=N)
        wr = hip.gemm_wr_plan(M, N, K, hip.EPI_STORE, ep)
        plan = ["gemm_wr", wr] if wr else list(hip.gemm_sk_plan(M, N, K))
        for impl in a.impls.split(","):
            torch.cuda.synchronize()
            marker.fill_(float(len(blocks)))  # block separator in the dispatch stream
            for i in range(a.launches):
                if impl == "ours":
                    hip.gemm(x, wps[(i + 1) % nbuf], M, N, K, hip.EPI_STORE, ep, sk_ws=sk_ws)
                elif impl == "coop":  # the decode GEMV family at <= 128 rows (tuned config)
                    hip.gemv(x, wps[(i + 1) % nbuf], M, N, K, hip.EPI_STORE, ep)
                else:
                    torch.matmul(x, ws_[(i + 1) % nbuf].t(), out=out)
            torch.cuda.synchronize()
            blocks.append({"impl": impl, "shape": name, "M": M, "N": N, "K": K,
                           "plan": plan if impl == "ours" else ("coop (gemv_tuning.json)" if impl == "coop" else "hipblaslt")})
        del ws_, wps
        torch.cuda.empty_cache()
    print(json.dumps({"blocks": blocks}), flush=True)


if __name__ == "__main__":
    main()
