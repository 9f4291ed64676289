#!/usr/bin/env python3
"""One gemm_sk configuration, timed in a hipGraph with weights cold (rotated over > 600 MB) and
hot (one copy, L2 / Infinity-Cache resident) - separates the weight-stream latency from the
MFMA / LDS work of the main loop. Also the target for rocprofv3 --pmc passes.

usage: sk_one.py M N K bn split [epi=store|resid]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import timeit  # noqa: E402


def main():
    M, N, K, bn, split = (int(v) for v in sys.argv[1:6])
    epi = hip.EPI_RESID if len(sys.argv) > 6 and sys.argv[6] == "resid" else hip.EPI_STORE
    nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
    wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
    ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N) if epi == hip.EPI_RESID else hip.make_epi(out=out, ldo=N)
    ws = hip.SkWorkspace("cuda")
    run = lambda i, w: hip.gemm_sk(x, w(i), M, N, K, epi, ep, bn=bn, grid=hip.N_CU, dp=1, split=split, ws=ws)  # noqa: E731
    cold = timeit(lambda i: run(i, lambda j: wps[j % nbuf]))
    hot = timeit(lambda i: run(i, lambda j: wps[0]))
    fl = 2.0 * M * N * K
    print(json.dumps({"M": M, "N": N, "K": K, "bn": bn, "split": split, "epi": epi, "cold_us": round(cold, 2),
                      "hot_us": round(hot, 2), "cold_tflops": round(fl / cold / 1e6, 1),
                      "hot_tflops": round(fl / hot / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
