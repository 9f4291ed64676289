#!/usr/bin/env python3
"""gemm_wr EPI_PARTIAL (K split) at decode batch sizes for every 7B projection shape vs the
tuned coop GEMV path the engine runs at <= 128 rows: cold weights, median of 20.
usage: wr_partial_probe.py [rows ...]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip, packing  # noqa: E402


def timeit(fn, reps=20):
    fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for r in range(reps):
        e0.record()
        fn(r)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    ts.sort()
    return round(ts[len(ts) // 2], 2)


def main():
    hip.lib()
    rows = [int(v) for v in sys.argv[1:]] or [128, 64]
    shapes = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008)}
    part = torch.empty(8, 128, 22016, device="cuda")
    cws = hip.CoopWorkspace("cuda") if hasattr(hip, "CoopWorkspace") else None
    for name, (N, K) in shapes.items():
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        for M in rows:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            res = {"shape": name, "M": M}
            out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")

            def coop(r):  # the engine's <= 128-row path (tuned coop / gemv plan), store epilogue
                hip.gemv(x, wps[r % nbuf], M, N, K, hip.EPI_STORE, hip.make_epi(out=out, ldo=N), ws=cws)
            try:
                res["gemv_tuned"] = timeit(coop)
            except Exception as e:  # noqa: BLE001
                res["gemv_tuned"] = str(e)[:80]
            for bn in (128, 256):
                if N % bn:
                    continue
                for sp in (1, 2, 3, 4, 6, 8):
                    if K // 256 < sp or sp * M * N > part.numel():
                        continue

                    def wrp(r, bn=bn, sp=sp):
                        hip.gemm_wr(x, wps[r % nbuf], M, N, K, hip.EPI_PARTIAL, hip.make_epi(out=part, ldo=N), bn=bn,
                                    split=sp, out_numel=part.numel())
                    res[f"wr_bn{bn}_s{sp}"] = timeit(wrp)
            best = min((v, k) for k, v in res.items() if k.startswith("wr_"))
            res["best_wr"] = best
            res["wt_TBps_best"] = round(N * K * 2 / best[0] / 1e6, 2)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
