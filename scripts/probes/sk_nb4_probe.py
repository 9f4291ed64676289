#!/usr/bin/env python3
"""gemm_sk.hip's 4-buffer DMA ring (bm 128 x bn 128, ~2.5 K-tiles = 80 KiB in flight per CU)
against its 3-buffer ring and against the decode GEMV kernels (gemv / gemv_coop, tuned) at
decode-sized M: the weights stream from HBM (rotated over > 600 MB of copies), where the bytes
in flight per CU bound the rate. One JSON line per (shape, M): best time per kernel family and
its config, weight TB/s, relative error vs torch fp32.
usage: sk_nb4_probe.py [M,M,...]

Round-4 result (profiles/r4_sk_ring_depth_probe.jsonl): the 4-buffer ring measured the same as
the 3-buffer ring at every shape and M (64-512 rows, within 1-3 %), so the variant was removed
from gemm_sk.hip; running this probe again needs that variant back (nb = 4)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import MODEL_SHAPES, timeit  # noqa: E402


def main():
    rows = [int(r) for r in sys.argv[1].split(",")] if len(sys.argv) > 1 else [64, 128, 256, 512]
    ws = hip.SkWorkspace("cuda", grid=1024, bn=256)
    cws = hip.CoopWorkspace("cuda", slab_floats=1 << 25, groups=1 << 15)
    for name, (N, K) in MODEL_SHAPES["llama2-7b"].items():
        if name == "lm_head":
            continue
        nbuf = max(2, (640 << 20) // (N * K * 2) + 1)
        w_rm = [torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16) for _ in range(nbuf)]
        wps = [packing.pack_b(w) for w in w_rm]
        for M in rows:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            ep = hip.make_epi(out=out, ldo=N)
            ref = x.float() @ w_rm[0].float().T
            rec = {"shape": name, "M": M, "N": N, "K": K}

            def err():
                torch.cuda.synchronize()
                return float(f"{((out.float() - ref).norm() / ref.norm()).item():.1e}")
            if M <= 128:
                t = timeit(lambda i: hip.gemv(x, wps[i % nbuf], M, N, K, hip.EPI_STORE, ep, ws=cws))
                hip.gemv(x, wps[0], M, N, K, hip.EPI_STORE, ep, ws=cws)
                rec["gemv_tuned"] = [round(t, 2), err()]
            plan = hip.gemm_sk_plan(M, N, K)
            t = timeit(lambda i: hip.gemm_sk(x, wps[i % nbuf], M, N, K, hip.EPI_STORE, ep, ws=ws))
            hip.gemm_sk(x, wps[0], M, N, K, hip.EPI_STORE, ep, ws=ws)
            rec["sk_plan"] = [round(t, 2), list(plan), err()]
            for nb in (3, 4):
                best = None
                for split in (0, 1, 2, 3, 4, 6, 8):
                    for dp in (1, 0):
                        def run(i, split=split, dp=dp, nb=nb):
                            hip.gemm_sk(x, wps[i % nbuf], M, N, K, hip.EPI_STORE, ep, bn=128, bm=128, nb=nb,
                                        grid=hip.N_CU, dp=dp, split=split, ws=ws)
                        try:
                            t = timeit(run)
                        except (RuntimeError, ValueError):
                            continue
                        if best is None or t < best[0]:
                            run(0)
                            best = [round(t, 2), {"split": split, "dp": dp}, err()]
                rec[f"sk128_nb{nb}"] = best
            fams = [(k, v[0]) for k, v in rec.items() if isinstance(v, list) and v and isinstance(v[0], float)]
            k, t = min(fams, key=lambda kv: kv[1])
            rec["best"] = k
            rec["best_weight_TBps"] = round(N * K * 2 / t / 1e6, 2)
            print(json.dumps(rec), flush=True)
        del w_rm, wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
