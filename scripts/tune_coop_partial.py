#!/usr/bin/env python3
"""Residual decode projections (o, down) at 17..128 rows: the coop kernel's in-kernel split
reduction + residual epilogue (tuned config) against EPI_PARTIAL (every split stores its fp32
tile, no last arriver) + lsa_resid_rmsnorm_partials, every coop config with <= 8 splits. Weights
rotated beyond the Infinity Cache; each variant timed as one hipGraph of 20 launches.

usage: tune_coop_partial.py [--models llama2-7b] [--rows 32,64,128] [--tune-file PATH]
One JSON line per (shape, rows); with --tune-file the winning partial configs are merged into
that table as "coop_partial" entries (None when the fused path wins)."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import MODEL_SHAPES, timeit  # noqa: E402

DEV = "cuda"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="llama2-7b")
    ap.add_argument("--rows", default="32,64,128")
    ap.add_argument("--tune-file", default="")
    a = ap.parse_args()
    hip.lib()
    ws = hip.CoopWorkspace(DEV, slab_floats=1 << 24)
    found = {}
    for model in a.models.split(","):
        for name in ("o", "down"):
            N, K = MODEL_SHAPES[model][name]
            nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
            wps = [packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
            for M in (int(r) for r in a.rows.split(",")):
                x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
                h = torch.randn(M, N, device=DEV).to(torch.bfloat16)
                ep = hip.make_epi(out=h, resid=h, ldo=N, ldr=N)
                fused = timeit(lambda i: hip.gemv(x, wps[i % nbuf], M, N, K, hip.EPI_RESID, ep, ws=ws))
                part = ws.slab[:8 * M * N].view(8, M, N)
                epp = hip.make_epi(out=part, ldo=N)
                res = []
                for c in packing.coop_candidates(N // 16, K, M):
                    sk = c[3]
                    if not 1 <= sk <= 8:  # sk = 0 (ragged): no split partials
                        continue

                    def run(i, c=c, sk=sk):
                        hip.gemv(x, wps[i % nbuf], M, N, K, hip.EPI_PARTIAL, epp, coop=c, ws=ws,
                                 out_numel=part.numel())
                        hip.resid_rmsnorm_partials(h, part, sk, M, 1e-5)
                    res.append((round(timeit(run), 2), list(c)))
                res.sort()
                best = res[0] if res else None
                line = {"model": model, "shape": name, "N": N, "K": K, "M": M, "fused_us": round(fused, 2),
                        "fused_cfg": list(packing.proj_config(N // 16, M, k=K)[1]),
                        "partial_best": best, "partial_all": res[:6]}
                print(json.dumps(line), flush=True)
                key = (N, K, packing.row_blocks(M))
                if key not in found:  # the smallest rows of a row block decide (as the GEMV table)
                    found[key] = best[1] if best and best[0] < fused else None
            del wps
            torch.cuda.empty_cache()
    if a.tune_file:
        tab = json.load(open(a.tune_file)) if os.path.exists(a.tune_file) else {"entries": []}
        ents = [e for e in tab["entries"] if not (e.get("algo") == "coop_partial"
                                                  and (e["N"], e["K"], e["mb"]) in found)]
        for (N, K, mb), cfg in sorted(found.items()):
            if cfg is not None:
                ents.append({"N": N, "K": K, "mb": mb, "even": False, "algo": "coop_partial", "cfg": cfg})
        tab["entries"] = ents
        with open(a.tune_file, "w") as f:
            json.dump(tab, f, indent=0)


if __name__ == "__main__":
    main()
