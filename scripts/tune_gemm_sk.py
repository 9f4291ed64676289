#!/usr/bin/env python3
"""Autotune gemm_sk's work decomposition per projection shape, with the epilogue the engine
runs (QKV: RoPE + KV append, o/down: residual add, gate_up: SwiGLU), weights rotated over
> 600 MB of copies so they stream from HBM as in a decode step. Residual projections are also
timed as split-K partials summed by the following norm (EPI_PARTIAL + resid_rmsnorm_partials)
against the fused EPI_RESID + rmsnorm pair; the winner goes in the entry's "partial" field. Both row-tile
heights (bm 256 / 128) are swept. Writes the winners to
llm_sharding_amd/ops/gemm_sk_tuning.json, which hip.gemm_sk_plan consults before its cost model.

usage: tune_gemm_sk.py [--rows 256,512,...] [--models llama2-7b,...] [--out PATH] [--iters N]
One JSON line per (model, shape, M) on stdout with every candidate's time."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from scripts.bench_kernels import EPIS, MODEL_HEADS, MODEL_SHAPES  # noqa: E402

DEV = "cuda"
SPLITS = (0, 1, 2, 3, 4, 6, 8)  # 0 = stream-K remainder, S = S equal K ranges per remainder tile


def timeit(fn, iters, warm=3):
    for i in range(warm):
        fn(i)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="256,384,512,640,768,1024,1536,2048")
    ap.add_argument("--models", default="llama2-7b")
    ap.add_argument("--out", default=os.path.join(ROOT, "llm_sharding_amd", "ops", "gemm_sk_tuning.json"))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-partial", action="store_true", help="skip the EPI_PARTIAL comparison")
    a = ap.parse_args()
    from llm_sharding_amd.config import llama2_7b
    from llm_sharding_amd.models.rope import rope_table
    rows = [int(r) for r in a.rows.split(",")]
    cos, sin = rope_table(llama2_7b(), 1024, DEV)
    sk_ws = hip.SkWorkspace(DEV)
    entries = []
    if os.path.exists(a.out):
        with open(a.out) as f:
            entries = json.load(f).get("entries", [])
    for model in a.models.split(","):
        for name, (N, K) in MODEL_SHAPES[model].items():
            if name == "lm_head":
                continue
            epi = EPIS[name]
            nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
            ws = [packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
            for M in rows:
                x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
                nh, nkv = MODEL_HEADS[model] if epi == hip.EPI_QKV else (1, 1)
                if epi == hip.EPI_QKV:
                    q = torch.zeros(M, nh * 128, dtype=torch.bfloat16, device=DEV)
                    kc = torch.zeros(M, nkv, 1024, 128, dtype=torch.bfloat16, device=DEV)
                    vc = torch.zeros_like(kc)
                    slot = torch.arange(M, dtype=torch.int32, device=DEV)
                    pos = torch.full((M,), 100, dtype=torch.int32, device=DEV)
                    ep = hip.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, cos=cos, sin=sin,
                                      ldo=q.shape[1], n_heads=nh, n_kv=nkv, head_dim=128, t_max=1024)
                elif epi == hip.EPI_SWIGLU:
                    out = torch.zeros(M, N // 2, dtype=torch.bfloat16, device=DEV)
                    ep = hip.make_epi(out=out, ldo=N // 2)
                else:
                    out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
                    ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
                res = []
                for bm in (256, 128):
                    for bn in (256, 192, 128):
                        if N % (16 if bn == 192 else bn):
                            continue
                        # dp 1: whole-tile rounds first, the remainder by split / stream-K; dp 0 (split 0):
                        # pure stream-K over the whole grid (every CU busy when the tiles do not fill a round)
                        for dp, sp in [(1, s_) for s_ in SPLITS] + [(0, 0)]:
                            try:
                                us = timeit(lambda i: hip.gemm_sk(x, ws[i % nbuf], M, N, K, epi, ep, bn=bn, grid=hip.N_CU,
                                                                  dp=dp, split=sp, ws=sk_ws, bm=bm), a.iters)
                            except (RuntimeError, ValueError) as e:  # a config the host rejects for this shape
                                print(f"# skip bm={bm} bn={bn} dp={dp} split={sp}: {e}", file=sys.stderr)
                                continue
                            res.append((round(us, 2), bn, sp, bm, dp))
                res.sort()
                partial = None
                if epi == hip.EPI_RESID and 128 < M <= hip.PARTIAL_MAX_ROWS and not a.no_partial:
                    # the engine follows every residual projection with an RMSNorm: compare
                    # fused (EPI_RESID + rmsnorm) against EPI_PARTIAL + resid_rmsnorm_partials
                    xn = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
                    pbuf = torch.zeros(hip.PARTIAL_MAX_SPLIT, M, N, dtype=torch.float32, device=DEV)
                    bbn, bsp, bbm, bdp = res[0][1], res[0][2], res[0][3], res[0][4]

                    def fused(i):
                        hip.gemm_sk(x, ws[i % nbuf], M, N, K, epi, ep, bn=bbn, grid=hip.N_CU, dp=bdp, split=bsp, ws=sk_ws,
                                    bm=bbm)
                        hip.rmsnorm(out, None, xn, M, 1e-5, N)
                    t_fused = timeit(fused, a.iters)
                    pres = []
                    for bn in (256, 192, 128):
                        if N % (16 if bn == 192 else bn):
                            continue
                        tiles = -(-M // hip.SK_BM) * -(-N // bn)
                        for sp in range(1, hip.PARTIAL_MAX_SPLIT + 1):
                            if tiles * sp > hip.N_CU or sp > K // 64:
                                continue
                            epp = hip.make_epi(out=pbuf, ldo=N)

                            def part(i):
                                hip.gemm_sk(x, ws[i % nbuf], M, N, K, hip.EPI_PARTIAL, epp, bn=bn, grid=hip.N_CU, dp=0,
                                            split=sp, ws=sk_ws, out_numel=pbuf.numel())
                                hip.resid_rmsnorm_partials(out, pbuf, sp, M, 1e-5, out=xn)
                            pres.append((round(timeit(part, a.iters), 2), bn, sp))
                    pres.sort()
                    partial = {"fused_us": round(t_fused, 2), "best": pres[0] if pres else None, "all": pres}
                plan = hip.gemm_sk_plan(M, N, K, tuned=False)
                model_us = next((r[0] for r in res if (r[1], r[2], r[3], r[4]) == (plan[0], plan[3], plan[4], plan[2])),
                                None)
                fl = 2.0 * M * N * K
                line = {"model": model, "shape": name, "N": N, "K": K, "M": M, "epi": epi,
                        "best_us": res[0][0], "best": [res[0][1], hip.N_CU, res[0][4], res[0][2], res[0][3]],
                        "best_tflops": round(fl / res[0][0] / 1e6, 1), "cost_model_us": model_us,
                        "all": res, "partial": partial}
                print(json.dumps(line), flush=True)
                entries = [e for e in entries if (e["N"], e["K"], e["M"]) != (N, K, M)]
                ent = {"N": N, "K": K, "M": M, "cfg": line["best"], "us": res[0][0]}
                if partial is not None:  # [bn, split] when partials + fused norm beat EPI_RESID + norm
                    pb = partial["best"]
                    ent["partial"] = [pb[1], pb[2]] if pb and pb[0] < partial["fused_us"] else None
                entries.append(ent)
            del ws
            torch.cuda.empty_cache()
    entries.sort(key=lambda e: (e["N"], e["K"], e["M"]))
    with open(a.out, "w") as f:
        json.dump({"note": "gemm_sk (bn, grid, dp, split) per (N, K, M), measured by scripts/tune_gemm_sk.py "
                           "on MI355X with the engine's epilogues", "entries": entries}, f, indent=0)


if __name__ == "__main__":
    main()
