#!/usr/bin/env python3
"""Kernel micro-benchmarks on the GPU: decode GEMV (every tile/wave config), attention
(split factors), prefill GEMM. Prints achieved HBM TB/s or TFLOP/s per case.

Timing: CUDA events around R back-to-back launches after warm-up; weights are rotated
through several copies whose total exceeds the 256 MiB Infinity Cache, so every launch
streams from HBM (cdna_hip_programming.md §2 'Caches & the L3 over-fetch masking').
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402

DEV = "cuda"


def timeit(fn, reps=20, replays=3):
    """Per-launch time (us) of ``reps`` launches captured in one hipGraph (no host overhead)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(0)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(reps):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(replays):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (reps * replays) * 1e3


MODEL_SHAPES = {
    "llama2-7b": {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008),
                  "lm_head": (32000, 4096)},
    "llama2-70b": {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672),
                   "lm_head": (32000, 8192)},
    "llama3.2-3b": {"qkv": (5120, 3072), "o": (3072, 3072), "gate_up": (16384, 3072), "down": (3072, 8192),
                    "lm_head": (128256, 3072)},
}
# (n_heads, n_kv) of each model: the QKV epilogue writes k/v into a cache of n_kv heads
MODEL_HEADS = {"llama2-7b": (32, 32), "llama2-70b": (64, 8), "llama3.2-3b": (24, 8)}
EPIS = {"qkv": hip.EPI_QKV, "o": hip.EPI_RESID, "gate_up": hip.EPI_SWIGLU, "down": hip.EPI_RESID,
        "lm_head": hip.EPI_ARGMAX}


def gemv_sweep(out_rows, models, rows_list, tune_entries, fp8=False):
    from llm_sharding_amd.models.rope import rope_table
    from llm_sharding_amd.config import llama2_7b
    cos, sin = rope_table(llama2_7b(), 1024, DEV)
    cws = hip.CoopWorkspace(DEV, slab_floats=1 << 25)
    for model in models:
        for name, (N, K) in MODEL_SHAPES[model].items():
            epi = EPIS[name]
            nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
            ws = [packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
            if fp8:
                nbuf8 = max(2, (600 << 20) // (N * K) + 1)
                q8, s8 = packing.quantize_fp8_rows(torch.randn(N, K, device=DEV).mul_(0.02))
                w8 = [packing.pack_b_fp8(q8).view(-1).clone() for _ in range(nbuf8)]
            for M in rows_list:
                x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
                out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
                nh, nkv = MODEL_HEADS[model] if epi == hip.EPI_QKV else (1, 1)
                assert epi != hip.EPI_QKV or N == (nh + 2 * nkv) * 128, (model, N)
                q = torch.zeros(M, max(N, 128), dtype=torch.bfloat16, device=DEV)
                kc = torch.zeros(M, nkv, 1024, 128, dtype=torch.bfloat16, device=DEV)
                slot = torch.arange(M, dtype=torch.int32, device=DEV)
                pos = torch.full((M,), 100, dtype=torch.int32, device=DEV)
                keys = torch.zeros(M, dtype=torch.int64, device=DEV)
                if epi == hip.EPI_QKV:
                    ep = hip.make_epi(out=q, k_cache=kc, v_cache=kc, slot=slot, pos=pos, cos=cos, sin=sin,
                                      ldo=q.shape[1], n_heads=nh, n_kv=nkv, head_dim=128, t_max=1024)
                elif epi == hip.EPI_ARGMAX:
                    ep = hip.make_epi(keys=keys)
                else:
                    ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
                norm = epi in (hip.EPI_QKV, hip.EPI_SWIGLU, hip.EPI_ARGMAX)
                even = epi == hip.EPI_SWIGLU
                res = []
                for tn, nw, u in packing.gemv_candidates(N // 16, K, M, even):
                    us = timeit(lambda i: hip.gemv(x, ws[i % nbuf], M, N, K, epi, ep, norm=norm, tn=tn, nw=nw, u=u))
                    res.append((us, "gemv", (tn, nw, u), N * K * 2 / us / 1e6))
                for cfg in packing.coop_candidates(N // 16, K, M, even):
                    us = timeit(lambda i: hip.gemv(x, ws[i % nbuf], M, N, K, epi, ep, norm=norm, coop=cfg, ws=cws))
                    res.append((us, "coop", cfg, N * K * 2 / us / 1e6))
                if fp8:
                    r8 = []
                    for cfg in packing.fp8_gemv_candidates(N // 16, K, M, even) if M <= 64 else []:
                        us = timeit(lambda i: hip.proj_fp8(x, w8[i % nbuf8], s8, M, N, K, epi, ep, norm=norm,
                                                           algo=("fp8", cfg)))
                        r8.append((us, "fp8", cfg, N * K / us / 1e6))
                    for cfg in packing.coop_fp8_candidates(N // 16, K, M):
                        us = timeit(lambda i: hip.proj_fp8(x, w8[i % nbuf8], s8, M, N, K, epi, ep, norm=norm,
                                                           algo=("coop_fp8", cfg), ws=cws))
                        r8.append((us, "coop_fp8", cfg, N * K / us / 1e6))
                    r8.sort(key=lambda r: r[0])
                    line8 = {"kernel": "gemv_fp8", "model": model, "shape": name, "N": N, "K": K, "M": M,
                             "best_us": round(r8[0][0], 2), "best_algo": r8[0][1], "best_cfg": list(r8[0][2]),
                             "best_TBps": round(r8[0][3], 2), "all": [(round(r[0], 2), r[1]) + tuple(r[2]) for r in r8]}
                    print(json.dumps(line8), flush=True)
                    out_rows.append(line8)
                    tune_entries.setdefault((N, K, packing.row_blocks(M), even, "fp8"), (r8[0][1], list(r8[0][2])))
                res.sort(key=lambda r: r[0])
                best = res[0]
                line = {"kernel": "gemv", "model": model, "shape": name, "N": N, "K": K, "M": M,
                        "best_us": round(best[0], 2), "best_algo": best[1], "best_cfg": list(best[2]),
                        "best_TBps": round(best[3], 2),
                        "all": [(round(r[0], 2), r[1]) + tuple(r[2]) for r in res]}
                print(json.dumps(line), flush=True)
                out_rows.append(line)
                tune_entries.setdefault((N, K, packing.row_blocks(M), even), (best[1], list(best[2])))  # smallest M of a row block wins (batch-1 latency)
            del ws
            torch.cuda.empty_cache()


def attn_sweep(out_rows):
    nh = nkv = 32
    hd = 128
    for rows in (1, 16, 64):
        for T in (128, 512, 2048):
            kc = torch.randn(rows, nkv, 2048, hd, device=DEV).to(torch.bfloat16)
            vc = torch.randn_like(kc)
            q = torch.randn(rows, nh * hd, device=DEV).to(torch.bfloat16)
            slot = torch.arange(rows, dtype=torch.int32, device=DEV)
            pos = torch.full((rows,), T - 1, dtype=torch.int32, device=DEV)
            out = torch.zeros(rows, nh * hd, dtype=torch.bfloat16, device=DEV)
            po = torch.zeros(rows * nh * 16 * hd, device=DEV)
            pl = torch.zeros(rows * nh * 16, device=DEV)
            res = []
            for ns in (1, 2, 4, 8, 16):
                us = timeit(lambda i: hip.attn(q, kc, vc, slot, pos, rows, nh, nkv, hd, ns, po, pl, out))
                gbs = rows * T * nkv * hd * 2 * 2 / us / 1e6
                res.append((round(us, 2), ns, round(gbs, 2)))
            line = {"kernel": "attn", "rows": rows, "T": T, "results(us,nsplit,TBps)": res}
            print(json.dumps(line), flush=True)
            out_rows.append(line)


def gemm_sweep(out_rows, rows_list=(128, 256, 512, 1024, 2048, 8192)):
    ws = hip.CoopWorkspace(DEV, slab_floats=1 << 26, groups=1 << 15)
    for (N, K) in ((12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008)):
        w = packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16))
        for M in rows_list:
            a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
            out = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
            ep = hip.make_epi(out=out, ldo=N)
            res = []
            for sk in (1, 2, 3, 4, 6, 8):
                if sk > 1 and hip.gemm_slab_floats(M, N, sk) > ws.slab.numel():
                    continue
                us = timeit(lambda i: hip.gemm(a, w, M, N, K, hip.EPI_STORE, ep, sk=sk, ws=ws), reps=10)
                res.append((round(us, 1), sk))
            res.sort()
            auto = hip.gemm_split(M, N, K, 2 if N % 128 == 0 else 1)
            line = {"kernel": "gemm", "N": N, "K": K, "M": M, "best_us": res[0][0], "best_sk": res[0][1],
                    "auto_sk": auto, "TFLOPs": round(2 * M * N * K / res[0][0] / 1e6, 1), "all(us,sk)": res}
            print(json.dumps(line), flush=True)
            out_rows.append(line)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="gemv,attn,gemm")
    ap.add_argument("--models", default="llama2-7b")
    ap.add_argument("--rows", default="1,16,32,64")
    ap.add_argument("--tune", action="store_true", help="merge the winners into the tuning table")
    ap.add_argument("--tune-file", default=packing.TUNING_FILE,
                    help="table to write (on a gpurun box: a path under gpurun_out/, then copy it back)")
    ap.add_argument("--fp8", action="store_true", help="also sweep the fp8-weight (W8A16) kernels")
    ap.add_argument("--out", default="gpurun_out/bench_kernels.json")
    a = ap.parse_args()
    hip.lib()
    rows = []
    tune = {}
    if "gemv" in a.only:
        gemv_sweep(rows, a.models.split(","), [int(r) for r in a.rows.split(",")], tune, fp8=a.fp8)
        if a.tune:
            old = {}
            if os.path.exists(packing.TUNING_FILE):
                for e in json.load(open(packing.TUNING_FILE)).get("entries", []):
                    key = (e["N"], e["K"], e["mb"], bool(e["even"]))
                    if e.get("algo") in ("fp8", "coop_fp8"):
                        key = key + ("fp8",)
                    elif e.get("algo") == "coop_partial":
                        key = key + ("partial",)
                    old[key] = (e.get("algo", "gemv"), e["cfg"])
            old.update(tune)
            ents = [{"N": k[0], "K": k[1], "mb": k[2], "even": k[3], "algo": v[0], "cfg": v[1]}
                    for k, v in sorted(old.items(), key=lambda kv: tuple(map(str, kv[0])))]
            with open(a.tune_file, "w") as f:
                json.dump({"device": torch.cuda.get_device_name(), "entries": ents}, f, indent=1)
            print(f"wrote {len(ents)} tuning entries to {a.tune_file}")
    if "attn" in a.only:
        attn_sweep(rows)
    if "gemm" in a.only:
        gemm_sweep(rows)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
