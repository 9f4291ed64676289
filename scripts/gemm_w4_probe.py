#!/usr/bin/env python3
"""scripts/probes/gemm_w4.hip (probe library probe_bin/liblsa_gemm_w4.so, scripts/probes/build_gemm_w4.sh; one wave per SIMD, 256 x 256 tiles, 128 x 128 per wave, 32-deep 4-slot LDS-DMA
ring, one barrier per stage) against the engine's GEMM dispatch (hip.gemm: gemm_sk / gemm_wr) and
hipBLASLt (torch.matmul) at projection shapes, plain-store epilogue, cold weights (rotated over
> 600 MB), 20 launches per hipGraph. Also checks gemm_w4 against an fp32 reference (global +
per-tile + per-row error, utils/numerics.py).

usage: gemm_w4_probe.py [M,M,...] [shape,shape,...]   one JSON line per (shape, M)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402
from llm_sharding_amd.utils.numerics import rel_err  # noqa: E402
from scripts.bench_kernels import timeit  # noqa: E402

_W4 = None


def gemm_w4(a, wp, M, N, K, ep, grid=0, variant=0):
    global _W4
    if _W4 is None:
        import ctypes
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        _W4 = ctypes.CDLL(os.path.join(root, "probe_bin", "liblsa_gemm_w4.so"))
        vp, i = ctypes.c_void_p, ctypes.c_int
        _W4.lsa_gemm_w4.argtypes = [vp, i, vp, i, i, i, ctypes.POINTER(hip.EpiArgs), i, i, vp]
    rc = _W4.lsa_gemm_w4(hip._p(a), a.stride(0), hip._p(wp), M, N, K, ctypes_byref(ep), grid, variant, hip._stream())
    assert rc == 0, rc


def ctypes_byref(x):
    import ctypes
    return ctypes.byref(x)

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "down": (4096, 11008), "gate_up_22528": (22528, 4096),
          "o70": (8192, 8192), "down70": (8192, 28672)}


def main():
    rows = [int(r) for r in sys.argv[1].split(",")] if len(sys.argv) > 1 else [512, 2048, 16384]
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else ["o", "qkv", "down"]
    sk_ws = hip.SkWorkspace("cuda")
    for name in names:
        N, K = SHAPES[name]
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        ws_ = [torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16) for _ in range(nbuf)]
        wps = [packing.pack_b(w) for w in ws_]
        for M in rows:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
            out2 = torch.empty_like(out)
            ref = torch.empty_like(out)
            ep = hip.make_epi(out=out, ldo=N)
            ep2 = hip.make_epi(out=out2, ldo=N)
            gemm_w4(x, wps[0], M, N, K, ep)
            torch.cuda.synchronize()
            e = rel_err(out, x.float() @ ws_[0].float().T)
            t_w4 = timeit(lambda i: gemm_w4(x, wps[i % nbuf], M, N, K, ep))
            t_v = {}
            for v in (1, 2):
                gemm_w4(x, wps[0], M, N, K, ep2, variant=v)
                torch.cuda.synchronize()
                ev = rel_err(out2, x.float() @ ws_[0].float().T)
                t_v[f"w4v{v}_us"] = round(timeit(lambda i: gemm_w4(x, wps[i % nbuf], M, N, K, ep2, variant=v)), 2)
                t_v[f"w4v{v}_ok"] = bool(ev < 8e-3)
            t_ours = timeit(lambda i: hip.gemm(x, wps[i % nbuf], M, N, K, hip.EPI_STORE, ep2, sk_ws=sk_ws))
            t_blas = timeit(lambda i: torch.matmul(x, ws_[i % nbuf].t(), out=ref))
            fl = 2.0 * M * N * K
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "w4_us": round(t_w4, 2),
                              "w4_tflops": round(fl / t_w4 / 1e6, 1), "ours_us": round(t_ours, 2),
                              "ours_tflops": round(fl / t_ours / 1e6, 1), "hipblaslt_us": round(t_blas, 2),
                              "hipblaslt_tflops": round(fl / t_blas / 1e6, 1), "w4_vs_ours": round(t_ours / t_w4, 3),
                              "w4_err": float(f"{e.global_:.2e}"), "w4_err_local": float(f"{e.local:.2e}"),
                              "w4_ok": bool(e < 8e-3), **t_v}), flush=True)
        del ws_, wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
