#!/usr/bin/env python3
"""Where gemv_coop.hip's time goes at 32..128 rows: the tuned configuration timed (hipGraph, cold
weights) on timing builds: production, exit after the main loop / after the k-group / split
reduction (-DLSA_COOP_ABLATE=1/2), the epilogue without its stores / with constant stores only
(3/4; outputs garbage). (A round-3 variant with non-temporal /
write-through epilogue stores changed nothing: profiles/r3_coop_phases.jsonl.)

    python scripts/coop_phases.py --build        (CPU host)
    python scripts/coop_phases.py [rows ...]     (GPU: one JSON line per shape x rows)"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# name -> compile flags
VARIANTS = {"prod": [], "main_loop": ["-DLSA_COOP_ABLATE=1"], "loop_reduce": ["-DLSA_COOP_ABLATE=2"],
            "epi_no_store": ["-DLSA_COOP_ABLATE=3"], "epi_const_store": ["-DLSA_COOP_ABLATE=4"]}


def so(v):
    return os.path.join(ROOT, "llm_sharding_amd", "_native", f"liblsa_coop_{v}.so")


def build():
    for v, flags in VARIANTS.items():
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950"]
                              + flags + ["-I", os.path.join(ROOT, "csrc", "kernels"),
                                         os.path.join(ROOT, "csrc", "kernels", "gemv_coop.hip"), "-o", so(v)])
        print("built", so(v))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--build":
        build()
        return
    import torch
    sys.path.insert(0, ROOT)
    from llm_sharding_amd.ops import hip, packing
    from scripts.bench_kernels import timeit
    rows = [int(v) for v in sys.argv[1:]] or [32, 64, 128]
    vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    libs = {}
    for v in VARIANTS:
        L = ctypes.CDLL(so(v))
        L.lsa_gemv_coop.argtypes = [vp, i, vp, vp, i, i, i, i, f, i, ctypes.POINTER(hip.EpiArgs), i, i, i, i, i, vp,
                                    vp, vp]
        libs[v] = L
    ws = hip.CoopWorkspace("cuda", slab_floats=1 << 25)
    for name, (N, K, epi) in {"qkv": (12288, 4096, hip.EPI_STORE), "o": (4096, 4096, hip.EPI_RESID),
                              "gate_up": (22016, 4096, hip.EPI_SWIGLU), "down": (4096, 11008, hip.EPI_RESID)}.items():
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        for M in rows:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
            ep = hip.make_epi(out=out, resid=out, ldo=N if epi != hip.EPI_SWIGLU else N // 2, ldr=N)
            algo, cfg = packing.proj_config(N // 16, M, need_even=epi == hip.EPI_SWIGLU, k=K)
            if algo != "coop":
                continue
            tnw, nw, kf, sk, kw = cfg
            res = {}
            for v in VARIANTS:
                L = libs[v]

                def run(j):
                    rc = L.lsa_gemv_coop(x.data_ptr(), K, None, wps[j % nbuf].data_ptr(), M, N, K, 0, 1e-5, epi,
                                         ctypes.byref(ep), tnw, nw, kf, sk, kw, ws.slab.data_ptr(),
                                         ws.counters.data_ptr(), torch.cuda.current_stream().cuda_stream)
                    assert rc == 0, rc
                res[v] = round(timeit(run), 2)
            print(json.dumps({"shape": name, "M": M, "cfg": list(cfg), "us": res,
                              "weight_TBps": round(N * K * 2 / res["prod"] / 1e6, 2)}), flush=True)
        del wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
