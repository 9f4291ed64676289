#!/usr/bin/env python3
"""Where a gemm_sk launch spends its time: per-workgroup s_memrealtime stamps (100 MHz) from
the diagnostic build of gemm_sk.hip (-DLSA_GEMM_STAMPS -> _native/liblsa_gemm_stamps.so, built
by `python scripts/gemm_stamps.py --build` on the CPU host), for one configuration.

Per work item the stamps are: 0 segment start, 1 prologue DMA landed, 2 main loop done,
3 partial slab stored + ticket drawn, 4 fixup done, 5 epilogue done.
usage: gemm_stamps.py M N K bn grid dp split [reps] [bm] | --build"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "llm_sharding_amd", "_native", "liblsa_gemm_stamps.so")


def build():
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950", "-DLSA_GEMM_STAMPS",
           "-I", os.path.join(ROOT, "csrc", "kernels"), os.path.join(ROOT, "csrc", "kernels", "gemm_sk.hip"), "-o", SO]
    subprocess.check_call(cmd)
    print("built", SO)


def main():
    if sys.argv[1] == "--build":
        build()
        return
    import torch
    sys.path.insert(0, ROOT)
    from llm_sharding_amd.ops import hip, packing
    M, N, K, bn, grid, dp, split = (int(v) for v in sys.argv[1:8])
    reps = int(sys.argv[8]) if len(sys.argv) > 8 else 5
    bm = int(sys.argv[9]) if len(sys.argv) > 9 else 256
    L = ctypes.CDLL(SO)
    vp, i = ctypes.c_void_p, ctypes.c_int
    L.lsa_gemm_sk.argtypes = [vp, i, vp, i, i, i, i, ctypes.POINTER(hip.EpiArgs), i, i, i, i, i, i, i, vp, vp,
                              ctypes.c_longlong, i, i, vp]
    nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
    wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    ep = hip.make_epi(out=out, ldo=N)
    ws = hip.SkWorkspace("cuda", grid=max(256, grid), bn=256)
    st = torch.zeros(max(256, grid) * 32, dtype=torch.int64, device="cuda")
    L.lsa_gemm_sk_set_stamps(ctypes.c_void_p(st.data_ptr()))
    for r in range(reps):
        st.zero_()
        rc = L.lsa_gemm_sk(ctypes.c_void_p(x.data_ptr()), x.stride(0), ctypes.c_void_p(wps[r % nbuf].data_ptr()), M, N, K,
                           hip.EPI_STORE, ctypes.byref(ep), bm, bn, 0, grid, dp, split, 8,
                           ctypes.c_void_p(ws.slab.data_ptr()), ctypes.c_void_p(ws.counters.data_ptr()),
                           ws.slab.numel(), ws.counters.numel(), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc
        torch.cuda.synchronize()
    s = st.view(-1, 32).cpu().double()
    act = s[:, 0] > 0
    s = s[act]
    t0 = s[:, 0].min()
    us = (s - t0) / 100.0  # 100 MHz -> us
    us[s == 0] = float("nan")
    names = ["seg_start", "prologue", "loop_end", "ticket", "fixup", "epilogue"]
    print(f"config M={M} N={N} K={K} bm={bm} bn={bn} grid={grid} dp={dp} split={split}: {int(act.sum())} active "
          f"workgroups, kernel span {float(torch.nan_to_num(us, nan=0.0).max()):.2f} us")
    for item in range(5):
        cols = us[:, item * 6:(item + 1) * 6]
        if not torch.isfinite(cols[:, 0]).any():
            break
        med = [float(c[torch.isfinite(c)].median()) if torch.isfinite(c).any() else float("nan") for c in cols.T]
        mx = [float(c[torch.isfinite(c)].max()) if torch.isfinite(c).any() else float("nan") for c in cols.T]
        print(f"item {item}: median " + "  ".join(f"{n}={v:7.2f}" for n, v in zip(names, med)))
        print(f"        max    " + "  ".join(f"{n}={v:7.2f}" for n, v in zip(names, mx)))


if __name__ == "__main__":
    main()
