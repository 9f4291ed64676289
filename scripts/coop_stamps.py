#!/usr/bin/env python3
"""Where a gemv_coop launch spends its time after the main loop: per-workgroup s_memrealtime stamps
(100 MHz) from the diagnostic build (-DLSA_COOP_STAMPS -> _native/liblsa_coop_stamps.so, built by
`python scripts/coop_stamps.py --build` on the CPU host), tuned config of the 7B shapes.

Stamps: 0 start, 1 main loop done (wave 0), 2 all waves done, 3 k-group sum done, 4 slab stored,
5 ticket drawn, 6 (last arriver) slabs summed, 7 tile in LDS, 8 epilogue done.
usage: coop_stamps.py [rows ...] | --build   (one text block per shape x rows)"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "llm_sharding_amd", "_native", "liblsa_coop_stamps.so")
NAMES = ["start", "loop_w0", "loop_all", "kgroup", "slab", "ticket", "summed", "tile", "epi"]


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--build":
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                               "-DLSA_COOP_STAMPS", "-I", os.path.join(ROOT, "csrc", "kernels"),
                               os.path.join(ROOT, "csrc", "kernels", "gemv_coop.hip"), "-o", SO])
        return
    import torch
    sys.path.insert(0, ROOT)
    from llm_sharding_amd.ops import hip, packing
    rows = [int(v) for v in sys.argv[1:]] or [64, 128]
    L = ctypes.CDLL(SO)
    vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    L.lsa_gemv_coop.argtypes = [vp, i, vp, vp, i, i, i, i, f, i, ctypes.POINTER(hip.EpiArgs), i, i, i, i, i, vp, vp, vp]
    ws = hip.CoopWorkspace("cuda", slab_floats=1 << 25)
    st = torch.zeros(4096 * 16, dtype=torch.int64, device="cuda")
    L.lsa_coop_set_stamps(ctypes.c_void_p(st.data_ptr()))
    for name, (N, K, epi) in {"qkv": (12288, 4096, hip.EPI_STORE), "o": (4096, 4096, hip.EPI_RESID),
                              "down": (4096, 11008, hip.EPI_RESID)}.items():
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        for M in rows:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
            ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
            algo, cfg = packing.proj_config(N // 16, M, k=K)
            if algo != "coop":
                continue
            tnw, nw, kf, sk, kw = cfg
            G = N // 16 // (tnw * nw)
            grid = G * sk
            acc = {}
            for rep in range(6):
                st.zero_()
                rc = L.lsa_gemv_coop(x.data_ptr(), K, None, wps[rep % nbuf].data_ptr(), M, N, K, 0, 1e-5, epi,
                                     ctypes.byref(ep), tnw, nw, kf, sk, kw, ws.slab.data_ptr(), ws.counters.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream)
                assert rc == 0
                torch.cuda.synchronize()
                if rep < 2:
                    continue  # warm-up
                s = st.view(-1, 16)[:grid, :9].cpu().double()
                t0 = s[:, 0][s[:, 0] > 0].min()
                for k in range(9):
                    v = s[:, k]
                    v = v[v > 0]
                    if v.numel():
                        acc.setdefault(k, []).append(((v - t0) / 100.0))  # 100 MHz -> us
            print(f"{name} M={M} cfg={cfg} grid={grid}")
            for k in range(9):
                if k not in acc:
                    continue
                v = torch.cat(acc[k])
                print(f"   {NAMES[k]:9s} n={v.numel() // 4:5d}  median {v.median().item():7.2f}  p90 "
                      f"{v.quantile(0.9).item():7.2f}  max {v.max().item():7.2f} us")
        del wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
