#!/usr/bin/env python3
"""Launch one skinny_gemm / gemv_coop configuration 8 times (weights rotated beyond the Infinity
Cache) for rocprofv3 counter passes.  usage: skinny_pmc.py {skinny|coop|abl<n>} M N K cfg..."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip, packing  # noqa: E402

kind = sys.argv[1]
M, N, K = (int(v) for v in sys.argv[2:5])
cfg = tuple(int(v) for v in sys.argv[5:])
hip.lib()
ws = hip.CoopWorkspace("cuda", slab_floats=1 << 25)
nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
ep = hip.make_epi(out=out, ldo=N)
if kind.startswith("abl"):
    vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    L = ctypes.CDLL(os.path.join(ROOT, "llm_sharding_amd", "_native", f"liblsa_skinny_{kind}.so"))
    L.lsa_skinny.argtypes = [vp, i, vp, vp, i, i, i, i, f, i, ctypes.POINTER(hip.EpiArgs), i, i, i, i, vp,
                             ctypes.c_longlong, vp, i, vp]
for j in range(8):
    if kind == "skinny":
        hip.gemv(x, wps[j % nbuf], M, N, K, hip.EPI_STORE, ep, skinny=cfg, ws=ws)
    elif kind == "coop":
        hip.gemv(x, wps[j % nbuf], M, N, K, hip.EPI_STORE, ep, coop=cfg, ws=ws)
    else:
        rc = L.lsa_skinny(x.data_ptr(), K, None, wps[j % nbuf].data_ptr(), M, N, K, 0, 1e-5, hip.EPI_STORE,
                          ctypes.byref(ep), *cfg, ws.slab.data_ptr(), ws.slab.numel(), ws.counters.data_ptr(),
                          ws.counters.numel(), torch.cuda.current_stream().cuda_stream)
        assert rc == 0
torch.cuda.synchronize()
print("done", kind, M, N, K, cfg)
