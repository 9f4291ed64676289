"""Launch the tuned coop GEMV at M=64 on qkv / o / down / gate_up shapes (8 launches each,
rotating weights beyond the Infinity Cache) for PMC collection under rocprofv3."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing
hip.lib()
M = int(os.environ.get("M", 64))
ws_ = hip.CoopWorkspace("cuda", slab_floats=1 << 24)
for name, (N, K, epi) in {"qkv": (12288, 4096, hip.EPI_STORE), "o": (4096, 4096, hip.EPI_RESID),
                          "down": (4096, 11008, hip.EPI_RESID), "gate_up": (22016, 4096, hip.EPI_SWIGLU)}.items():
    nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
    ws = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    out = torch.zeros(M, max(N, 1), dtype=torch.bfloat16, device="cuda")
    ep = hip.make_epi(out=out, resid=out, ldo=out.shape[1], ldr=out.shape[1])
    algo, cfg = packing.proj_config(N // 16, M, need_even=epi == hip.EPI_SWIGLU, k=K)
    print(name, algo, cfg, flush=True)
    for i in range(8):
        hip.gemv(x, ws[i % nbuf], M, N, K, epi, ep, ws=ws_)
    torch.cuda.synchronize()
    del ws
