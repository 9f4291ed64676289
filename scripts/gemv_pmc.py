"""Launch the o_proj-shaped decode GEMV at M=1/16/32/64 (tuned configs) for PMC collection."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing
hip.lib()
N, K = int(os.environ.get("N", 4096)), int(os.environ.get("K", 4096))
ws = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(8)]
for M in (1, 16, 32, 64):
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
    ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
    for i in range(6):
        hip.gemv(x, ws[i % 8], M, N, K, hip.EPI_RESID, ep)
torch.cuda.synchronize()
