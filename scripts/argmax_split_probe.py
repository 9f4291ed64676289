import torch, sys
sys.path.insert(0, "/root/repo")
from llm_sharding_amd.ops import hip, packing
torch.manual_seed(0)
M, N, K = 160, 32000, 4096
a = (torch.randn(M, K, device="cuda")).to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
ws = hip.SkWorkspace("cuda")
def keys_for(lo, hi):
    k = torch.zeros(M, dtype=torch.int64, device="cuda")
    hip.gemm_sk(a, packing.pack_b(w[lo:hi].contiguous()), M, hi - lo, K, hip.EPI_ARGMAX, hip.make_epi(keys=k, col_offset=lo), ws=ws)
    return k
print("plans", hip.gemm_sk_plan(M, 32000, K), hip.gemm_sk_plan(M, 16000, K))
full = keys_for(0, 32000)
h1, h2 = keys_for(0, 16000), keys_for(16000, 32000)
split = torch.maximum(h1, h2)
print("full==split:", bool((full == split).all()), int((full != split).sum()))
d = (full != split).nonzero().flatten()[:5]
for r in d.tolist():
    print(r, int(full[r] >> 32), int(split[r] >> 32), 0xFFFFFFFF - int(full[r] & 0xFFFFFFFF), 0xFFFFFFFF - int(split[r] & 0xFFFFFFFF))
