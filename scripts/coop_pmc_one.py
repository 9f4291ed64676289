"""8 launches of the coop qkv M=128 configuration from a coop_phases.py timing build (PMC driver)."""
import ctypes, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip, packing  # noqa: E402
v = sys.argv[1]
vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
L = ctypes.CDLL(os.path.join(ROOT, "llm_sharding_amd", "_native", f"liblsa_coop_{v}.so"))
L.lsa_gemv_coop.argtypes = [vp, i, vp, vp, i, i, i, i, f, i, ctypes.POINTER(hip.EpiArgs), i, i, i, i, i, vp, vp, vp]
M, N, K = 128, 12288, 4096
ws = hip.CoopWorkspace("cuda", slab_floats=1 << 25)
nbuf = 6
wps = [packing.pack_b(torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
ep = hip.make_epi(out=out, ldo=N)
for j in range(8):
    assert L.lsa_gemv_coop(x.data_ptr(), K, None, wps[j % nbuf].data_ptr(), M, N, K, 0, 1e-5, hip.EPI_STORE,
                           ctypes.byref(ep), 1, 8, 2, 2, 1, ws.slab.data_ptr(), ws.counters.data_ptr(),
                           torch.cuda.current_stream().cuda_stream) == 0
torch.cuda.synchronize()
