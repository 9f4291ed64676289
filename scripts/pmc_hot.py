#!/usr/bin/env python3
"""Target program for rocprofv3 --pmc passes over the headline's hot kernels (plain launches,
5 each, distinct template instantiations so the kernel names separate them):
  * gemm_sk 7B qkv at M=512 (decode batch) and M=16384 (prompt prefill), plan configs, fused epilogue
  * flash prefill attention, one 2048-token sequence, 7B heads
  * split-KV decode attention, 512 rows x 150 keys, 7B heads
Summarise with scripts/pmc_hot_summary.py."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402

DEV = "cuda"


def main():
    torch.manual_seed(0)
    sk = hip.SkWorkspace(DEV)
    N, K = 12288, 4096
    w = packing.pack_b(torch.randn(N, K, device=DEV).mul_(0.02).to(torch.bfloat16))
    for M in (512, 16384):
        x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        epi = hip.EPI_STORE if M == 512 else hip.EPI_RESID
        ep = hip.make_epi(out=out, ldo=N) if epi == hip.EPI_STORE else hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
        for _ in range(5):
            hip.gemm_sk(x, w, M, N, K, epi, ep, ws=sk)
        torch.cuda.synchronize()
        del x, out
    nh = nkv = 32
    hd, S = 128, 2048
    kc = torch.randn(1, nkv, S, hd, device=DEV).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(S, nh * hd, device=DEV).to(torch.bfloat16)
    o = torch.zeros(S, nh * hd, dtype=torch.bfloat16, device=DEV)
    th = hip.build_prefill_tiles([0] * S, list(range(S)), tile_rows=hip.prefill_tile_rows(nh, nkv))
    td = th.to(DEV)
    for _ in range(5):
        hip.attn_prefill(q, kc, vc, td, nh, nkv, hd, o, tiles_host=th)
    torch.cuda.synchronize()
    rows, T, tmax = 512, 150, 192
    kcd = torch.randn(rows, nkv, tmax, hd, device=DEV).to(torch.bfloat16)
    vcd = torch.randn_like(kcd)
    qd = torch.randn(rows, nh * hd, device=DEV).to(torch.bfloat16)
    slot = torch.arange(rows, dtype=torch.int32, device=DEV)
    pos = torch.full((rows,), T - 1, dtype=torch.int32, device=DEV)
    po = torch.empty(rows * nh * 2 * hd, dtype=torch.float32, device=DEV)
    pl = torch.empty(rows * nh * 2, dtype=torch.float32, device=DEV)
    od = torch.zeros(rows, nh * hd, dtype=torch.bfloat16, device=DEV)
    cnt = torch.zeros(rows * nkv, dtype=torch.int32, device=DEV)
    for _ in range(5):
        hip.attn(qd, kcd, vcd, slot, pos, rows, nh, nkv, hd, 1, po, pl, od, counters=cnt)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
