#!/usr/bin/env python3
"""GQA decode attention: MFMA kernel (lsa_attn_decode_mfma, 2 or 4 waves per item) vs the split-KV
VALU kernel at Llama-2-70B heads (64 / 8) and Llama-3.2-3B heads (24 / 8), hd 128, 512 rows,
contexts 150 / 1024 / 4096 keys; hipGraph-timed, KV rotated over 3 copies. One JSON line per
(heads, T, kernel) with the K/V stream rate."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip  # noqa: E402
from scripts.bench_kernels import timeit  # noqa: E402

DEV = "cuda"


def main():
    hd = 128
    for nh, nkv, rows, T in ((64, 8, 512, 150), (64, 8, 512, 1024), (64, 8, 128, 4096), (24, 8, 512, 150),
                             (24, 8, 512, 1024)):
        tmax = -(-(T + 1) // 64) * 64
        kcs = [torch.randn(rows, nkv, tmax, hd, device=DEV).to(torch.bfloat16) for _ in range(3)]
        vcs = [torch.randn_like(k) for k in kcs]
        q = torch.randn(rows, nh * hd, device=DEV).to(torch.bfloat16)
        slot = torch.arange(rows, dtype=torch.int32, device=DEV)
        pos = torch.full((rows,), T - 1, dtype=torch.int32, device=DEV)
        out = torch.zeros(rows, nh * hd, dtype=torch.bfloat16, device=DEV)
        ns = max(1, min(8, 512 // (rows * nkv) if rows * nkv < 512 else 1, T // 256))
        po = torch.empty(rows * nh * 8 * hd, device=DEV)
        pl = torch.empty(rows * nh * 8, device=DEV)
        cnt = torch.zeros(rows * nkv, dtype=torch.int32, device=DEV)
        nbytes = rows * nkv * T * hd * 2 * 2
        for name, mf, nw in (("mfma_nw4", True, 4), ("mfma_nw2", True, 2), ("mfma_nw1", True, 1),
                             ("split_valu", False, 0)):
            hip.ATTN_MFMA, hip.ATTN_GQA_NW = mf, nw
            us = timeit(lambda i: hip.attn(q, kcs[i % 3], vcs[i % 3], slot, pos, rows, nh, nkv, hd, ns, po, pl, out,
                                           counters=cnt))
            print(json.dumps({"heads": [nh, nkv], "rows": rows, "T": T, "kernel": name, "nsplit": ns if not mf else 1,
                              "us": round(us, 2), "kv_TBps": round(nbytes / us / 1e6, 3)}), flush=True)
        hip.ATTN_MFMA, hip.ATTN_GQA_NW = True, 0
        del kcs, vcs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
