#!/usr/bin/env python3
"""Register-ring depth of the cooperative decode GEMV (csrc/kernels/gemv_coop.hip, template D):
configs instantiated at both d = 3 and d = 4 timed against each other on the 7B decode
projections at 32 / 64 / 128 rows, over the 8 best configs of the round-4 re-tune
(profiles/r4_decode_proj_sweep.jsonl, copied to coop_depth_cfgs.json). Weights rotate over
> 600 MB (HBM-cold), as in a decode step. One JSON line per (shape, rows).

(The d = 4 / 5 / 6 numbers in profiles/r4_coop_depth_probe.jsonl came from an earlier form of this
probe that rebuilt the whole kernel file at a fixed depth; they picked the d = 4 instantiations.)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    from llm_sharding_amd.ops import hip, packing
    from llm_sharding_amd.models.rope import rope_table
    from llm_sharding_amd.config import llama2_7b
    from scripts.bench_kernels import EPIS, MODEL_SHAPES, timeit
    # the 8 best coop configs per (shape, rows) of profiles/r4_decode_proj_sweep.jsonl
    with open(os.path.join(ROOT, "scripts", "probes", "coop_depth_cfgs.json")) as f:
        sweep = {(k.split(",")[0], int(k.split(",")[1])): [tuple(c) for c in v] for k, v in json.load(f).items()}
    dev = "cuda"
    cos, sin = rope_table(llama2_7b(), 1024, dev)
    cws = hip.CoopWorkspace(dev, slab_floats=1 << 25)
    for name in ("qkv", "o", "gate_up", "down"):
        N, K = MODEL_SHAPES["llama2-7b"][name]
        epi = EPIS[name]
        nbuf = max(2, (600 << 20) // (N * K * 2) + 1)
        ws = [packing.pack_b(torch.randn(N, K, device=dev).mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
        for M in (128, 64, 32):
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            out = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            q = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            kc = torch.zeros(M, 32, 1024, 128, dtype=torch.bfloat16, device=dev)
            slot = torch.arange(M, dtype=torch.int32, device=dev)
            pos = torch.full((M,), 100, dtype=torch.int32, device=dev)
            if epi == hip.EPI_QKV:
                ep = hip.make_epi(out=q, k_cache=kc, v_cache=kc, slot=slot, pos=pos, cos=cos, sin=sin, ldo=N,
                                  n_heads=32, n_kv=32, head_dim=128, t_max=1024)
            else:
                ep = hip.make_epi(out=out, resid=out, ldo=N, ldr=N)
            norm = epi in (hip.EPI_QKV, hip.EPI_SWIGLU)
            res = {"shape": name, "M": M}
            cands = packing.coop_candidates(N // 16, K, M, epi == hip.EPI_SWIGLU)
            for d in (3, 4):
                best = None
                for cfg in sweep.get((name, M), []):
                    c = packing.coop_norm(cfg)[:5] + (d,)
                    if c not in cands:
                        continue
                    us = timeit(lambda i: hip.gemv(x, ws[i % nbuf], M, N, K, epi, ep, norm=norm, coop=c, ws=cws))
                    if best is None or us < best[0]:
                        best = (round(us, 2), list(c))
                res[f"d{d}"] = best
            print(json.dumps(res), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
