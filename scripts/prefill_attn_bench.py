#!/usr/bin/env python3
"""Flash prefill attention roofline (attn_prefill.hip): one sequence of S tokens, causal, the
heads of Llama-2-7B (32/32) and Llama-2-70B (64/8), head_dim 128. FLOPs counted as
4 * nh * hd * (keys actually attended, S(S+1)/2). One JSON line per (model, S)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip  # noqa: E402

DEV = "cuda"


def main():
    for name, nh, nkv in (("llama2-7b", 32, 32), ("llama2-70b", 64, 8)):
        for S in (512, 2048, 4096, 8192):
            hd = 128
            kc = torch.randn(1, nkv, S, hd, device=DEV).to(torch.bfloat16)
            vc = torch.randn_like(kc)
            q = torch.randn(S, nh * hd, device=DEV).to(torch.bfloat16)
            out = torch.zeros(S, nh * hd, dtype=torch.bfloat16, device=DEV)
            th = hip.build_prefill_tiles([0] * S, list(range(S)), tile_rows=hip.prefill_tile_rows(nh, nkv, S))
            td = th.to(DEV)

            def run():
                hip.attn_prefill(q, kc, vc, td, nh, nkv, hd, out, tiles_host=th)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            n = 10
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(n):
                run()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1e3 / n
            fl = 4.0 * nh * hd * S * (S + 1) / 2
            print(json.dumps({"model": name, "S": S, "n_heads": nh, "n_kv": nkv, "us": round(us, 1),
                              "tflops": round(fl / us / 1e6, 1), "tiles": int(th.shape[0])}), flush=True)
            del kc, vc, q, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
