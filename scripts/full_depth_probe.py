#!/usr/bin/env python3
"""Error growth over depth on the HIP path vs the fp32 golden model (Llama-2-7B shapes, random
init): prefill hidden rel err after L layers, logits rel err and greedy agreement of the engine's
fused head vs the golden head applied to the engine's own hidden state."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.config import get_preset  # noqa: E402
from llm_sharding_amd.models.reference import ReferenceLlama  # noqa: E402
from llm_sharding_amd.runtime.engine import RandomSource, StageEngine  # noqa: E402

DEV = "cuda"


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm()).item()


def main():
    cfg = get_preset("llama2-7b")
    src = RandomSource(cfg, 21)
    layers = [src.layer(i, DEV, torch.bfloat16) for i in range(cfg.num_hidden_layers)]
    ref = ReferenceLlama(cfg, src.embedding(DEV, torch.bfloat16), layers, src.final_norm(DEV, torch.bfloat16),
                         src.lm_head(DEV, torch.bfloat16), max_pos=64)
    ref.cos, ref.sin = ref.cos.to(DEV), ref.sin.to(DEV)
    rows, P = 4, 16
    ids = torch.randint(3, cfg.vocab_size, (rows, P), generator=torch.Generator().manual_seed(rows)).to(DEV)
    h0 = ref.embed[ids]
    for L in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else '1,2,4,8,16,32').split(',')]:
        eng = StageEngine(cfg, 0, L, DEV, torch.bfloat16, has_embed=True, has_head=(L == 32), source=src,
                          max_slots=int(os.environ.get('FD_SLOTS', rows)), max_seq=64,
                          max_prefill_rows=int(os.environ.get('FD_PREFILL', 128)))
        sl, po = eng.prefill_rows(list(range(rows)), [P] * rows)
        h = eng.forward(eng.embed(ids.reshape(-1)), sl, po).reshape(rows, P, -1)
        ref.reset()
        hr = ref.forward_hidden(h0, 0, L)
        print(f"L={L:2d} hidden rel err {rel(h, hr):.3e}  |h| rms {hr.pow(2).mean().sqrt().item():.3e}", flush=True)
        if L == 32:
            lg_ref = ref.logits(hr[:, -1])
            lg_eh = ref.logits(h[:, -1].float())
            tok = eng.head(h.reshape(rows * P, -1), [r * P + P - 1 for r in range(rows)])
            print("logits rel err (golden head on engine hidden)", rel(lg_eh, lg_ref))
            print("golden argmax", lg_ref.argmax(-1).tolist(), "golden-head-on-engine-hidden argmax",
                  lg_eh.argmax(-1).tolist(), "engine head", tok.tolist())
            top = lg_ref.topk(3, -1)
            print("golden top3", top.values.tolist(), "max|lg|", lg_ref.abs().amax(-1).tolist())
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
