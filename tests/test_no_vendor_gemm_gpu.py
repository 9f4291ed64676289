"""Guard: the GPU engine never calls a vendor GEMM (torch.matmul / F.linear / addmm / bmm ->
hipBLASLt / rocBLAS) - every projection, the attention and the lm_head run on the hand-written
HIP kernels (profiles/r2_bench_decode_kernels.txt shows no Cijk kernels; this pins it in a test).
Prefill at 130 / 600 rows (coop GEMV / gemm_sk + flash prefill) and hipGraph decode at 1 / 64 /
200 rows (GEMV, coop, gemm_sk) run with those torch entry points patched to raise."""
from unittest import mock

import pytest
import torch
import torch.nn.functional as F

from llm_sharding_amd.config import LlamaConfig
from llm_sharding_amd.runtime.engine import DecodeGraph, RandomSource, StageEngine

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _forbidden(*a, **k):
    raise AssertionError("vendor GEMM called on the GPU engine path")


@pytest.mark.parametrize("prompt_rows,decode_rows", [(130, 1), (600, 64), (600, 200)])
def test_engine_uses_no_vendor_gemm(prompt_rows, decode_rows):
    cfg = LlamaConfig(num_hidden_layers=2, vocab_size=4096, max_position_embeddings=1024, name="7b-2L")
    eng = StageEngine(cfg, 0, 2, DEV, torch.bfloat16, has_embed=True, has_head=True, source=RandomSource(cfg, 3),
                      max_slots=decode_rows, max_seq=256, max_prefill_rows=max(prompt_rows, decode_rows))
    P = max(1, prompt_rows // decode_rows)
    slots = list(range(decode_rows))
    ids = torch.randint(3, cfg.vocab_size, (decode_rows * P,), device=DEV)
    with mock.patch.object(torch, "matmul", _forbidden), mock.patch.object(F, "linear", _forbidden), \
            mock.patch.object(torch, "addmm", _forbidden), mock.patch.object(torch, "bmm", _forbidden), \
            mock.patch.object(torch.Tensor, "__matmul__", _forbidden):
        sl, po = eng.prefill_rows(slots, [P] * decode_rows)
        h = eng.forward(eng.embed(ids), sl, po)
        eng.advance(slots, [P] * decode_rows)
        first = eng.head(h, [r * P + P - 1 for r in range(decode_rows)])
        dg = DecodeGraph(eng, decode_rows, "full", history_len=2)
        dg.tokens.copy_(first.to(torch.int32))
        dg.capture()
        dg.replay()
        dg.replay()
        torch.cuda.synchronize()
    toks = dg.history.cpu()
    assert bool(((toks >= 0) & (toks < cfg.vocab_size)).all())
