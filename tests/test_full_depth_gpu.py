"""Full-depth Llama-2-7B on the HIP path against the fp32 golden model.

Every other engine test cuts the model to 2 layers; here all 32 layers and the 32000-row lm_head
run, so error growth over depth and over many decode steps is pinned:

* a 4-sequence prompt prefill (64 rows: the fused GEMV / cooperative kernels) and 24
  teacher-forced hipGraph decode steps (batch 4), final hidden state of every step vs golden;
* a 160-sequence prefill (800 rows: gemm_sk stream-K GEMMs + flash prefill attention) and 8
  teacher-forced decode steps at 160 rows (gemm_sk with fused epilogues inside the graph).

Weights are random-init of the 7B architecture, drawn on the GPU with the same seeded generator
for the engine (RandomSource) and the golden model, so both see identical values. Teacher forcing
(feeding the golden model's greedy token) keeps a near-tie argmax from making the two runs diverge;
every engine token must be near-optimal under the golden logits, within a bound derived from the measured hidden-state error (_check_tokens).
Reference behaviour: the HF decoder stack run layer by layer in /root/reference/utils/shard_loader.py:57-74.

Regression tripwire (tests/fixtures/full_depth_7b.json, recorded on this tree with
``LSA_RECORD_FULL_DEPTH=1``; tests/test_fixture_fresh.py fails the CPU suite when the kernels or
routing changed since the recording):
* each decode step's hidden rel err vs golden <= 1.25 x the recorded value of that step;
* greedy tokens identical to golden >= 80 % (a logged floor beside the derived bound);
* a fingerprint of the engine's own hidden states (8 fixed random projections per row and step)
  equal to the recording within 1e-3 - the kernels are deterministic, so this is bitwise on an
  unchanged tree, and a 1 % perturbation of ONE layer's output (far below what the golden
  comparison can resolve against 3.4e-2 of bf16 noise) trips it:
  test_full_depth_tripwire_catches_one_layer_perturbation.
"""
import json
import math
import os
import subprocess

import pytest
import torch

from llm_sharding_amd.config import get_preset
from llm_sharding_amd.models.reference import ReferenceLlama
from llm_sharding_amd.runtime.engine import DecodeGraph, RandomSource, StageEngine

pytestmark = pytest.mark.gpu
DEV = "cuda"
SEED = 21


FIXTURE = os.environ.get("LSA_FULL_DEPTH_FIXTURE") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures",
                                                                  "full_depth_7b.json")
RECORD = os.environ.get("LSA_RECORD_FULL_DEPTH") == "1"
STEP_FACTOR = 1.25    # per-step hidden rel err vs the recorded value
MATCH_FLOOR = 0.80    # greedy tokens identical to golden
FP_TOL = 1e-3         # engine fingerprint vs the recording (0 on an unchanged tree)


def rel_err(a, b):
    a, b = a.float(), b.float().to(a.device)
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _fingerprint(h):
    """[rows, H] -> [rows, 8]: fixed random projections of the engine's hidden states."""
    H = h.shape[-1]
    R = torch.randn(H, 8, generator=torch.Generator().manual_seed(1234)).to(h.device)
    return (h.float().reshape(-1, H) @ R / math.sqrt(H)).cpu()


def _load_fixture():
    if not os.path.exists(FIXTURE):
        return {}
    with open(FIXTURE) as fh:
        return json.load(fh)


def _record(key, res):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    from fixture_hash import tree_hash  # tests/fixture_hash.py
    fx = _load_fixture()
    fx[key] = dict(res)
    fx["kernel_hash"] = tree_hash(root)
    try:
        fx["commit"] = subprocess.run(["git", "-C", root, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                      text=True).stdout.strip() or "unknown"
    except OSError:
        fx["commit"] = "unknown"
    os.makedirs(os.path.dirname(FIXTURE), exist_ok=True)
    with open(FIXTURE, "w") as fh:
        json.dump(fx, fh, indent=1)


def _tripwire(key, res):
    """Compare a run against the recorded one (or record it)."""
    if RECORD:
        _record(key, res)
        return
    fx = _load_fixture().get(key)
    assert fx, f"no recorded run {key!r} in {FIXTURE}: record with LSA_RECORD_FULL_DEPTH=1 on the GPU box"
    bad = [(i, e, r) for i, (e, r) in enumerate(zip(res["steps"], fx["steps"])) if e > STEP_FACTOR * r + 1e-5]
    assert not bad, f"{key}: decode hidden rel err above {STEP_FACTOR} x the recording at steps {bad}"
    rate = res["match"] / res["tokens"]
    assert rate >= MATCH_FLOOR, f"{key}: only {res['match']}/{res['tokens']} greedy tokens identical to golden"
    fp_now, fp_rec = torch.tensor(res["fingerprint"]), torch.tensor(fx["fingerprint"])
    d = ((fp_now - fp_rec).norm() / fp_rec.norm()).item()
    print(f"[full-depth] {key}: fingerprint vs recording ({fx.get('commit', '?')}) rel {d:.2e}, exact match "
          f"{rate:.1%} (recorded {fx['match'] / fx['tokens']:.1%})")
    assert d <= FP_TOL, f"{key}: engine hidden-state fingerprint moved {d:.3e} from the recording (> {FP_TOL:g})"


@pytest.fixture(scope="module")
def model():
    cfg = get_preset("llama2-7b")
    src = RandomSource(cfg, SEED)
    eng = StageEngine(cfg, 0, cfg.num_hidden_layers, DEV, torch.bfloat16, has_embed=True, has_head=True,
                      source=src, max_slots=160, max_seq=64, max_prefill_rows=800)
    # the golden model: the same draws (same device, same seeds), kept in fp32 on the GPU
    ref = ReferenceLlama(cfg, src.embedding(DEV, torch.bfloat16),
                         [src.layer(i, DEV, torch.bfloat16) for i in range(cfg.num_hidden_layers)],
                         src.final_norm(DEV, torch.bfloat16), src.lm_head(DEV, torch.bfloat16), max_pos=64)
    ref.cos, ref.sin = ref.cos.to(DEV), ref.sin.to(DEV)
    yield cfg, eng, ref
    del eng, ref
    torch.cuda.empty_cache()


def _check_tokens(lg, got, le, slack=0.01):
    """The engine's greedy token ``got`` against the golden logits ``lg``, with a bound DERIVED
    from the measured hidden-state error instead of a constant: ``le`` = the golden fp32 head
    applied to the ENGINE's final hidden state. For the golden argmax m and the engine's choice c
    (which its own logits l' rank first: l'[c] >= l'[m]),
        lg[m] - lg[c] <= (lg[m] - le[m]) + (le[c] - lg[c]) + (le[m] - l'[m]) + (l'[c] - le[c]);
    the first two terms are measured here, the last two are the engine head's own error on the
    same hidden state (bf16-folded norm weight, bf16 inputs, fp32 accumulation): bounded by
    ``slack`` x max|lg| (0.01; the head kernel alone is within 8e-3 rel of fp32 in
    tests/test_kernels_gpu.py). A wrong in-graph argmax shows as a gap beyond that bound however
    small the hidden-state error is; the hidden-state error itself is asserted by the caller.
    Returns (exact matches, rows)."""
    got = got.to(lg.device).long()
    m = lg.argmax(-1)
    lg_c, lg_m = lg.gather(1, got[:, None])[:, 0], lg.gather(1, m[:, None])[:, 0]
    le_c, le_m = le.gather(1, got[:, None])[:, 0], le.gather(1, m[:, None])[:, 0]
    scale = lg.abs().amax(-1)
    gap = lg_m - lg_c
    bound = (lg_m - le_m) + (le_c - lg_c) + slack * scale
    assert bool((gap <= bound + 1e-6).all()), (
        f"token gaps {(gap / scale).tolist()} exceed the derived bound {(bound / scale).tolist()} (x max|logit|): "
        f"engine {got.tolist()} golden {m.tolist()}")
    return int((got == m).sum()), got.numel()


def _run(cfg, eng, ref, rows, prompt, steps, tol_prefill, tol_step):
    eng.reset()
    ref.reset()
    slots = list(range(rows))
    ids = torch.randint(3, cfg.vocab_size, (rows, prompt), generator=torch.Generator().manual_seed(rows))
    sl, po = eng.prefill_rows(slots, [prompt] * rows)
    h = eng.forward(eng.embed(ids.reshape(-1).to(DEV)), sl, po)
    eng.advance(slots, [prompt] * rows)
    href = ref.forward_hidden(ref.embed[ids.to(DEV)])
    e0 = rel_err(h.reshape(rows, prompt, -1), href)
    print(f"[full-depth] rows {rows}: prefill rel err {e0:.2e}")
    assert e0 < tol_prefill, f"prefill rel err {e0:.3e}"
    lg = ref.logits(href[:, -1])
    first = eng.head(h, [r * prompt + prompt - 1 for r in range(rows)])
    m, n = _check_tokens(lg, first, ref.logits(h.reshape(rows, prompt, -1)[:, -1].float()))
    dg = DecodeGraph(eng, rows, "full")
    dg.capture()
    errs, fps = [], [_fingerprint(h.reshape(rows, prompt, -1)[:, -1])]
    for _ in range(steps):
        tok = lg.argmax(-1)  # teacher forcing: the golden model's greedy token
        dg.tokens.copy_(tok.to(torch.int32))
        dg.replay()
        torch.cuda.synchronize()
        href = ref.forward_hidden(ref.embed[tok[:, None]])[:, -1]
        errs.append(rel_err(dg.out_hidden, href))
        fps.append(_fingerprint(dg.out_hidden))
        lg = ref.logits(href)
        # the step's argmax, written in-graph
        mi, ni = _check_tokens(lg, dg.tokens, ref.logits(dg.out_hidden.float().to(href.device)))
        m, n = m + mi, n + ni
    print(f"[full-depth] rows {rows}: prefill rel err {e0:.2e}, decode max {max(errs):.2e} "
          f"last {errs[-1]:.2e}, greedy tokens identical to golden {m}/{n}")
    assert max(errs) < tol_step, f"decode rel errs {['%.2e' % e for e in errs]}"
    # every token that differs from the golden argmax was checked above against the bound derived
    # from the measured hidden-state error; the exact-match rate is kept as a logged floor
    # (_tripwire) and the per-step errors against the recording of this tree
    return {"prefill": e0, "steps": errs, "match": m, "tokens": n,
            "fingerprint": torch.stack(fps).tolist()}


SMALL = dict(rows=4, prompt=16, steps=24, tol_prefill=4e-2, tol_step=5e-2)
BIG = dict(rows=160, prompt=5, steps=8, tol_prefill=4e-2, tol_step=5e-2)


def test_full_depth_7b_small_batch(model):
    cfg, eng, ref = model
    _tripwire("small_batch", _run(cfg, eng, ref, **SMALL))


def test_full_depth_7b_big_batch(model):
    cfg, eng, ref = model
    _tripwire("big_batch", _run(cfg, eng, ref, **BIG))


def test_full_depth_tripwire_catches_one_layer_perturbation(model):
    """Negative control: layer 7's down projection scaled by 1 + 1e-2 in the engine only (the
    golden model is untouched). The golden comparison cannot resolve it (bf16 noise is 3.4e-2 at
    full depth); the tripwire must."""
    if RECORD:
        pytest.skip("recording")
    cfg, eng, ref = model
    lw = eng.layers[7]
    saved = lw.down.clone()
    lw.down.mul_(1.0 + 1e-2)
    try:
        res = _run(cfg, eng, ref, **SMALL)
        with pytest.raises(AssertionError, match="fingerprint moved"):
            _tripwire("small_batch", res)
    finally:
        lw.down.copy_(saved)
