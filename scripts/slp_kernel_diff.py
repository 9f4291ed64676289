#!/usr/bin/env python3
"""Which kernels of a decode step compute different bits when the kernel library is built WITH
SLP vectorisation (the round-1..4 flags, probe_bin/liblsa_kernels_slp.so from
``LSA_VARIANT_SLP=1 scripts/probes/build_kernels_variant.sh slp``) instead of the product build
(-fno-slp-vectorize)? VERDICT r5 item 3: the two builds gave different headline token digests.

Both libraries are loaded into ONE process (RTLD_LOCAL, ops/hip.load_library). One decode step of
a 2-layer Llama-2-7B stage (random init, random KV history of 140 tokens) runs eagerly through
the DecodeGraph body at 512 rows (the headline), 128 rows and 1 row. Every leaf kernel call is
intercepted: from one snapshot of every device buffer the step can write, the call runs with
library B (SLP), the buffers are restored, the call runs again with library A (product), and the
two results are compared bitwise - so each kernel sees IDENTICAL inputs in both builds and a
difference is that kernel's own. A kernel that differs is re-run twice more per build from the
same snapshot to tell a deterministic difference (operation order / FMA contraction) from a
nondeterministic one (a hazard read). The step then continues on A's results.

usage: python scripts/slp_kernel_diff.py [--slp probe_bin/liblsa_kernels_slp.so] [--out FILE]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from llm_sharding_amd.config import get_preset  # noqa: E402
from llm_sharding_amd.ops import hip  # noqa: E402
from llm_sharding_amd.runtime.engine import DecodeGraph, RandomSource, StageEngine  # noqa: E402

LEAVES = ("gemm", "gemm_sk", "gemm_wr", "gemv", "attn", "attn_prefill", "embed", "row_ss", "resid_rmsnorm_partials",
          "rmsnorm", "argmax_finalize", "pos_advance")


def tensors_of(obj, prefix, out):
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            out.append((prefix, obj))
    elif isinstance(obj, (list, tuple)):
        for i, v in enumerate(obj):
            tensors_of(v, f"{prefix}[{i}]", out)
    elif hasattr(obj, "__dict__") and type(obj).__module__.startswith("llm_sharding_amd.ops"):
        for k, v in vars(obj).items():
            tensors_of(v, f"{prefix}.{k}", out)


def summarize_args(args) -> list:
    return [a for a in args if isinstance(a, (int, float, str)) and not isinstance(a, bool)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--slp", default=os.path.join(ROOT, "probe_bin", "liblsa_kernels_slp.so"))
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "slp_kernel_diff.jsonl"))
    ap.add_argument("--rows", default="512,128,1")
    a = ap.parse_args()
    LA = hip.load_library(hip.KERNELS_SO)      # product: -fno-slp-vectorize
    LB = hip.load_library(a.slp)               # SLP build
    hip._lib = LA
    cfg = get_preset("llama2-7b")
    import dataclasses
    cfg = dataclasses.replace(cfg, num_hidden_layers=2)
    dev = torch.device("cuda", 0)
    T = 140
    eng = StageEngine(cfg, 0, 2, dev, torch.bfloat16, has_embed=True, has_head=True, source=RandomSource(cfg, 0),
                      max_slots=512, max_seq=192, max_prefill_rows=512)
    g = torch.Generator(device=dev).manual_seed(5)
    for kc in eng.k_cache + eng.v_cache:
        kc.copy_(torch.randn(kc.shape, generator=g, device=dev).to(kc.dtype))
    eng.seq_len = [T] * 512

    records = []
    depth = [0]
    ctx = {"rows": 0, "call": 0, "state": []}

    def snapshot():
        return [t.clone() for _, t in ctx["state"]]

    def restore(snap):
        for (_, t), s0 in zip(ctx["state"], snap):
            t.copy_(s0)

    def run(fn, L, args, kw):
        hip._lib = L
        try:
            r = fn(*args, **kw)
        finally:
            hip._lib = LA
        torch.cuda.synchronize()
        return r

    def wrap(name, fn):
        def w(*args, **kw):
            if depth[0]:
                return fn(*args, **kw)
            depth[0] += 1
            try:
                torch.cuda.synchronize()
                snap = snapshot()
                run(fn, LB, args, kw)
                out_b = [t.clone() for _, t in ctx["state"]]
                restore(snap)
                r = run(fn, LA, args, kw)
                diffs, written = {}, []
                for (nm, t), s0, b in zip(ctx["state"], snap, out_b):
                    if not torch.equal(t, s0) or not torch.equal(b, s0):
                        written.append(nm)
                    if not torch.equal(t, b):
                        if t.is_floating_point():
                            d = (t.float() - b.float()).abs()
                            rel = float(d.max() / t.float().abs().max().clamp_min(1e-30))
                            diffs[nm] = {"n_diff": int((t != b).sum()), "numel": t.numel(), "max_abs": float(d.max()),
                                         "max_rel_of_range": rel}
                        else:
                            diffs[nm] = {"n_diff": int((t != b).sum()), "numel": t.numel()}
                rec = {"rows": ctx["rows"], "call": ctx["call"], "fn": name, "args": summarize_args(args),
                       "epi": kw.get("epi"), "writes": written, "differs": diffs}
                if diffs:  # deterministic? two more runs per build from the same snapshot
                    a_res = [t.clone() for _, t in ctx["state"]]
                    det = {}
                    for tag, L, ref in (("A", LA, a_res), ("B", LB, out_b)):
                        same = True
                        for _ in range(2):
                            restore(snap)
                            run(fn, L, args, kw)
                            same &= all(torch.equal(t, x) for (_, t), x in zip(ctx["state"], ref))
                        det[tag] = same
                    rec["deterministic"] = det
                    restore(snap)
                    r = run(fn, LA, args, kw)
                records.append(rec)
                ctx["call"] += 1
                print(json.dumps(rec), flush=True)
                return r
            finally:
                depth[0] -= 1
        return w

    for n in LEAVES:
        setattr(hip, n, wrap(n, getattr(hip, n)))

    for rows in [int(x) for x in a.rows.split(",")]:
        dg = DecodeGraph(eng, rows, "full")
        dg.tokens.copy_(torch.randint(3, cfg.vocab_size, (rows,), generator=torch.Generator().manual_seed(rows))
                        .to(torch.int32))
        st = []
        tensors_of([getattr(eng, x) for x in StageEngine.SCRATCH_ATTRS if not isinstance(getattr(eng, x), int)],
                   "eng", st)
        tensors_of(eng.k_cache, "k_cache", st)
        tensors_of(eng.v_cache, "v_cache", st)
        for x in ("tokens", "keys", "pos", "h_in", "step_ctr"):
            tensors_of(getattr(dg, x), f"dg.{x}", st)
        names = {}
        for nm, t in st:  # dedupe by storage
            names.setdefault((t.data_ptr(), t.numel()), (nm, t))
        ctx.update(rows=rows, call=0, state=list(names.values()))
        dg._body()
        torch.cuda.synchronize()
        del dg
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        for r in records:
            f.write(json.dumps(r) + "\n")
    nd = [r for r in records if r["differs"]]
    print(f"[slp-diff] {len(records)} kernel calls, {len(nd)} differ: "
          f"{sorted({(r['rows'], r['fn'], tuple(r['args'][:4])) for r in nd})}", flush=True)


if __name__ == "__main__":
    main()
