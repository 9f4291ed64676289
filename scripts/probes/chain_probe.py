#!/usr/bin/env python3
"""Driver of the persistent-chain probe (scripts/probes/chain_probe.hip; build with
scripts/probes/build_chain_probe.sh): the weight-streaming chain of a Llama-2-7B layer at batch 1
(qkv 12288x4096 -> o 4096x4096 -> gate_up 22016x4096 -> down 4096x11008, each op's input = the
previous op's output prefix) as ONE persistent launch (run-ahead LDS-DMA loader + granule
hand-offs) vs the library's tuned decode GEMV launched once per op (eager and hipGraph-replayed).
Checks the chain's output against an fp32 torch reference with the same bf16 rounding between
ops, then times both. One JSON line."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from llm_sharding_amd.ops import hip, packing  # noqa: E402

SO = os.path.join(ROOT, "build", "probes", "libchain_probe.so")
SHAPES = [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008)]
DEV = "cuda"


def main():
    L = ctypes.CDLL(SO)
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    L.lsa_chain_probe.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(i32), ctypes.POINTER(i32), vp,
                                  ctypes.POINTER(vp), vp, ctypes.c_uint, i32, vp]
    L.lsa_chain_probe.restype = i32
    hip.lib()
    torch.manual_seed(0)
    W = [(torch.randn(n, k, device=DEV) * (1.0 / k ** 0.5)).to(torch.bfloat16) for n, k in SHAPES]
    Wp = [packing.pack_b(w) for w in W]
    x0 = torch.randn(SHAPES[0][1], device=DEV).to(torch.bfloat16)
    gran = [torch.zeros(n // 2, dtype=torch.int64, device=DEV) for n, _ in SHAPES]
    err = torch.zeros(3, dtype=torch.int32, device=DEV)
    wa = (vp * 4)(*[w.data_ptr() for w in W])
    na = (i32 * 4)(*[n for n, _ in SHAPES])
    ka = (i32 * 4)(*[k for _, k in SHAPES])
    ga = (vp * 4)(*[g.data_ptr() for g in gran])

    def persistent(epoch, check=0):
        rc = L.lsa_chain_probe(wa, na, ka, x0.data_ptr(), ga, err.data_ptr(), epoch, check,
                               torch.cuda.current_stream().cuda_stream)
        if rc != 0:
            raise RuntimeError(f"lsa_chain_probe rc {rc}")

    # correctness (epoch 1) against fp32 with bf16 rounding between ops
    persistent(1, check=1)
    torch.cuda.synchronize()
    e = int(err[0].item())
    mism = [int(err[1].item()), int(err[2].item())]

    def decoded(p):
        return gran[p].view(torch.int32).view(-1, 2)[:, 0].contiguous().view(torch.bfloat16).float()

    # per op: the kernel's output against fp32 of the kernel's OWN input (isolates each stage)
    per_op, x = [], x0.float()
    for p, (w, (n, k)) in enumerate(zip(W, SHAPES)):
        ref = w.float() @ x[:k]
        got = decoded(p)
        per_op.append(round(float((got - ref).norm() / ref.norm()), 5))
        x = got
    tags_ok = all(bool((gran[p].view(torch.int32).view(-1, 2)[:, 1] == 1 * 4 + p + 1).all()) for p in range(4))
    rel = max(per_op)
    if e or not tags_ok or not rel < 2e-2:
        print(json.dumps({"failed": True, "err_flags": e, "staged_w_x_mismatch_lanes": mism, "tags_ok": tags_ok,
                          "rel_err_per_op": per_op,
                          "op0_first": decoded(0)[:4].tolist(), "op0_ref": (W[0].float() @ x0.float())[:4].tolist()}),
              flush=True)
        raise SystemExit(9)

    # y buffers of the launch-per-op baseline
    ys = [torch.zeros(1, n, dtype=torch.bfloat16, device=DEV) for n, _ in SHAPES]

    def launches():
        inp = x0.view(1, -1)
        for p, (n, k) in enumerate(SHAPES):
            hip.gemv(inp, Wp[p], 1, n, k, hip.EPI_STORE, hip.make_epi(out=ys[p], ldo=n))
            inp = ys[p]

    reps = 200
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for ep in range(2, 12):
        persistent(ep)
    torch.cuda.synchronize()
    ev0.record()
    for ep in range(12, 12 + reps):
        persistent(ep)
    ev1.record()
    torch.cuda.synchronize()
    t_persist = ev0.elapsed_time(ev1) * 1e3 / reps
    e |= int(err[0].item())

    for _ in range(10):
        launches()
    torch.cuda.synchronize()
    ev0.record()
    for _ in range(reps):
        launches()
    ev1.record()
    torch.cuda.synchronize()
    t_eager = ev0.elapsed_time(ev1) * 1e3 / reps

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        launches()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(20):
            launches()
    g.replay()
    torch.cuda.synchronize()
    ev0.record()
    for _ in range(10):
        g.replay()
    ev1.record()
    torch.cuda.synchronize()
    t_graph = ev0.elapsed_time(ev1) * 1e3 / 200

    wbytes = sum(n * k * 2 for n, k in SHAPES)
    print(json.dumps({"chain": "7B qkv -> o -> gate_up -> down, batch 1", "weight_MB": round(wbytes / 1e6, 1),
                      "persistent_us": round(t_persist, 2), "launches_eager_us": round(t_eager, 2),
                      "launches_graph_us": round(t_graph, 2),
                      "persistent_TBps": round(wbytes / t_persist / 1e6, 2),
                      "launches_graph_TBps": round(wbytes / t_graph / 1e6, 2),
                      "rel_err_per_op_max": round(rel, 5), "tags_ok": tags_ok, "err_flags": e}), flush=True)


if __name__ == "__main__":
    main()
