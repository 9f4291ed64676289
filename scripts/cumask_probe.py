#!/usr/bin/env python3
"""Can memory-bound decode attention and compute-bound projection GEMMs share the chip? (VERDICT
r2 item 2.) Streams created with hipExtStreamCreateWithCUMask (CUs spread evenly over the
mask); at the headline decode shape (Llama-2-7B, 512 rows, ~150 keys):
  * attention alone on C CUs -> KV TB/s vs C;
  * the qkv / gate_up GEMM alone on 256 - C CUs (grid = 256 - C);
  * both concurrently on complementary masks vs back to back on the full chip.
One JSON line per measurement."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_amd.ops import hip, packing  # noqa: E402

DEV = "cuda"
N_CU = 256
_RAW = []  # every CU-masked stream this process created: destroyed before exit (destroy_streams)


def masked_stream(cus):
    lib = ctypes.CDLL("libamdhip64.so")
    words = (ctypes.c_uint32 * 8)()
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = lib.hipExtStreamCreateWithCUMask(ctypes.byref(s), 8, words)
    assert rc == 0, rc
    _RAW.append(s.value)
    return torch.cuda.ExternalStream(s.value)


def destroy_streams():
    """The streams were created outside torch (ExternalStream does not own them): left alive,
    the HIP runtime's process-exit teardown raced the profiler's and crashed (SIGSEGV after the
    last output line under rocprofv3, profiles/r4_attn_gemm_overlap.md). Drain, then destroy."""
    lib = ctypes.CDLL("libamdhip64.so")
    torch.cuda.synchronize()
    while _RAW:
        rc = lib.hipStreamDestroy(ctypes.c_void_p(_RAW.pop()))
        assert rc == 0, rc


def spread(n, offset=0):
    step = N_CU / n
    return sorted({int(offset + i * step) % N_CU for i in range(n)})


def time_on(stream, fn, iters=20):
    with torch.cuda.stream(stream):
        for i in range(3):
            fn(i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(iters):
            fn(i)
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    rows, nh, hd, T = 512, 32, 128, 150
    tmax = 192
    kcs = [torch.randn(rows, nh, tmax, hd, device=DEV).to(torch.bfloat16) for _ in range(2)]
    vcs = [torch.randn_like(k) for k in kcs]
    q = torch.randn(rows, nh * hd, device=DEV).to(torch.bfloat16)
    slot = torch.arange(rows, dtype=torch.int32, device=DEV)
    pos = torch.full((rows,), T - 1, dtype=torch.int32, device=DEV)
    out = torch.zeros(rows, nh * hd, dtype=torch.bfloat16, device=DEV)
    po = torch.empty(rows * nh * 2 * hd, device=DEV)
    pl = torch.empty(rows * nh * 2, device=DEV)
    cnt = torch.zeros(rows * nh, dtype=torch.int32, device=DEV)
    kv_bytes = rows * nh * T * hd * 2 * 2

    def attn(i):
        hip.attn(q, kcs[i % 2], vcs[i % 2], slot, pos, rows, nh, nh, hd, 1, po, pl, out, counters=cnt)

    K = 4096
    shapes = {"qkv": 12288, "gate_up": 22016}
    ws = {k: [packing.pack_b(torch.randn(n, K, device=DEV).mul_(0.02).to(torch.bfloat16)) for _ in range(3)]
          for k, n in shapes.items()}
    x = torch.randn(rows, K, device=DEV).to(torch.bfloat16)
    outs = {k: torch.empty(rows, n, dtype=torch.bfloat16, device=DEV) for k, n in shapes.items()}
    sk_ws = hip.SkWorkspace(DEV)

    def gemm(name, grid):
        N = shapes[name]
        ep = hip.make_epi(out=outs[name], ldo=N)
        bn, _, dp, split, bm = hip.gemm_sk_plan(rows, N, K)

        def run(i):
            hip.gemm_sk(x, ws[name][i % 3], rows, N, K, hip.EPI_STORE, ep, bn=bn, grid=grid, dp=dp, split=split, bm=bm,
                        ws=sk_ws)
        return run

    full = masked_stream(range(N_CU))
    if os.environ.get("CUMASK_TRACE"):
        # concurrent configurations for a kernel trace: do the two streams' kernels overlap in
        # time, and how fast does each run beside the other? (attention on C spread CUs, qkv on
        # the rest; one round per C, 4 attention + 12 GEMM launches)
        for C in [int(c) for c in os.environ["CUMASK_TRACE"].split(",")]:
            att_cus = spread(C)
            gem_cus = [c for c in range(N_CU) if c not in set(att_cus)]
            sa, sg = masked_stream(att_cus), masked_stream(gem_cus)
            sa_alone = time_on(sa, attn)
            g = gemm("qkv", len(gem_cus))
            print(json.dumps({"what": "alone", "attn_cus": C, "attn_us": round(sa_alone, 2),
                              "attn_TBps": round(kv_bytes / sa_alone / 1e6, 3),
                              "gemm_us": round(time_on(sg, g), 2)}), flush=True)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            cur = torch.cuda.current_stream()
            e0.record(cur)
            sa.wait_stream(cur)
            sg.wait_stream(cur)
            with torch.cuda.stream(sa):
                for i in range(4):
                    attn(i)
            with torch.cuda.stream(sg):
                for i in range(12):
                    g(i)
            cur.wait_stream(sa)
            cur.wait_stream(sg)
            e1.record(cur)
            torch.cuda.synchronize()
            print(json.dumps({"what": "trace", "attn_cus": C, "total_us": round(e0.elapsed_time(e1) * 1e3, 1)}),
                  flush=True)
        return
    t_attn_full = time_on(full, attn)
    print(json.dumps({"what": "attn", "cus": N_CU, "us": round(t_attn_full, 2),
                      "TBps": round(kv_bytes / t_attn_full / 1e6, 3)}), flush=True)
    for C in (32, 64, 96, 128, 160, 192):
        s = masked_stream(spread(C))
        t = time_on(s, attn)
        print(json.dumps({"what": "attn", "cus": C, "us": round(t, 2), "TBps": round(kv_bytes / t / 1e6, 3)}), flush=True)
    for name in shapes:
        tg_full = time_on(full, gemm(name, N_CU))
        print(json.dumps({"what": name, "cus": N_CU, "us": round(tg_full, 2)}), flush=True)
        for C in (64, 96, 128):
            att_cus = spread(C)
            gem_cus = [c for c in range(N_CU) if c not in set(att_cus)]
            sa, sg = masked_stream(att_cus), masked_stream(gem_cus)
            g = gemm(name, len(gem_cus))
            tg = time_on(sg, g)
            # concurrent: both streams launched back to back, timed from a common start
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            cur = torch.cuda.current_stream()
            e0.record(cur)
            sa.wait_stream(cur)
            sg.wait_stream(cur)
            iters = 10
            with torch.cuda.stream(sa):
                for i in range(iters):
                    attn(i)
            with torch.cuda.stream(sg):
                for i in range(iters):
                    g(i)
            cur.wait_stream(sa)
            cur.wait_stream(sg)
            e1.record(cur)
            torch.cuda.synchronize()
            tc = e0.elapsed_time(e1) * 1e3 / iters
            print(json.dumps({"what": f"{name}+attn", "attn_cus": C, "gemm_cus": len(gem_cus),
                              "gemm_alone_us": round(tg, 2), "concurrent_us": round(tc, 2),
                              "serial_full_chip_us": round(tg_full + t_attn_full, 2)}), flush=True)


if __name__ == "__main__":
    try:
        main()
    finally:
        destroy_streams()
