#!/usr/bin/env python3
"""Where a persistent batch-1 decode step (decode_persistent.hip) spends layer 1: per-workgroup
s_memrealtime stamps (100 MHz) from the diagnostic build (-DLSA_PERSIST_STAMPS ->
_native/liblsa_persist_stamps.so, `python scripts/persist_stamps.py --build` on the CPU host).
Prints, per phase, the median / max over workgroups of start and done times (us from the
layer's first stamp) and the barrier exits. usage: persist_stamps.py [--build] [model]"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "llm_sharding_amd", "_native", "liblsa_persist_stamps.so")


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                           "-DLSA_PERSIST_STAMPS", "-I", os.path.join(ROOT, "csrc", "kernels"),
                           os.path.join(ROOT, "csrc", "kernels", "decode_persistent.hip"), "-o", SO])
    print("built", SO)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--build":
        build()
        return
    import torch
    sys.path.insert(0, ROOT)
    from llm_sharding_amd.config import get_preset
    from llm_sharding_amd.ops import hip
    from llm_sharding_amd.runtime.engine import DecodeGraph, RandomSource, StageEngine
    cfg = get_preset(sys.argv[1] if len(sys.argv) > 1 else "llama2-7b")
    eng = StageEngine(cfg, 0, cfg.num_hidden_layers, "cuda", torch.bfloat16, has_embed=True, has_head=True,
                      source=RandomSource(cfg, 0), max_slots=1, max_seq=256)
    eng.seq_len[0] = 128
    g = DecodeGraph(eng, 1, "full", slots=[0], persistent=True)
    L = ctypes.CDLL(SO)
    real = hip.lib()
    fn = L.lsa_decode_persistent
    fn.argtypes, fn.restype = real.lsa_decode_persistent.argtypes, ctypes.c_int
    st = torch.zeros(hip.N_CU * 16, dtype=torch.int64, device="cuda")
    L.lsa_persist_set_stamps(ctypes.c_void_p(st.data_ptr()))

    class Shim:  # hip.decode_persistent with the diagnostic library
        def __getattr__(self, k):
            return fn if k == "lsa_decode_persistent" else getattr(real, k)
    orig = hip.lib
    hip.lib = lambda: Shim()
    try:
        rows = []
        for r in range(6):
            st.zero_()
            g._body()
            torch.cuda.synchronize()
            assert int(g.err.item()) == 0
            if r >= 2:
                rows.append(st.view(hip.N_CU, 16)[:, :11].cpu().double())
    finally:
        hip.lib = orig
    names = ["qkv_start", "qkv_done", "attn_start", "attn_done", "o_start", "o_done", "gu_start", "gu_done",
             "down_start", "down_done", "next_exit"]
    for s in rows:
        t0 = s[:, 0].min()
        us = (s - t0) / 100.0
        line = "  ".join(f"{n}={us[:, i].median():.2f}/{us[:, i].max():.2f}" for i, n in enumerate(names))
        print(line, flush=True)


if __name__ == "__main__":
    main()
