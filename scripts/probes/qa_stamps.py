#!/usr/bin/env python3
"""Where the fused QKV + attention launch (scripts/probes/qkv_attn.hip) spends its time at batch
1, Llama-2-7B layer shapes: per-workgroup s_memrealtime stamps (100 MHz) from the diagnostic
builds (-DLSA_QA_STAMPS -> _native/liblsa_qa_stamps*.so, `--build` on the CPU host), plus
hipGraph-timed A/B of the fused launch (no-stamp build, _native/liblsa_qa.so) against
gemv(EPI_QKV) + attn (the two library launches it replaces). Measured slower than the two
launches (profiles/r4_qkv_attn_fusion.md), so the kernel is a probe, not a library route.

usage: qa_stamps.py [T] | --build"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "llm_sharding_amd", "_native", "liblsa_qa_stamps.so")
PROD_SO = os.path.join(ROOT, "llm_sharding_amd", "_native", "liblsa_qa.so")
SRC = os.path.join(ROOT, "scripts", "probes", "qkv_attn.hip")
CFGS = {(1, 4, 4), (1, 4, 8), (2, 4, 4)}  # (tn, nw, u) built in qkv_attn.hip


VARIANTS = {"": [], "_u8": ["-DQA_U=8"], "_u16": ["-DQA_U=16"], "_u8_pf": ["-DQA_U=8", "-DQA_PF=1"],
            "_nocons": ["-DLSA_QA_NOCONS"]}


def build():
    base = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
            "-I", os.path.join(ROOT, "csrc", "kernels")]
    subprocess.check_call(base + ["-o", PROD_SO, SRC])
    print("built", PROD_SO)
    for suf, flags in VARIANTS.items():
        so = SO.replace(".so", suf + ".so")
        subprocess.check_call(base + ["-DLSA_QA_STAMPS", *flags, "-o", so, SRC])
        print("built", so)


def _load(so):
    from llm_sharding_amd.ops import hip
    L = ctypes.CDLL(so)
    vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    L.lsa_qkv_attn.argtypes = [vp, i, vp, i, i, i, f, ctypes.POINTER(hip.EpiArgs), i, i, i, f, vp, i, vp, vp, vp]
    L.lsa_qkv_attn_sync_words.argtypes = [i]
    return L


def qkv_attn_config(M, N, K, n_heads, n_kv, head_dim):
    """(tn, nw, u) of the tuned streaming GEMV at this shape when qkv_attn.hip has it built."""
    from llm_sharding_amd.ops.packing import proj_config
    algo, cfg = proj_config(N // 16, M, need_even=False, k=K)
    if algo != "gemv" or tuple(cfg) not in CFGS or (K // 32) % cfg[2] or head_dim != 128:
        return None
    return tuple(cfg)


def fused(L, x, wp, M, N, K, eps, ep, ao, sync, err, cfg):
    import torch
    rc = L.lsa_qkv_attn(ctypes.c_void_p(x.data_ptr()), x.stride(0), ctypes.c_void_p(wp.data_ptr()), M, N, K, eps,
                        ctypes.byref(ep), cfg[0], cfg[1], cfg[2], ep.head_dim ** -0.5, ctypes.c_void_p(ao.data_ptr()),
                        ao.stride(0), ctypes.c_void_p(sync.data_ptr()), ctypes.c_void_p(err.data_ptr()),
                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc


def main():
    if sys.argv[1:2] == ["--build"]:
        build()
        return
    import torch
    from llm_sharding_amd.config import LlamaConfig
    from llm_sharding_amd.models.rope import rope_table
    from llm_sharding_amd.ops import hip, packing
    from scripts.bench_kernels import timeit
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    nh = nkv = 32
    hd, H = 128, 4096
    N = (nh + 2 * nkv) * hd
    t_max = 1024
    cfg = LlamaConfig()
    nbuf = 8
    wps = [packing.pack_b(torch.randn(N, H, device="cuda").mul_(0.02).to(torch.bfloat16)) for _ in range(nbuf)]
    x = torch.randn(1, H, device="cuda").to(torch.bfloat16)
    kc = torch.randn(1, nkv, t_max, hd, device="cuda").to(torch.bfloat16)
    vc = torch.randn_like(kc)
    slot = torch.zeros(1, dtype=torch.int32, device="cuda")
    pos = torch.full((1,), T - 1, dtype=torch.int32, device="cuda")
    cos, sin = rope_table(cfg, t_max, "cuda")
    q = torch.empty(1, nh * hd, dtype=torch.bfloat16, device="cuda")
    ao = torch.empty_like(q)
    ep = hip.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, cos=cos, sin=sin, ldo=q.stride(0),
                      n_heads=nh, n_kv=nkv, head_dim=hd, t_max=t_max)
    P = _load(PROD_SO)
    sync = torch.zeros(P.lsa_qkv_attn_sync_words(nkv), dtype=torch.int32, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    po = torch.empty(nh * hd * 16, device="cuda")
    pl = torch.empty(nh * 16, device="cuda")
    cnt = torch.zeros(4096, dtype=torch.int32, device="cuda")
    qcfg = qkv_attn_config(1, N, H, nh, nkv, hd)
    res = {"T": T, "cfg": qcfg}
    res["fused_us"] = round(timeit(lambda i: fused(P, x, wps[i % nbuf], 1, N, H, 1e-5, ep, ao, sync, err, qcfg)), 2)
    res["gemv_qkv_us"] = round(timeit(lambda i: hip.gemv(x, wps[i % nbuf], 1, N, H, hip.EPI_QKV, ep, norm=True)), 2)
    res["attn_us"] = round(timeit(lambda i: hip.attn(q, kc, vc, slot, pos, 1, nh, nkv, hd, 1, po, pl, ao,
                                                     counters=cnt, min_chunk=256)), 2)
    res["two_launches_us"] = round(timeit(lambda i: (hip.gemv(x, wps[i % nbuf], 1, N, H, hip.EPI_QKV, ep, norm=True),
                                                      hip.attn(q, kc, vc, slot, pos, 1, nh, nkv, hd, 1, po, pl, ao,
                                                               counters=cnt, min_chunk=256))), 2)
    for suf in VARIANTS:
        so = SO.replace(".so", suf + ".so")
        if not os.path.exists(so):
            continue
        L = _load(so)
        st = torch.zeros(4 * 1024, dtype=torch.int64, device="cuda")
        L.lsa_qa_set_stamps(ctypes.c_void_p(st.data_ptr()))
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for r in range(3):
            st.zero_()
            rc = L.lsa_qkv_attn(ctypes.c_void_p(x.data_ptr()), x.stride(0), ctypes.c_void_p(wps[r].data_ptr()), 1, N, H,
                                1e-5, ctypes.byref(ep), qcfg[0], qcfg[1], qcfg[2], hd ** -0.5,
                                ctypes.c_void_p(ao.data_ptr()), ao.stride(0), ctypes.c_void_p(sync.data_ptr()),
                                ctypes.c_void_p(err.data_ptr()), stream)
            assert rc == 0, rc
            torch.cuda.synchronize()
        s = st.view(-1, 4).cpu().double()
        n_prod = N // 16 // qcfg[0]
        us = lambda v: round(float(v) / 100.0 * 1e0, 2)  # 100 MHz ticks -> us
        prod, cons = s[:n_prod], s[n_prod:n_prod + nkv]
        t0 = prod[:, 0].min()
        d = {"producer_start_p50_max": [us((prod[:, 0] - t0).median()), us((prod[:, 0] - t0).max())],
             "producer_done_p50_max": [us((prod[:, 1] - t0).median()), us((prod[:, 1] - t0).max())]}
        if "nocons" not in suf:
            d.update({"consumer_start_p50_max": [us((cons[:, 0] - t0).median()), us((cons[:, 0] - t0).max())],
                      "consumer_wait_done_p50_max": [us((cons[:, 1] - t0).median()), us((cons[:, 1] - t0).max())],
                      "consumer_end_p50_max": [us((cons[:, 2] - t0).median()), us((cons[:, 2] - t0).max())]})
        res["stamps_us" + suf] = d
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
