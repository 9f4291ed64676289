"""ctypes bindings for the in-tree HIP kernel library (``_native/liblsa_kernels.so``).

Every wrapper takes torch tensors that live on the current ROCm device, checks the shapes the
kernel's grid assumes (a bad shape must never reach the GPU: an out-of-bounds wave can reset
the whole node), and launches on ``torch.cuda.current_stream()`` so that the launches are
captured by ``torch.cuda.graph`` (hipGraph) like any other stream work.

The library is loaded AFTER ``import torch`` so that its ``libamdhip64.so.7`` dependency
resolves (by soname) to the HIP runtime torch already loaded: one runtime, shared streams.
If the library is missing on a machine with a GPU we raise - there is no silent fallback.
"""
from __future__ import annotations

import ctypes
import functools
import json
import os
from contextlib import contextmanager
from typing import Optional

import torch

from . import routes

NATIVE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native")
# LSA_KERNELS_SO: load another build of the kernel library (A/B runs of build flags only; the
# product and every test use the in-tree _native/liblsa_kernels.so)
KERNELS_SO = os.environ.get("LSA_KERNELS_SO") or os.path.join(NATIVE_DIR, "liblsa_kernels.so")

EPI_STORE, EPI_RESID, EPI_SWIGLU, EPI_QKV, EPI_ARGMAX, EPI_PARTIAL = range(6)
_STATUS = {0: "ok", 1: "bad shape", 2: "unsupported", 3: "launch failed"}
_UNSUPPORTED = 2  # LSA_UNSUPPORTED: no kernel instantiation for the shape


class EpiArgs(ctypes.Structure):
    _fields_ = [
        ("out", ctypes.c_void_p), ("resid", ctypes.c_void_p), ("k_cache", ctypes.c_void_p),
        ("v_cache", ctypes.c_void_p), ("slot", ctypes.c_void_p), ("pos", ctypes.c_void_p),
        ("cos_t", ctypes.c_void_p), ("sin_t", ctypes.c_void_p), ("keys", ctypes.c_void_p),
        ("bias", ctypes.c_void_p),
        ("ldo", ctypes.c_int), ("ldr", ctypes.c_int), ("n_heads", ctypes.c_int),
        ("n_kv", ctypes.c_int), ("head_dim", ctypes.c_int), ("t_max", ctypes.c_int),
        ("col_offset", ctypes.c_int), ("act", ctypes.c_int),
        ("ss_out", ctypes.c_void_p), ("ss_in", ctypes.c_void_p), ("ss_n", ctypes.c_int), ("ss_eps", ctypes.c_float),
    ]


_lib = None


def available() -> bool:
    return os.path.exists(KERNELS_SO)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(KERNELS_SO):
        raise RuntimeError(
            f"HIP kernel library not built: {KERNELS_SO} missing. Run `python csrc/build.py` "
            "(or __graft_entry__.build()).")
    _lib = load_library(KERNELS_SO, ctypes.RTLD_GLOBAL)
    return _lib


def load_library(path: str, mode: int = ctypes.RTLD_LOCAL) -> ctypes.CDLL:
    """Load one build of the kernel library with every entry point's signature declared.
    Two builds can live in one process when both are loaded RTLD_LOCAL (each resolves its own
    kernels; scripts/slp_kernel_diff.py runs every kernel of a step from both)."""
    L = ctypes.CDLL(path, mode=mode)
    vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    L.lsa_gemv.argtypes = [vp, i, vp, vp, i, i, i, i, f, i, ctypes.POINTER(EpiArgs), i, i, i, vp]
    L.lsa_gemv_coop.argtypes = [vp, i, vp, vp, i, i, i, i, f, i, ctypes.POINTER(EpiArgs), i, i, i, i, i, i, vp, vp, vp]
    L.lsa_gemv_fp8.argtypes = [vp, i, vp, vp, vp, i, i, i, i, f, i, ctypes.POINTER(EpiArgs), i, i, i, vp]
    L.lsa_dequant_fp8_packed.argtypes = [vp, vp, vp, i, i, vp]
    L.lsa_gemv_coop_fp8.argtypes = [vp, i, vp, vp, vp, i, i, i, i, f, i, ctypes.POINTER(EpiArgs), i, i, i, i, vp, vp, vp]
    L.lsa_gemm.argtypes = [vp, i, vp, i, i, i, i, ctypes.POINTER(EpiArgs), i, i, vp, vp, vp]
    L.lsa_attn_decode.argtypes = [vp, i, vp, vp, vp, vp, vp, i, i, i, i, i, f, i, i, vp, vp, vp, i, vp, vp]
    L.lsa_attn_prefill.argtypes = [vp, i, vp, vp, vp, i, i, i, i, i, f, i, vp, i, vp]
    L.lsa_attn_decode_mfma.argtypes = [vp, i, vp, vp, vp, vp, vp, i, i, i, i, i, f, vp, i, i, vp]
    L.lsa_embed.argtypes = [vp, i, vp, i, vp, i, vp]
    L.lsa_rmsnorm.argtypes = [vp, i, vp, i, i, f, vp, i, vp]
    L.lsa_layernorm.argtypes = [vp, i, vp, vp, vp, vp, i, i, f, vp, i, vp]
    L.lsa_resid_rmsnorm_partials.argtypes = [vp, i, vp, i, ctypes.c_longlong, i, vp, i, i, f, vp, i, vp]
    L.lsa_row_ss.argtypes = [vp, i, i, i, vp, vp]
    L.lsa_argmax_finalize.argtypes = [vp, i, vp, vp, i, vp, i, i, vp, vp]
    L.lsa_pos_advance.argtypes = [vp, i, i, vp]
    L.lsa_gemm_wr.argtypes = [vp, i, vp, i, i, i, i, ctypes.POINTER(EpiArgs), i, i, vp]
    L.lsa_gemm_sk.argtypes = [vp, i, vp, i, i, i, i, ctypes.POINTER(EpiArgs), i, i, i, i, i, i, i, vp, vp, ctypes.c_longlong, i,
                              vp]
    L.lsa_attn_oproj.argtypes = [vp, i, vp, vp, vp, vp, vp, i, i, i, i, f, vp, vp, i, i, ctypes.POINTER(EpiArgs), vp, i,
                                 vp]
    for name in ("lsa_gemv", "lsa_gemv_coop", "lsa_attn_oproj", "lsa_gemv_fp8", "lsa_dequant_fp8_packed", "lsa_gemv_coop_fp8", "lsa_gemm",
                 "lsa_gemm_sk", "lsa_gemm_wr", "lsa_attn_decode", "lsa_attn_prefill", "lsa_embed", "lsa_rmsnorm", "lsa_layernorm",
                 "lsa_resid_rmsnorm_partials", "lsa_row_ss",
                 "lsa_argmax_finalize", "lsa_pos_advance", "lsa_version"):
        getattr(L, name).restype = ctypes.c_int
    if os.environ.get("LSA_ATTN_SMALL_MAX_WGS"):  # A/B runs of the small-grid decode attention's range
        L.lsa_attn_set_small_max_wgs.argtypes = [i]
        _check(L.lsa_attn_set_small_max_wgs(int(os.environ["LSA_ATTN_SMALL_MAX_WGS"])), "lsa_attn_set_small_max_wgs")
    return L


def _p(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what}: {_STATUS.get(rc, rc)}")


def _req(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


def _is_bf16_cuda(*ts) -> bool:
    return all(t is None or (t.is_cuda and t.dtype == torch.bfloat16) for t in ts)


ACT_NONE, ACT_GELU = 0, 1  # EpiArgs.act (EPI_STORE): identity / tanh-GELU (GPT-2 "gelu_new")


def make_epi(out=None, resid=None, k_cache=None, v_cache=None, slot=None, pos=None, cos=None,
             sin=None, keys=None, ldo=0, ldr=0, n_heads=0, n_kv=0, head_dim=0, t_max=0,
             col_offset=0, bias=None, act=ACT_NONE, ss_out=None, ss_in=None, ss_eps=0.0) -> EpiArgs:
    """Epilogue arguments. ``bias``: optional fp32 [N] added to every output column (in packed
    column order); ``cos=None`` with EPI_QKV: no RoPE, natural q|k|v column order.
    ``ss_out`` / ``ss_in`` (gemm_sk): fp32 [>= M, H/64] row partial sums of squares - a RESID
    GEMM writes them for its outputs, a QKV / SWIGLU GEMM reading the raw residual stream as A
    applies the RMSNorm scale from them (the norm weight is folded into its W)."""
    if bias is not None:
        _req(bias.dtype == torch.float32 and bias.is_contiguous(), "epilogue bias: contiguous fp32")
    # vectorised epilogues store 16-B runs: rows must start 16-B aligned
    _req(ldo % 8 == 0 and ldr % 8 == 0, f"epilogue: ldo/ldr ({ldo}, {ldr}) must be multiples of 8")
    for t in (out, resid, bias):
        _req(t is None or t.data_ptr() % 16 == 0, "epilogue: out/resid/bias must be 16-byte aligned")
    _req(head_dim == 0 or (head_dim & (head_dim - 1)) == 0, f"epilogue: head_dim {head_dim} not a power of two")
    ssb = ss_in if ss_in is not None else ss_out
    for t in (ss_out, ss_in):
        _req(t is None or (t.dtype == torch.float32 and t.dim() == 2 and t.is_contiguous()), "epilogue: ss fp32 [M, H/64]")
    return EpiArgs(_p(out), _p(resid), _p(k_cache), _p(v_cache), _p(slot), _p(pos), _p(cos), _p(sin),
                   _p(keys), _p(bias), ldo, ldr, n_heads, n_kv, head_dim, t_max, col_offset, int(act),
                   _p(ss_out), _p(ss_in), 0 if ssb is None else ssb.shape[1], float(ss_eps))


# ------------------------------------------------------------------------------ projections
class CoopWorkspace:
    """Split-K partial slabs + per-column-group arrival counters for ``lsa_gemv_coop``.

    Launches on one stream may share a workspace (they are stream-ordered and the last
    arriving workgroup resets its counter before the kernel ends). The counters are zeroed
    once here; the slab needs no initialisation."""

    def __init__(self, device, slab_floats: int = 1 << 22, groups: int = 1 << 14):
        self.slab = torch.empty(max(slab_floats, 1), dtype=torch.float32, device=device)
        self.counters = torch.zeros(groups, dtype=torch.int32, device=device)


_WS = {}


def default_workspace(device=None) -> CoopWorkspace:
    """Process-wide workspace per (device, stream), grown on demand (outside graph capture)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    if key not in _WS:
        _WS[key] = CoopWorkspace(dev, slab_floats=1 << 24)
    return _WS[key]


def _check_epi(epi: int, ep: EpiArgs, N: int) -> None:
    """Host-side guard for the in-kernel stores: a QKV epilogue writes q + k/v columns into
    caches of n_kv heads, so its column count must match the head geometry exactly."""
    if epi == EPI_QKV:
        _req(N == (ep.n_heads + 2 * ep.n_kv) * ep.head_dim,
             f"QKV epilogue: N={N} != (n_heads {ep.n_heads} + 2 n_kv {ep.n_kv}) x head_dim {ep.head_dim}")
    elif epi == EPI_ARGMAX:
        _req(bool(ep.keys), "ARGMAX epilogue needs keys")


def gemv(x: torch.Tensor, wp: torch.Tensor, M: int, N: int, K: int, epi: int, ep: EpiArgs,
         norm: bool = False, eps: float = 1e-5, a_rows: Optional[torch.Tensor] = None,
         tn: int = 0, nw: int = 0, u: int = 0, coop: Optional[tuple] = None,
         ws: Optional[CoopWorkspace] = None, out_numel: int = 0) -> None:
    """Decode / short-prefill projection, M <= 128 rows (> 64: coop kernel only). ``wp`` is ``pack_b(W)`` (``pack_b(fold_norm(W, g))``
    when ``norm``: RMSNorm of the A rows is then applied in-kernel), W: [N, K].

    Kernel choice: explicit ``tn/nw/u`` -> streaming GEMV (gemv.hip); explicit
    ``coop=(tnw, nw, kf, sk[, kw[, d]])`` -> cooperative split-K (gemv_coop.hip); neither -> the tuned
    choice of :func:`packing.proj_config`. EPI_PARTIAL (coop only): split s writes its fp32 tile
    to ``ep.out`` viewed as [sk][M][ldo] (``out_numel`` = its capacity in floats, checked) for
    :func:`resid_rmsnorm_partials`."""
    from .packing import GEMV_CONFIGS, coop_candidates, coop_norm, coop_slab_floats, proj_config, row_blocks
    _req(1 <= M <= 128, f"gemv supports 1..128 rows, got {M}")
    _check_epi(epi, ep, N)
    _req(_is_bf16_cuda(x, wp), "gemv: bf16 cuda tensors required")
    _req(wp.numel() == N * K and N % 16 == 0 and K % 32 == 0, "gemv: packed weight shape")
    _req(x.dim() == 2 and x.shape[1] >= K and x.stride(1) == 1, "gemv: x must be [rows, >=K] row-major")
    if a_rows is None:
        _req(x.shape[0] >= M, "gemv: x has fewer rows than M")
    else:
        _req(a_rows.dtype == torch.int32 and a_rows.is_cuda and a_rows.numel() >= M, "gemv: a_rows")
    if tn == 0 and coop is None:
        algo, cfg = proj_config(N // 16, M, need_even=(epi == EPI_SWIGLU), k=K)
        if algo == "coop":
            coop = cfg
        else:
            tn, nw, u = cfg
    _req(epi != EPI_PARTIAL or coop is not None, "gemv: EPI_PARTIAL needs an explicit coop config")
    if coop is not None:
        coop = coop_norm(coop)
        tnw, cnw, kf, sk, kw, depth = coop
        if epi == EPI_PARTIAL:
            _req(out_numel >= sk * M * ep.ldo, f"gemv partial: output holds {out_numel} floats, "
                 f"{sk} splits x {M} rows x ldo {ep.ldo} needed")
        _req(coop in coop_candidates(N // 16, K, M, epi == EPI_SWIGLU),
             f"gemv: coop config {coop} invalid for N={N} K={K} M={M}")
        if ws is None:
            ws = default_workspace(x.device)
        need = coop_slab_floats(N, M, tnw, cnw, kf, sk)
        _req(ws.slab.numel() >= need, f"gemv: coop workspace too small ({ws.slab.numel()} < {need} floats)")
        _req(ws.counters.numel() >= N // 16 // (tnw * cnw), "gemv: coop workspace counters too small")
        rc = lib().lsa_gemv_coop(_p(x), x.stride(0), _p(a_rows), _p(wp), M, N, K, int(norm), float(eps), epi,
                                 ctypes.byref(ep), tnw, cnw, kf, sk, kw, depth, _p(ws.slab), _p(ws.counters), _stream())
        _check(rc, "lsa_gemv_coop")
        return
    mb = row_blocks(M)
    _req((tn, mb, nw, u) in GEMV_CONFIGS, f"gemv: config tn={tn} nw={nw} u={u} not built for {M} rows")
    _req((K // 32) % u == 0, f"gemv: K={K} must be a multiple of {32 * u}")
    rc = lib().lsa_gemv(_p(x), x.stride(0), _p(a_rows), _p(wp), M, N, K, int(norm), float(eps), epi,
                        ctypes.byref(ep), tn, nw, u, _stream())
    _check(rc, "lsa_gemv")


def gemv_fp8(x: torch.Tensor, wq: torch.Tensor, wscale: torch.Tensor, M: int, N: int, K: int, epi: int,
             ep: EpiArgs, norm: bool = False, eps: float = 1e-5, a_rows: Optional[torch.Tensor] = None,
             cfg: Optional[tuple] = None) -> None:
    """W8A16 decode projection (gemv_fp8.hip), M <= 64: ``wq`` = pack_b_fp8(q) (uint8),
    ``wscale`` fp32 [N] per-row scale (the RMSNorm weight folded in before quantisation)."""
    from .packing import FP8_CONFIGS, fp8_config, row_blocks
    _req(1 <= M <= 64, f"gemv_fp8 supports 1..64 rows, got {M}")
    _check_epi(epi, ep, N)
    _req(_is_bf16_cuda(x), "gemv_fp8: bf16 cuda activations")
    _req(wq.is_cuda and wq.dtype == torch.uint8 and wq.numel() == N * K, "gemv_fp8: packed fp8 weights [N*K] uint8")
    _req(wscale.is_cuda and wscale.dtype == torch.float32 and wscale.numel() >= N, "gemv_fp8: fp32 scales [N]")
    _req(N % 16 == 0 and K % 64 == 0, "gemv_fp8: N % 16, K % 64")
    _req(x.dim() == 2 and x.shape[1] >= K and x.stride(1) == 1, "gemv_fp8: x must be [rows, >=K] row-major")
    if a_rows is None:
        _req(x.shape[0] >= M, "gemv_fp8: x has fewer rows than M")
    else:
        _req(a_rows.dtype == torch.int32 and a_rows.is_cuda and a_rows.numel() >= M, "gemv_fp8: a_rows")
    tn, nw, u2 = cfg if cfg is not None else fp8_config(N // 16, M, need_even=(epi == EPI_SWIGLU), k=K)
    _req((tn, row_blocks(M), nw, u2) in FP8_CONFIGS, f"gemv_fp8: config {(tn, nw, u2)} not built for {M} rows")
    rc = lib().lsa_gemv_fp8(_p(x), x.stride(0), _p(a_rows), _p(wq), _p(wscale), M, N, K, int(norm), float(eps), epi,
                            ctypes.byref(ep), tn, nw, u2, _stream())
    _check(rc, "lsa_gemv_fp8")


def proj_fp8(x: torch.Tensor, wq: torch.Tensor, wscale: torch.Tensor, M: int, N: int, K: int, epi: int,
             ep: EpiArgs, norm: bool = False, eps: float = 1e-5, a_rows: Optional[torch.Tensor] = None,
             ws: Optional[CoopWorkspace] = None, algo: Optional[tuple] = None) -> None:
    """W8A16 projection for 1..128 rows: plain fp8 GEMV or the cooperative kernel with fp8
    weights (``packing.fp8_proj_config`` unless ``algo=(name, cfg)`` is given)."""
    from .packing import coop_fp8_candidates, coop_slab_floats, fp8_proj_config
    _req(1 <= M <= 128, f"proj_fp8 supports 1..128 rows, got {M}")
    _check_epi(epi, ep, N)
    name, cfg = algo if algo is not None else fp8_proj_config(N // 16, M, need_even=(epi == EPI_SWIGLU), k=K)
    if name == "fp8":
        gemv_fp8(x, wq, wscale, M, N, K, epi, ep, norm=norm, eps=eps, a_rows=a_rows, cfg=cfg)
        return
    _req(_is_bf16_cuda(x), "proj_fp8: bf16 cuda activations")
    _req(wq.is_cuda and wq.dtype == torch.uint8 and wq.numel() == N * K, "proj_fp8: packed fp8 weights")
    _req(wscale.is_cuda and wscale.dtype == torch.float32 and wscale.numel() >= N, "proj_fp8: fp32 scales")
    _req(x.dim() == 2 and x.shape[1] >= K and x.stride(1) == 1, "proj_fp8: x must be [rows, >=K] row-major")
    if a_rows is None:
        _req(x.shape[0] >= M, "proj_fp8: x has fewer rows than M")
    else:
        _req(a_rows.dtype == torch.int32 and a_rows.is_cuda and a_rows.numel() >= M, "proj_fp8: a_rows")
    cfg = tuple(cfg)
    _req(cfg in coop_fp8_candidates(N // 16, K, M), f"proj_fp8: coop config {cfg} invalid for N={N} K={K} M={M}")
    tnw, cnw, kf, sk = cfg
    if ws is None:
        ws = default_workspace(x.device)
    _req(ws.slab.numel() >= coop_slab_floats(N, M, tnw, cnw, kf, sk), "proj_fp8: coop workspace too small")
    _req(ws.counters.numel() >= N // 16 // (tnw * cnw), "proj_fp8: coop workspace counters too small")
    rc = lib().lsa_gemv_coop_fp8(_p(x), x.stride(0), _p(a_rows), _p(wq), _p(wscale), M, N, K, int(norm), float(eps),
                                 epi, ctypes.byref(ep), tnw, cnw, kf, sk, _p(ws.slab), _p(ws.counters), _stream())
    _check(rc, "lsa_gemv_coop_fp8")


def dequant_fp8_packed(wq: torch.Tensor, wscale: torch.Tensor, out: torch.Tensor, N: int, K: int) -> torch.Tensor:
    """Packed fp8 (+ row scales) -> packed bf16 (pack_b layout) in ``out`` (>= N*K bf16)."""
    _req(wq.is_cuda and wq.dtype == torch.uint8 and wq.numel() == N * K, "dequant_fp8: weights")
    _req(wscale.dtype == torch.float32 and wscale.numel() >= N, "dequant_fp8: scales")
    _req(_is_bf16_cuda(out) and out.numel() >= N * K, "dequant_fp8: out")
    _check(lib().lsa_dequant_fp8_packed(_p(wq), _p(wscale), _p(out), N, K, _stream()), "lsa_dequant_fp8_packed")
    return out.view(-1)[:N * K].view(N // 16, K // 32, 64, 8)


def gemm_split(M: int, N: int, K: int, tn: int) -> int:
    """Split-K factor for the prefill GEMM, fitted to the MI355X sweep
    (profiles/r1_gemm_splitk_sweep.jsonl): small grids (few 128-row x 64*tn-col tiles) are split
    over K until ~384*sqrt(K/4096) workgroups stream the weights (long-K shapes like down_proj
    want more), at most 8 ways and >= 8 K-tiles of 64 per split."""
    tiles = -(-M // 128) * (N // (64 * tn))
    target = 384.0 * (K / 4096.0) ** 0.5
    return int(max(1, min(8, int(target // tiles), (K // 64) // 8)))


def gemm_slab_floats(M: int, N: int, sk: int) -> int:
    return 0 if sk <= 1 else sk * (-(-M // 128) * 128) * N


def gemm(a: torch.Tensor, wp: torch.Tensor, M: int, N: int, K: int, epi: int, ep: EpiArgs,
         tn: int = 2, sk: int = 0, ws: Optional["CoopWorkspace"] = None,
         sk_ws: Optional["SkWorkspace"] = None, legacy: bool = False) -> None:
    """Projection GEMM for > 128 rows (any M). Shapes with N % 128 == 0 (every Llama / GPT-2
    projection) run the stream-K LDS-DMA kernel (:func:`gemm_sk`, workspace ``sk_ws``); other
    shapes (or ``legacy=True``) the 128-row-tile kernel of gemm.hip, N a multiple of 64*tn,
    ``sk`` its split-K factor (0 = :func:`gemm_split`; > 1 uses ``ws``)."""
    if not legacy and N % 128 == 0 and K % 64 == 0 and epi != EPI_ARGMAX and a.stride(0) % 8 == 0 \
            and a.data_ptr() % 16 == 0:
        wr = gemm_wr_plan(M, N, K, epi, ep)
        if wr:
            gemm_wr(a, wp, M, N, K, epi, ep, bn=wr)
        else:
            gemm_sk(a, wp, M, N, K, epi, ep, ws=sk_ws)
        return
    _req(not (ep.ss_out or ep.ss_in), "gemm: the fused-norm epilogue fields need the gemm_sk path")
    _req(_is_bf16_cuda(a, wp), "gemm: bf16 cuda tensors required")
    _req(wp.numel() == N * K and K % 64 == 0, "gemm: packed weight shape")
    _req(a.dim() == 2 and a.shape[0] >= M and a.shape[1] >= K and a.stride(1) == 1, "gemm: A shape")
    _check_epi(epi, ep, N)
    if N % (64 * tn):
        tn = 1
    _req(N % (64 * tn) == 0, f"gemm: N={N} not a multiple of {64 * tn}")
    _req(not (epi == EPI_SWIGLU and tn != 2), "gemm: SwiGLU needs N % 128 == 0")
    if sk == 0:
        sk = gemm_split(M, N, K, tn)
    _req(1 <= sk <= K // 64, f"gemm: split-K {sk} out of range")
    slab = cnt = None
    if sk > 1:
        if ws is None:
            ws = default_workspace(a.device)
        need = gemm_slab_floats(M, N, sk)
        tiles = -(-M // 128) * (N // (64 * tn))
        if ws.slab.numel() < need or ws.counters.numel() < tiles:
            sk = 1  # workspace too small for this call: fall back to the unsplit kernel
        else:
            slab, cnt = ws.slab, ws.counters
    rc = lib().lsa_gemm(_p(a), a.stride(0), _p(wp), M, N, K, epi, ctypes.byref(ep), tn, sk, _p(slab), _p(cnt),
                        _stream())
    _check(rc, "lsa_gemm")


SK_BM = 256  # gemm_sk.hip row tile (default; 128-row tiles for small / odd M: plan field bm)

# gemm_wr.hip (weights streamed into MFMA registers, 128 x bn tiles, whole-K tiles): the qkv
# projections (store / QKV epilogue) where it measured faster than gemm_sk's best plan and than
# hipBLASLt. Per (N, K): (first row, last row, bn) ranges, each bounded by measured row counts
# (cold-weight probes, profiles/r4_gemm_wr_shapes.jsonl; the 7B range also in the engine,
# profiles/r3_gemm_wr.md, and the 3B / 13B ranges in engine A/B runs, profiles/r4_gemm_wr_engine_ab.txt):
#   Llama-2-7B qkv  12288 x 4096: 384-512 rows bn 192 (54-57 us vs gemm_sk 59-81, hipBLASLt 57-59),
#                                 256 rows bn 128 (49 vs 52, hipBLASLt 65)
#   Llama-2-13B qkv 15360 x 5120: 320-384 rows bn 192 (69-72 us vs 88-94, hipBLASLt 80-86),
#                                 448-512 rows bn 256 (78-82 us vs 91-95, hipBLASLt 98-102),
#                                 256 rows bn 128 (64 vs 69, hipBLASLt 80)
#   Llama-3.2-3B qkv 5120 x 3072: 256-512 rows bn 128 (37-38 us vs 40-46, hipBLASLt 41-49)
#   Llama-3.2-3B gate_up 16384 x 3072 (SwiGLU): 320-512 rows bn 256 (store epilogue 52-60 us vs
#                                 gemm_sk 68-74, hipBLASLt 57-74), 256 rows bn 128 (41 vs 73, 58)
#   Llama-2-7B gate_up 22016 x 4096 (SwiGLU): 256 rows bn 256 (store 68 us vs gemm_sk 75, 76)
#   Llama-2-13B gate_up 27648 x 5120 (SwiGLU): 256 rows bn 256 (94 us vs 101, 104)
# A range starting at 193 rows covers the same 2-row-tile grid as its measured 256-row point.
# (70B qkv, 10240 x 8192, measured a tie at 384 rows and slower at 448: not routed.)
# LSA_GEMM_WR=0 turns the route off (A/B runs).
def gemm_wr_plan(M: int, N: int, K: int, epi: int, ep: "EpiArgs") -> Optional[int]:
    """bn for :func:`gemm_wr`, or None when gemm_sk takes the shape (the route table:
    ops/routes.py)."""
    if os.environ.get("LSA_GEMM_WR", "1") == "0" or ep.act or ep.bias or ep.ss_out:
        return None
    if epi not in (EPI_STORE, EPI_QKV, EPI_SWIGLU):
        return None
    mt = -(-M // 128)
    # the last row tile at least half full: the kernel computes whole 128-row tiles, gemm_sk's
    # 128-row plans do not (measured at 448 and 512 rows)
    if M - (mt - 1) * 128 < 64:
        return None
    r = routes.route(M, N, K, epi)
    if r.kernel != "gemm_wr":
        return None
    bn = r.params["bn"]
    if N % bn == 0 and K % 64 == 0 and not (epi == EPI_SWIGLU and bn == 192):
        return bn
    return None


def gemm_wr(a: torch.Tensor, wp: torch.Tensor, M: int, N: int, K: int, epi: int, ep: EpiArgs, bn: int = 192,
            grid: int = 0) -> None:
    """Projection GEMM with the weights fetched straight into MFMA B registers (gemm_wr.hip):
    128 x ``bn`` tiles, one per workgroup per round, A staged by LDS-DMA, EPI_STORE / EPI_QKV /
    EPI_SWIGLU (the last two with the fused RMSNorm row scale, ``ep.ss_in``). K % 64 == 0,
    N % bn == 0."""
    _req(_is_bf16_cuda(a, wp), "gemm_wr: bf16 cuda tensors required")
    _req(wp.numel() == N * K and K % 64 == 0, "gemm_wr: packed weight shape (K % 64 == 0)")
    _req(a.dim() == 2 and a.shape[0] >= M >= 1 and a.shape[1] >= K and a.stride(1) == 1 and a.stride(0) % 8 == 0
         and a.data_ptr() % 16 == 0, "gemm_wr: A must be [>=M, >=K] row-major with 16-B aligned rows")
    _req(bn in (128, 192, 256) and N % bn == 0, f"gemm_wr: N={N} does not tile by bn={bn}")
    _req(epi in (EPI_STORE, EPI_QKV, EPI_SWIGLU), "gemm_wr: EPI_STORE / EPI_QKV / EPI_SWIGLU")
    _req(epi != EPI_SWIGLU or bn != 192, "gemm_wr: SwiGLU needs bn 128 / 256 (whole gate/up pairs per wave)")
    _req(not ep.ss_out, "gemm_wr: no ss_out epilogue")
    _check_epi(epi, ep, N)
    rc = lib().lsa_gemm_wr(_p(a), a.stride(0), _p(wp), M, N, K, epi, ctypes.byref(ep), bn, grid or N_CU, _stream())
    _check(rc, "lsa_gemm_wr")


class SkWorkspace:
    """Stream-K partial slabs (2 per workgroup, 256 x BN fp32 each) + per-tile arrival tickets
    for ``lsa_gemm_sk``. Tickets reset themselves (the last arriver zeroes its tile's); slabs
    need no initialisation. One workspace per stream / concurrently replayed graph."""

    def __init__(self, device, grid: int = 256, bn: int = 256):
        self.grid, self.bn = grid, bn
        self.slab = torch.empty(2 * grid * SK_BM * bn, dtype=torch.float32, device=device)
        self.counters = torch.zeros(4 * grid, dtype=torch.int32, device=device)


_SKWS = {}


def default_sk_workspace(device=None) -> SkWorkspace:
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    if key not in _SKWS:
        _SKWS[key] = SkWorkspace(dev)
    return _SKWS[key]


N_CU = 256


SK_TUNING_FILE = os.environ.get("LSA_GEMM_SK_TUNING") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                     "gemm_sk_tuning.json")
_SK_TUNED = None
_SK_PARTIAL = None


def _sk_load() -> None:
    global _SK_TUNED, _SK_PARTIAL
    _SK_TUNED, _SK_PARTIAL = {}, {}
    if os.path.exists(SK_TUNING_FILE):
        with open(SK_TUNING_FILE) as f:
            for e in json.load(f).get("entries", []):
                _SK_TUNED.setdefault((e["N"], e["K"]), []).append((e["M"], tuple(e["cfg"])))
                if "partial" in e:  # measured on a residual projection: [bn, split] or null
                    pp = e["partial"]
                    if pp is not None and not (1 <= pp[1] <= PARTIAL_MAX_SPLIT):
                        pp = None  # the engine's partial buffer holds PARTIAL_MAX_SPLIT K ranges
                    _SK_PARTIAL.setdefault((e["N"], e["K"]), []).append((e["M"], pp))


def _sk_tuned() -> dict:
    """(N, K) -> [(M, (bn, grid, dp, split)), ...] from scripts/tune_gemm_sk.py's measurements."""
    if _SK_TUNED is None:
        _sk_load()
    return _SK_TUNED


def _sk_partial() -> dict:
    """(N, K) -> [(M, [bn, split] | None), ...]: residual projections measured both ways."""
    if _SK_PARTIAL is None:
        _sk_load()
    return _SK_PARTIAL


@functools.lru_cache(maxsize=4096)
def gemm_sk_plan(M: int, N: int, K: int, tuned: bool = True) -> tuple:
    """(bn, grid, dp, split, bm) for ``gemm_sk``. Grid = one workgroup per CU (the kernel holds
    ~136-144 KiB of LDS). Whole tiles go out in data-parallel rounds; the remainder either as
    equal K splits (concurrent workgroups stream the same K offsets: L2 reuse) or by stream-K.

    ``tuned``: a shape measured by scripts/tune_gemm_sk.py (same N, K and the same number of
    128-row tiles, nearest M) takes its measured winner (bm = 256 unless the entry says 128). Otherwise a cost model: per 64-deep K
    step ~1.5 us for a 256x256 tile, ~1.1 us for 256x128 (scripts/bench_gemm_sk.py); stream-K's
    staggered K offsets lose ~2x of that to L2 misses; every extra partial costs one 256 x bn
    fp32 slab read (~100 GB/s per workgroup)."""
    if tuned:
        m128 = -(-M // 128)
        cands = [(abs(m - M), cfg) for m, cfg in _sk_tuned().get((N, K), ()) if -(-m // 128) == m128]
        if cands:
            cfg = min(cands)[1]
            if N % (16 if cfg[0] == 192 else cfg[0]) == 0:
                return (cfg[0], N_CU, cfg[2], cfg[3], cfg[4] if len(cfg) > 4 else SK_BM)
    nkt = K // 64
    best = None
    # per 64-deep K step: 256 x bn tiles ~1.5 / 1.2 / 1.1 us; 128 x bn ~0.72x that (the step is bound
    # by the (bm + bn) x 64 operand bytes each workgroup stages, not by its MFMAs)
    for bm, f in ((256, 1.0), (128, 0.72)):
        mt = -(-M // bm)
        for bn, c_it in ((256, 1.5 * f), (192, 1.2 * f), (128, 1.1 * f)):
            if N % (16 if bn == 192 else bn):
                continue
            tiles = mt * -(-N // bn)
            rounds, rem = divmod(tiles, N_CU)
            slab_us = bm * bn * 4 / 100e3
            cands = [(rounds * nkt * c_it if rem == 0 else float("inf"), (bn, N_CU, 1, 0, bm))]
            if rem:
                for sp in range(1, min(8, nkt, N_CU // rem) + 1):
                    t = (rounds * nkt + -(-nkt // sp)) * c_it + (sp - 1) * slab_us
                    cands.append((t, (bn, N_CU, 1, sp, bm)))
                per = rem * nkt / N_CU
                cands.append(((rounds * nkt + per) * c_it + per * c_it + 2 * slab_us, (bn, N_CU, 1, 0, bm)))
            for c in cands:
                if best is None or c[0] < best[0] - 1e-9:
                    best = c
    return best[1]


def gemm_sk(a: torch.Tensor, wp: torch.Tensor, M: int, N: int, K: int, epi: int, ep: EpiArgs,
            bn: int = 0, grid: int = 0, dp: int = 1, group_m: int = 8, nb: int = 0, split: int = -1,
            ws: Optional[SkWorkspace] = None, bm: int = 0, out_numel: int = 0) -> None:
    """Projection GEMM for any M (gemm_sk.hip): ``bm`` x ``bn`` tiles (bm 256 / 128), LDS-DMA
    staged, data-parallel rounds + stream-K, fused epilogue. ``wp`` = pack_b(W[N, K]); K % 64
    == 0; N % bn == 0 for bn = 128 / 256, N % 16 == 0 for bn = 192 (partial last column tile).
    bn = bm = 0: the plan's (gemm_sk_plan). EPI_PARTIAL writes ``split`` x M x ldo fp32 values
    to ``ep.out``: ``out_numel`` (its capacity in floats) is required and checked first."""
    _req(_is_bf16_cuda(a, wp), "gemm_sk: bf16 cuda tensors required")
    _req(wp.numel() == N * K and K % 64 == 0 and K >= 64, "gemm_sk: packed weight shape")
    _req(a.dim() == 2 and a.shape[0] >= M >= 1 and a.shape[1] >= K and a.stride(1) == 1 and a.stride(0) % 8 == 0,
         "gemm_sk: A must be [>=M, >=K] row-major with 16-B aligned rows")
    _req(a.data_ptr() % 16 == 0, "gemm_sk: A must be 16-byte aligned")
    _check_epi(epi, ep, N)
    _req(epi in (EPI_STORE, EPI_RESID, EPI_SWIGLU, EPI_QKV, EPI_PARTIAL, EPI_ARGMAX), f"gemm_sk: epilogue {epi} not supported")
    if epi == EPI_PARTIAL:  # exactly `split` K ranges per tile, every tile in one round
        _req(bn in (128, 192, 256) and split >= 1 and grid >= 1, "gemm_sk partial: explicit bn, grid and split required")
        _req(out_numel >= split * M * ep.ldo, f"gemm_sk partial: output holds {out_numel} floats, "
             f"split {split} x {M} rows x ldo {ep.ldo} needed")
    pb, pg, pd, ps, pm = gemm_sk_plan(M, N, K)
    if ep.ss_out and pb == 192:  # the fused-norm partials are per 64 columns of one wave (TN = 64)
        pb = 256 if N % 256 == 0 else 128
    if epi == EPI_ARGMAX:
        # the argmax epilogue reduces over power-of-two lane groups; whole-K tiles only, so every
        # logit is summed in the same order whatever N range (split lm_head) it is computed in
        if pb == 192:
            pb = 256 if N % 256 == 0 else 128
        ps = split = 1
    if not bn:
        bn, grid, split = pb, grid or pg, ps if split < 0 else split
        bm = bm or pm
    bm = bm or SK_BM
    grid = grid or pg
    if split < 0:
        split = 0
    _req(bn in (128, 192, 256) and N % (16 if bn == 192 else bn) == 0 and (bn != 192 or epi != EPI_SWIGLU or N % 32 == 0),
         f"gemm_sk: N={N} does not tile by bn={bn}")
    _req(1 <= grid <= 1024, "gemm_sk: grid")
    if ws is None:
        ws = default_sk_workspace(a.device)
    _req(bm in (128, 256), "gemm_sk: bm")
    _req(ws.slab.numel() >= 2 * grid * bm * bn and ws.counters.numel() >= 2 * grid,
         f"gemm_sk: workspace too small for grid={grid} bn={bn}")
    rc = lib().lsa_gemm_sk(_p(a), a.stride(0), _p(wp), M, N, K, epi, ctypes.byref(ep), bm, bn, nb, grid, dp, split, group_m,
                           _p(ws.slab), _p(ws.counters), ws.slab.numel(), ws.counters.numel(), _stream())
    _check(rc, "lsa_gemm_sk")


# ------------------------------------------------------------------------------ attention
def attn(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, slot: torch.Tensor,
         pos: torch.Tensor, rows: int, n_heads: int, n_kv: int, head_dim: int, nsplit: int,
         part_o: torch.Tensor, part_lse: torch.Tensor, out: torch.Tensor,
         kv_len: Optional[torch.Tensor] = None, min_chunk: int = 64,
         scale: Optional[float] = None, counters: Optional[torch.Tensor] = None) -> None:
    """Split-KV attention of ``rows`` query rows against the static cache; with nsplit > 1 the
    last-arriving split of each (row, kv-head) merges the partials in-kernel. ``counters``:
    >= rows * n_kv zeroed int32 (left zeroed; default: the stream's coop workspace)."""
    _req(_is_bf16_cuda(q, k_cache, v_cache, out), "attn: bf16 cuda tensors")
    _req(k_cache.dim() == 4 and k_cache.shape == v_cache.shape, "attn: cache [slots, n_kv, T, hd]")
    _req(k_cache.shape[1] == n_kv and k_cache.shape[3] == head_dim, "attn: cache dims")
    _req(q.shape[0] >= rows and q.shape[1] >= n_heads * head_dim, "attn: q shape")
    _req(part_o.numel() >= rows * n_heads * nsplit * head_dim and part_lse.numel() >= rows * n_heads * nsplit,
         "attn: workspace too small")
    _req(part_o.dtype == torch.float32 and part_lse.dtype == torch.float32, "attn: fp32 workspace")
    _req(slot.dtype == torch.int32 and pos.dtype == torch.int32, "attn: int32 slot/pos")
    t_max = k_cache.shape[2]
    sc = head_dim ** -0.5 if scale is None else scale
    g = n_heads // n_kv
    if 2 <= g <= 16 and rows * n_kv >= ATTN_MFMA_MIN_ITEMS and ATTN_MFMA:
        # GQA with enough (row, kv-head) work items to fill the GPU unsplit: the MFMA kernel
        # (attn_prefill.hip gqa_decode_kernel: the G query heads are the MFMA columns, one K/V
        # stream per item serves all of them)
        rc = lib().lsa_attn_decode_mfma(_p(q), q.stride(0), _p(k_cache), _p(v_cache), _p(slot), _p(pos), _p(kv_len),
                                        rows, n_heads, n_kv, head_dim, t_max, float(sc), _p(out), out.stride(0),
                                        ATTN_GQA_NW, _stream())
        _check(rc, "lsa_attn_decode_mfma")
        return
    if nsplit > 1 and counters is None:
        counters = default_workspace(q.device).counters
    _req(nsplit == 1 or (counters.dtype == torch.int32 and counters.numel() >= rows * n_kv),
         "attn: counters too small")
    rc = lib().lsa_attn_decode(_p(q), q.stride(0), _p(k_cache), _p(v_cache), _p(slot), _p(pos), _p(kv_len),
                               rows, n_heads, n_kv, head_dim, t_max, float(sc), nsplit, min_chunk,
                               _p(part_o), _p(part_lse), _p(out), out.stride(0),
                               _p(counters) if nsplit > 1 else None, _stream())
    _check(rc, "lsa_attn_decode")


def attn_oproj(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, slot: torch.Tensor,
               pos: torch.Tensor, n_heads: int, n_kv: int, head_dim: int, attn_out: torch.Tensor,
               wp: torch.Tensor, N: int, ep: EpiArgs, sync: torch.Tensor, kv_len: Optional[torch.Tensor] = None,
               scale: Optional[float] = None, max_wg: int = 0) -> bool:
    """Batch-1 decode attention fused with the o projection and its residual add
    (attn_oproj.hip): ``attn_out`` [1][K] gets the attention output, ``ep`` (EPI_RESID: out, resid)
    gets resid + attn_out @ Wo^T, ``wp`` = pack_b(Wo) [N, K], K = n_heads * head_dim. ``sync``:
    >= 4 zeroed int32, left zeroed; sync[2] != 0 afterwards means an arrival poll timed out.
    ``max_wg`` caps the grid (0: one workgroup per CU). False when no instantiation covers the
    shape (the caller then runs :func:`attn` + :func:`gemv`)."""
    K = n_heads * head_dim
    _req(_is_bf16_cuda(q, k_cache, v_cache, attn_out, wp), "attn_oproj: bf16 cuda tensors")
    _req(k_cache.dim() == 4 and k_cache.shape == v_cache.shape, "attn_oproj: cache [slots, n_kv, T, hd]")
    _req(k_cache.shape[1] == n_kv and k_cache.shape[3] == head_dim, "attn_oproj: cache dims")
    _req(q.shape[0] >= 1 and q.shape[1] >= K and q.stride(1) == 1, "attn_oproj: q shape")
    _req(attn_out.is_contiguous() and attn_out.numel() >= K, "attn_oproj: attn_out")
    _req(wp.numel() == N * K and N % 16 == 0, "attn_oproj: packed weight shape")
    _req(slot.dtype == torch.int32 and pos.dtype == torch.int32, "attn_oproj: int32 slot/pos")
    _req(sync.dtype == torch.int32 and sync.is_cuda and sync.numel() >= 4, "attn_oproj: sync")
    _req(bool(ep.out) and bool(ep.resid), "attn_oproj: EPI_RESID epilogue needs out and resid")
    sc = head_dim ** -0.5 if scale is None else scale
    rc = lib().lsa_attn_oproj(_p(q), q.stride(0), _p(k_cache), _p(v_cache), _p(slot), _p(pos), _p(kv_len),
                              n_heads, n_kv, head_dim, k_cache.shape[2], float(sc), _p(attn_out), _p(wp), N, K,
                              ctypes.byref(ep), _p(sync), int(max_wg), _stream())
    if rc == _UNSUPPORTED:
        return False
    _check(rc, "lsa_attn_oproj")
    return True


# GQA decode attention on MFMA (lsa_attn_decode_mfma) from this many (row, kv-head) items up;
# below it the split-KV VALU kernel, which spreads long contexts over more workgroups
ATTN_MFMA_MIN_ITEMS = int(os.environ.get("LSA_ATTN_MFMA_MIN_ITEMS", "512"))
ATTN_MFMA = os.environ.get("LSA_ATTN_MFMA", "1") == "1"
ATTN_GQA_NW = int(os.environ.get("LSA_ATTN_GQA_NW", "0"))  # waves per (row, kv-head) item: 1 / 2 / 4 (0 = 1)

PREFILL_TILE_ROWS = 128  # positions per tile with one query head per workgroup


def prefill_tile_rows(n_heads: int, n_kv: int, rows: int = 0) -> int:
    """Positions per flash-prefill tile: 8 waves x 16 rows shared by the GQA group's heads
    that one workgroup covers (all G of them when G divides 8; lsa_prefill_tile_rows). With
    ``rows`` (the prefill's total query rows) the tile is halved, down to 16 positions, while
    the (tile, head-group) work items would leave CUs idle - a 512-token 7B prompt gets 256
    items of 64 positions instead of 128 of 128."""
    g = n_heads // n_kv
    hpw = g if 8 % g == 0 else 1
    t = PREFILL_TILE_ROWS // hpw
    while rows and t > 16 and -(-rows // t) * (n_heads // hpw) < N_CU:
        t //= 2
    return t


def build_prefill_tiles(slot, pos, kv_len=None, device=None, tile_rows: int = PREFILL_TILE_ROWS):
    """Host-side tile table for :func:`attn_prefill`: rows are grouped into runs of one
    sequence (same slot, consecutive positions) and each run is cut into <= ``tile_rows``-row
    tiles ``[row0, nrows, slot, pos0, kvlen, 0, 0, 0]`` (int32; ``tile_rows`` =
    :func:`prefill_tile_rows` of the model). Causal tiles get ``kvlen = last position + 1``;
    with an explicit per-row ``kv_len`` (the reference's unmasked prefill) every row of a run
    must share it. Heaviest tiles first (balance)."""
    slot = [int(x) for x in (slot.tolist() if torch.is_tensor(slot) else slot)]
    pos = [int(x) for x in (pos.tolist() if torch.is_tensor(pos) else pos)]
    kvl = None if kv_len is None else [int(x) for x in (kv_len.tolist() if torch.is_tensor(kv_len) else kv_len)]
    tiles = []
    r, n = 0, len(slot)
    while r < n:
        e = r + 1
        while (e < n and slot[e] == slot[r] and pos[e] == pos[e - 1] + 1 and e - r < tile_rows
               and (kvl is None or kvl[e] == kvl[r])):
            e += 1
        kv = pos[e - 1] + 1 if kvl is None else kvl[r]
        tiles.append([r, e - r, slot[r], pos[r], kv, 0, 0, 0])
        r = e
    tiles.sort(key=lambda t: -t[4])
    return torch.tensor(tiles, dtype=torch.int32, device=device)


_TILES_OK = None  # the last tile table attn_prefill validated (identity + the bounds it was checked against)


def attn_prefill(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, tiles: torch.Tensor,
                 n_heads: int, n_kv: int, head_dim: int, out: torch.Tensor, causal: bool = True,
                 scale: Optional[float] = None, tiles_host: Optional[torch.Tensor] = None) -> None:
    """Flash prefill attention (attn_prefill.hip) for the rows described by ``tiles``
    (:func:`build_prefill_tiles`), reading K/V already appended to the static cache."""
    _req(_is_bf16_cuda(q, k_cache, v_cache, out), "attn_prefill: bf16 cuda tensors")
    _req(k_cache.dim() == 4 and k_cache.shape == v_cache.shape, "attn_prefill: cache [slots, n_kv, T, hd]")
    _req(k_cache.shape[1] == n_kv and k_cache.shape[3] == head_dim and head_dim in (64, 128), "attn_prefill: dims")
    _req(n_heads % n_kv == 0 and q.shape[1] >= n_heads * head_dim and out.shape[1] >= n_heads * head_dim,
         "attn_prefill: q/out width")
    _req(tiles.dtype == torch.int32 and tiles.is_cuda and tiles.dim() == 2 and tiles.shape[1] == 8,
         "attn_prefill: tiles int32 [n, 8]")
    th = tiles.cpu() if tiles_host is None else tiles_host
    slots, t_max = k_cache.shape[0], k_cache.shape[2]
    # a forward validates its tile table once, not once per layer (~40 us of host time each)
    # (the validated table object itself is held, so its identity cannot be reused by a new one)
    key = (tiles.data_ptr(), n_heads, n_kv, q.shape[0], out.shape[0], slots, t_max)
    global _TILES_OK
    if th.numel() and not (_TILES_OK is not None and _TILES_OK[0] is th and _TILES_OK[1] == key):
        row0, nr, sl, p0, kv = (th[:, i] for i in range(5))
        _req(bool((nr >= 1).all() and (nr <= prefill_tile_rows(n_heads, n_kv)).all()), "attn_prefill: tile rows")
        _req(bool((row0 >= 0).all()) and int((row0 + nr).max()) <= min(q.shape[0], out.shape[0]),
             "attn_prefill: tile rows out of range")
        _req(bool((sl >= 0).all() and (sl < slots).all()), "attn_prefill: slot out of range")
        _req(bool((p0 >= 0).all()) and int((p0 + nr).max()) <= t_max, "attn_prefill: positions beyond cache")
        _req(bool((kv >= 1).all() and (kv <= t_max).all()), "attn_prefill: kvlen out of range")
        _TILES_OK = (th, key)
    sc = head_dim ** -0.5 if scale is None else scale
    rc = lib().lsa_attn_prefill(_p(q), q.stride(0), _p(k_cache), _p(v_cache), _p(tiles), tiles.shape[0], n_heads,
                                n_kv, head_dim, t_max, float(sc), int(causal), _p(out), out.stride(0), _stream())
    _check(rc, "lsa_attn_prefill")


# ------------------------------------------------------------------------------ elementwise
def embed(ids: torch.Tensor, table: torch.Tensor, out: torch.Tensor, rows: Optional[int] = None) -> None:
    rows = ids.numel() if rows is None else rows
    _req(ids.dtype == torch.int32 and ids.is_cuda, "embed: int32 ids")
    _req(_is_bf16_cuda(table, out) and out.shape[1] >= table.shape[1], "embed: shapes")
    rc = lib().lsa_embed(_p(ids), rows, _p(table), table.shape[1], _p(out), out.stride(0), _stream())
    _check(rc, "lsa_embed")


def row_ss(h: torch.Tensor, rows: int, ss: torch.Tensor) -> None:
    """ss[r][b] = sum of squares of h[r, 64b:64b+64] (fp32) for the fused RMSNorm of gemm_sk."""
    _req(_is_bf16_cuda(h) and ss.dtype == torch.float32 and ss.shape[1] * 64 == h.shape[1], "row_ss: shapes")
    rc = lib().lsa_row_ss(_p(h), h.stride(0), rows, h.shape[1], _p(ss), _stream())
    _check(rc, "lsa_row_ss")


def resid_rmsnorm_partials(h: torch.Tensor, partials: torch.Tensor, S: int, rows: int, eps: float,
                           out: Optional[torch.Tensor] = None, w: Optional[torch.Tensor] = None) -> None:
    """h[:rows] = bf16(h + sum_s partials[s]) (fixed order), then ``out`` = rmsnorm(h) [* w]
    (no norm when ``out`` is None). ``partials``: fp32 [S_alloc, >= rows, H] written by
    ``gemm_sk(..., EPI_PARTIAL, split=S)`` with ldo = H (elementwise.hip)."""
    H = h.shape[1]
    _req(_is_bf16_cuda(h, w, out) and partials.dtype == torch.float32 and partials.is_cuda, "resid_rmsnorm_partials: dtypes")
    _req(partials.dim() == 3 and partials.shape[0] >= S and partials.shape[2] == H and partials.is_contiguous()
         and partials.shape[1] >= rows, "resid_rmsnorm_partials: partials must be [>=S, >=rows, H] contiguous")
    # the GEMM wrote partial k at k * rows * H (its M = rows), not at the allocation's stride
    rc = lib().lsa_resid_rmsnorm_partials(_p(h), h.stride(0), _p(partials), S, rows * H, H, _p(w), rows, H, float(eps),
                                          _p(out), 0 if out is None else out.stride(0), _stream())
    _check(rc, "lsa_resid_rmsnorm_partials")


def gemm_sk_partial_plan(M: int, N: int, K: int) -> Optional[tuple]:
    """(bn, split) for a residual projection run as EPI_PARTIAL + resid_rmsnorm_partials, or
    None when the fused EPI_RESID plan is better. Tuned shapes carry a measured ``partial``
    entry (scripts/tune_gemm_sk.py); otherwise None (no partials above PARTIAL_MAX_ROWS)."""
    if M > PARTIAL_MAX_ROWS:
        return None
    if _PARTIAL_FORCE is not None:  # force_partial_plan(): tests pin the mode
        return None if _PARTIAL_FORCE is False else _PARTIAL_FORCE
    mt = -(-M // SK_BM)
    cands = [(abs(m - M), pp) for m, pp in _sk_partial().get((N, K), ()) if -(-m // SK_BM) == mt]
    if not cands:
        return None
    pp = min(cands)[1]
    return None if pp is None else tuple(pp)


PARTIAL_MAX_ROWS = 1024   # rows of the engine's split-K partial buffer
PARTIAL_MAX_SPLIT = 8
_PARTIAL_FORCE = None


@contextmanager
def force_partial_plan(plan):
    """Within the block every residual projection of <= PARTIAL_MAX_ROWS rows uses ``plan``
    ((bn, split), or False for the fused EPI_RESID path) instead of the tuning table."""
    global _PARTIAL_FORCE
    prev, _PARTIAL_FORCE = _PARTIAL_FORCE, plan
    try:
        yield
    finally:
        _PARTIAL_FORCE = prev


def rmsnorm(x: torch.Tensor, w: Optional[torch.Tensor], out: torch.Tensor, rows: int, eps: float,
            H: Optional[int] = None) -> None:
    """out = x * rsqrt(mean(x^2)+eps) [* w]. ``w=None``: weight folded into the next GEMM."""
    H = w.numel() if w is not None else (H or x.shape[1])
    _req(_is_bf16_cuda(x, w, out), "rmsnorm: bf16 cuda tensors")
    rc = lib().lsa_rmsnorm(_p(x), x.stride(0), _p(w), rows, H, float(eps), _p(out), out.stride(0), _stream())
    _check(rc, "lsa_rmsnorm")


def layernorm(x: torch.Tensor, out: torch.Tensor, w: torch.Tensor, b: torch.Tensor, rows: int, eps: float,
              pos_emb: Optional[torch.Tensor] = None, pos: Optional[torch.Tensor] = None) -> None:
    """out = LayerNorm(x) * w + b (GPT-2). With ``pos_emb``: first ``x += pos_emb[pos]`` in
    place (learned absolute positions, bf16-rounded as HF does)."""
    H = w.numel()
    _req(_is_bf16_cuda(x, w, b, out) and b.numel() == H and x.shape[1] >= H, "layernorm: bf16 cuda tensors")
    if pos_emb is not None:
        _req(pos is not None and pos.dtype == torch.int32 and pos.numel() >= rows and pos_emb.shape[1] == H,
             "layernorm: pos_emb needs int32 positions")
    rc = lib().lsa_layernorm(_p(x), x.stride(0), _p(pos_emb), _p(pos), _p(w), _p(b), rows, H, float(eps),
                             _p(out), out.stride(0), _stream())
    _check(rc, "lsa_layernorm")


def argmax_finalize(keys: torch.Tensor, rows: int, tokens: torch.Tensor, pos: Optional[torch.Tensor] = None,
                    pos_inc: int = 1, history: Optional[torch.Tensor] = None,
                    step_ctr: Optional[torch.Tensor] = None) -> None:
    _req(keys.dtype == torch.int64 and tokens.dtype == torch.int32, "argmax_finalize: dtypes")
    hs = history.stride(0) if history is not None else 0
    hl = history.shape[0] if history is not None else 0
    if history is not None:
        _req(history.dtype == torch.int32 and history.shape[1] >= rows, "argmax_finalize: history shape")
    rc = lib().lsa_argmax_finalize(_p(keys), rows, _p(tokens), _p(pos), pos_inc, _p(history), hs, hl,
                                   _p(step_ctr), _stream())
    _check(rc, "lsa_argmax_finalize")


def pos_advance(pos: torch.Tensor, rows: int, inc: int = 1) -> None:
    rc = lib().lsa_pos_advance(_p(pos), rows, inc, _stream())
    _check(rc, "lsa_pos_advance")
