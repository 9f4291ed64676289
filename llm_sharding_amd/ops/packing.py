"""Weight packing for the gfx950 projection kernels (csrc/kernels/common.h).

``pack_b`` rearranges a torch ``nn.Linear`` weight ``W[N, K]`` into the
v_mfma_f32_16x16x32_bf16 B-fragment order::

    Wp[nt][kt][lane][j] = W[nt*16 + (lane & 15)][kt*32 + 8*(lane >> 4) + j]

Fused matrices (built once at shard-load time, replacing the reference's separate
q/k/v and gate/up ``nn.Linear`` modules inside HF ``LlamaDecoderLayer``):

* QKV: rows ``[q; k; v]``; q and k rows are permuted per head so that each 16-row tile
  holds dims ``8t..8t+7`` and their rotate_half partners ``hd/2+8t..`` (the RoPE epilogue
  then finds a partner at column ``n ^ 8``).
* gate/up: 16-row tiles interleaved ``g0 u0 g1 u1 ...`` so one workgroup owns both halves of
  a SwiGLU output tile.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch


def pack_b(w: torch.Tensor) -> torch.Tensor:
    N, K = w.shape
    if N % 16 or K % 32:
        raise ValueError(f"pack_b needs N%16==0 and K%32==0, got {tuple(w.shape)}")
    return w.contiguous().view(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(N // 16, K // 32, 64, 8)


def unpack_b(wp: torch.Tensor) -> torch.Tensor:
    NT, KT = wp.shape[0], wp.shape[1]
    return wp.view(NT, KT, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(NT * 16, KT * 32)


def rope_head_perm(head_dim: int) -> list:
    half = head_dim // 2
    out = []
    for tt in range(head_dim // 16):
        for cc in range(16):
            out.append(8 * tt + cc if cc < 8 else half + 8 * tt + (cc - 8))
    return out


def rope_rows_perm(n_heads: int, head_dim: int) -> torch.Tensor:
    p = torch.tensor(rope_head_perm(head_dim), dtype=torch.long)
    return torch.cat([p + h * head_dim for h in range(n_heads)])


def fuse_qkv(wq: torch.Tensor, wk: torch.Tensor, wv: torch.Tensor, n_heads: int, n_kv: int,
             head_dim: int) -> torch.Tensor:
    pq = rope_rows_perm(n_heads, head_dim).to(wq.device)
    pk = rope_rows_perm(n_kv, head_dim).to(wk.device)
    return torch.cat([wq.index_select(0, pq), wk.index_select(0, pk), wv], dim=0)


def fuse_gate_up(wg: torch.Tensor, wu: torch.Tensor) -> torch.Tensor:
    I, H = wg.shape
    if I % 16:
        raise ValueError("intermediate_size must be a multiple of 16")
    return torch.stack([wg.view(I // 16, 16, H), wu.view(I // 16, 16, H)], dim=1).reshape(2 * I, H)


def fold_norm(w: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """``W' = W * diag(g)`` (fp32 product, rounded once): RMSNorm's weight folded into the
    following projection, so the decode GEMV applies only ``rsqrt(mean(x^2)+eps)`` per row."""
    return (w.float() * g.float()[None, :]).to(w.dtype)


N_CU = 256  # MI355X compute units

FP8 = getattr(torch, "float8_e4m3fn", None)  # OCP e4m3: the MI355X (gfx950) native fp8 encoding


def quantize_fp8_rows(w: torch.Tensor) -> tuple:
    """Per-output-row symmetric OCP e4m3: w ~= q * scale[:, None]. Returns (q uint8 [N, K], scale fp32 [N])."""
    amax = w.float().abs().amax(dim=1).clamp(min=1e-12)
    scale = amax / 448.0
    q = (w.float() / scale[:, None]).clamp(-448.0, 448.0).to(FP8)
    return q.view(torch.uint8), scale.float()


def dequantize_fp8_rows(q: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    return q.view(FP8).float() * scale.float()[:, None]


def pack_b_fp8(q: torch.Tensor) -> torch.Tensor:
    """fp8 bytes [N, K] (K % 64 == 0) -> Wq[nt][kt/2][lane][16]: per lane and 16-B load, the
    8 elements of MFMA B fragment 2*kt2 (bytes 0-7) and of fragment 2*kt2+1 (bytes 8-15), each
    in pack_b's element order."""
    N, K = q.shape
    if N % 16 or K % 64:
        raise ValueError(f"pack_b_fp8 needs N%16==0 and K%64==0, got {tuple(q.shape)}")
    p = q.contiguous().view(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(N // 16, K // 32, 64, 8)
    return p.view(N // 16, K // 64, 2, 64, 8).permute(0, 1, 3, 2, 4).reshape(N // 16, K // 64, 64, 16).contiguous()


# (tn, mb, nw, u2) instantiated in csrc/kernels/gemv_fp8.hip (LSA_FP8_CONFIGS) - keep in sync.
FP8_CONFIGS = [(1, 1, 4, 2), (1, 1, 8, 2), (1, 1, 4, 4), (2, 1, 4, 2), (2, 1, 8, 2), (4, 1, 4, 1),
               (1, 2, 4, 2), (1, 2, 8, 2), (2, 2, 4, 1), (2, 2, 8, 1), (1, 4, 4, 1), (1, 4, 8, 1), (2, 4, 4, 1),
               (2, 4, 8, 1)]


def fp8_gemv_candidates(n_tiles: int, k: int, rows: int, need_even: bool = False) -> list:
    mb = row_blocks(rows)
    return [(tn, nw, u2) for (tn, b, nw, u2) in FP8_CONFIGS
            if b == mb and n_tiles % tn == 0 and (not need_even or tn % 2 == 0) and (k // 32) % (2 * u2) == 0]


def fp8_config(n_tiles: int, rows: int, need_even: bool = False, k: int = 4096) -> tuple:
    """(tn, nw, u2) for the plain fp8 GEMV (rows <= 64): the candidate giving >= 256 workgroups
    with the most weight bytes in flight per wave."""
    cands = fp8_gemv_candidates(n_tiles, k, rows, need_even)
    if not cands:
        raise ValueError(f"no fp8 GEMV config for {n_tiles} tiles, K={k}, rows={rows}")

    def cost(c):
        tn, nw, u2 = c
        g = n_tiles // tn
        eff = g / (N_CU * -(-g // N_CU))
        return (1.0 + 0.4 * rows / (16.0 * tn)) / eff - 0.01 * (nw * u2 / 16.0)
    return min(cands, key=cost)


def fp8_proj_config(n_tiles: int, rows: int, need_even: bool = False, k: int = 4096) -> tuple:
    """("fp8", (tn, nw, u2)) [gemv_fp8.hip] or ("coop_fp8", (tnw, nw, kf, sk)) [gemv_coop.hip,
    fp8 weights] for a W8A16 projection of ``rows`` rows: the measured table if it has the
    shape, else the plain kernel up to 16 rows and the cooperative one above (it shares the
    activations through LDS instead of re-reading them per workgroup)."""
    t = _tuned().get((n_tiles * 16, k, row_blocks(rows), bool(need_even), "fp8"))
    if t is not None:
        algo, cfg = t
        if (algo == "fp8" and rows <= 64 and cfg in fp8_gemv_candidates(n_tiles, k, rows, need_even)) or \
           (algo == "coop_fp8" and cfg in coop_fp8_candidates(n_tiles, k, rows)):
            return t
    if rows > 16:
        cands = coop_fp8_candidates(n_tiles, k, rows)
        pref = [c for c in cands if c[:3] == (1, 8, 4)] or [c for c in cands if c[:2] == (1, 8)] or cands
        for c in pref:
            if (n_tiles // (c[0] * c[1])) * c[3] >= N_CU:
                return ("coop_fp8", c)
        if pref:
            return ("coop_fp8", pref[-1])
    return ("fp8", fp8_config(n_tiles, rows, need_even, k))


# (tn, mb, nw, u) instantiated in csrc/kernels/gemv.hip (LSA_GEMV_CONFIGS) - keep in sync.
GEMV_CONFIGS = [
    (1, 1, 4, 4), (1, 1, 8, 4), (1, 1, 16, 4), (1, 1, 4, 8), (1, 1, 8, 8),
    (1, 2, 4, 4), (1, 2, 8, 4), (1, 2, 16, 2), (1, 4, 4, 2), (1, 4, 8, 2),
    (2, 1, 4, 4), (2, 1, 8, 4), (2, 1, 16, 2), (2, 1, 8, 2), (2, 2, 4, 2),
    (2, 2, 8, 2), (2, 4, 4, 2), (2, 4, 8, 2), (4, 1, 4, 2), (4, 1, 8, 2),
    (4, 2, 4, 2), (4, 2, 8, 2), (4, 4, 4, 2),
]

_TUNED = None
# LSA_GEMV_TUNING (diagnostic): another table, for A/B runs of a candidate table against this one
TUNING_FILE = os.environ.get("LSA_GEMV_TUNING") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                "gemv_tuning.json")


def row_blocks(rows: int) -> int:
    return 1 if rows <= 16 else (2 if rows <= 32 else (4 if rows <= 64 else 8))


def gemv_candidates(n_tiles: int, k: int, rows: int, need_even: bool = False) -> list:
    mb = row_blocks(rows)
    return [(tn, nw, u) for (tn, b, nw, u) in GEMV_CONFIGS
            if b == mb and n_tiles % tn == 0 and (not need_even or tn % 2 == 0) and (k // 32) % u == 0]


# (mb, tnw, nw, kf, kw, d) instantiated in csrc/kernels/gemv_coop.hip (LSA_COOP_CONFIGS) - keep in sync.
# kw = k-groups of nw waves per workgroup (kw * nw waves stream the same nw * tnw tiles);
# d = register-ring depth (prefetch distance d - 1 chunks).
COOP_CONFIGS = [(2, 1, 8, 8, 1, 3), (4, 1, 8, 8, 1, 3), (2, 1, 8, 4, 1, 3), (4, 1, 8, 4, 1, 3), (2, 2, 8, 4, 1, 3),
                (4, 2, 8, 4, 1, 3), (2, 2, 4, 4, 1, 3), (4, 2, 4, 4, 1, 3), (8, 1, 8, 4, 1, 3), (8, 1, 8, 2, 1, 3),
                (8, 2, 4, 2, 1, 3), (2, 1, 4, 4, 1, 3), (4, 1, 4, 4, 1, 3), (2, 1, 4, 8, 1, 3), (8, 1, 4, 2, 1, 3),
                (2, 1, 4, 8, 2, 3), (4, 1, 4, 4, 2, 3), (4, 1, 4, 8, 2, 3), (4, 1, 8, 4, 2, 3), (4, 2, 4, 4, 2, 3),
                (8, 1, 4, 2, 2, 3), (8, 1, 4, 4, 2, 3), (4, 1, 4, 4, 4, 3), (4, 1, 2, 4, 2, 3), (4, 1, 2, 4, 1, 3),
                (2, 1, 2, 4, 2, 3), (8, 1, 2, 2, 2, 3),
                (8, 1, 3, 2, 1, 3), (8, 1, 3, 2, 2, 3), (8, 1, 6, 2, 1, 3), (8, 1, 1, 2, 2, 3), (8, 1, 1, 2, 4, 3),
                (8, 1, 2, 2, 1, 3), (4, 1, 3, 4, 1, 3), (4, 1, 3, 4, 2, 3),
                (8, 1, 8, 2, 1, 4), (8, 1, 8, 4, 1, 4), (4, 1, 8, 4, 1, 4), (2, 1, 8, 4, 1, 4), (2, 1, 4, 4, 1, 4)]
GEMV_MAX_ROWS = 128  # rows 65..128 are served by the coop kernel only
COOP_SPLITS = (1, 2, 4, 8, 16)


def coop_candidates(n_tiles: int, k: int, rows: int, need_even: bool = False) -> list:
    """(tnw, nw, kf, sk, kw, d) for the cooperative split-K GEMV (rows 17..128): every split
    (and every k-group of a split) keeps at least one K chunk of 32*kf, and kw > 1 needs the
    chunks to divide evenly over sk*kw. need_even (SwiGLU): an even tile count per workgroup.

    sk = 0 is the ragged mode (gemv_coop.hip): no K split, the tiles (SwiGLU: gate / up pairs)
    dealt evenly to one workgroup per CU, at most nw * tnw each - for tile counts that are not a
    multiple of a workgroup's tiles (Llama-2-7B gate_up: 1,376 tiles fill 172 CUs as groups of 8).
    Not for EPI_PARTIAL or fp8 weights; chosen only through the tuning table."""
    if rows <= 16:
        return []
    mb = row_blocks(rows)
    out = []
    for (b, tnw, nw, kf, kw, d) in COOP_CONFIGS:
        if b != mb or n_tiles % (tnw * nw) or k % (32 * kf) or (need_even and (tnw * nw) % 2):
            continue
        nch = k // (32 * kf)
        for sk in COOP_SPLITS:
            if nch < sk * kw or (kw > 1 and nch % (sk * kw)):
                continue
            if (n_tiles // (tnw * nw)) * sk <= 4 * N_CU:
                out.append((tnw, nw, kf, sk, kw, d))
    for (b, tnw, nw, kf, kw, d) in COOP_CONFIGS:  # ragged (sk = 0)
        p = 2 if need_even else 1
        units = n_tiles // p
        if (b == mb and kw == 1 and k % (32 * kf) == 0 and n_tiles % p == 0 and p % tnw == 0 and units >= N_CU
                and p * -(-units // N_CU) <= tnw * nw):
            out.append((tnw, nw, kf, 0, kw, d))
    return out


# (mb, tnw, nw, kf) with fp8 weights (LSA_COOP_FP8_CONFIGS in gemv_coop.hip) - keep in sync.
COOP_FP8_CONFIGS = [(2, 1, 8, 4), (4, 1, 8, 4), (2, 1, 4, 4), (4, 1, 4, 4), (8, 1, 8, 4), (8, 1, 4, 2), (2, 1, 8, 8),
                    (4, 1, 8, 8)]


def coop_fp8_candidates(n_tiles: int, k: int, rows: int) -> list:
    if rows <= 16:
        return []
    mb = row_blocks(rows)
    out = []
    for (b, tnw, nw, kf) in COOP_FP8_CONFIGS:
        if b != mb or n_tiles % (tnw * nw) or k % (32 * kf):
            continue
        for sk in COOP_SPLITS:
            if k // (32 * kf) >= sk and (n_tiles // (tnw * nw)) * sk <= 4 * N_CU:
                out.append((tnw, nw, kf, sk))
    return out


def coop_norm(cfg) -> tuple:
    """A coop config as the full (tnw, nw, kf, sk, kw, d) tuple: tables and callers written
    before k-groups / ring depths existed give 4 or 5 entries (kw = 1, d = 3)."""
    c = tuple(cfg)
    if len(c) == 4:
        c = c + (1,)
    if len(c) == 5:
        c = c + (3,)
    return c


def coop_slab_floats(n: int, rows: int, tnw: int, nw: int, kf: int, sk: int, kw: int = 1) -> int:
    """fp32 workspace a coop launch needs (0 when sk == 1)."""
    if sk <= 1:  # one split, or the ragged mode (sk = 0): no slab
        return 0
    mr = 16 * row_blocks(rows)
    return sk * n * mr + sk * (n // 16 // (tnw * nw)) * mr


def coop_workspace_need(shapes, max_rows: int = 64, even_n=()) -> tuple:
    """(slab floats, counters) that the decode projections ``shapes`` = [(N, K), ...] need at
    every row count up to ``max_rows`` under the configs :func:`proj_config` picks."""
    floats, groups = 0, 0
    for n, k in shapes:
        for rows in (32, 64, 128):
            if rows // 2 >= max_rows:
                continue
            algo, cfg = proj_config(n // 16, rows, need_even=(n, k) in even_n, k=k)
            if algo == "coop":
                tnw, nw, kf, sk = cfg[:4]
                floats = max(floats, coop_slab_floats(n, rows, tnw, nw, kf, sk))
                groups = max(groups, n // 16 // (tnw * nw))
    return floats, groups


def _tuned() -> dict:
    global _TUNED
    if _TUNED is None:
        _TUNED = {}
        if os.path.exists(TUNING_FILE):
            with open(TUNING_FILE) as f:
                for e in json.load(f).get("entries", []):
                    if e.get("algo") in ("fp8", "coop_fp8"):
                        _TUNED[(e["N"], e["K"], e["mb"], bool(e["even"]), "fp8")] = (e["algo"], tuple(e["cfg"]))
                    elif e.get("algo") == "coop_partial":
                        _TUNED[(e["N"], e["K"], e["mb"], False, "partial")] = (e["algo"], coop_norm(e["cfg"]))
                    else:
                        cfg = tuple(e["cfg"])
                        if e.get("algo") == "coop":
                            cfg = coop_norm(cfg)
                        _TUNED[(e["N"], e["K"], e["mb"], bool(e["even"]))] = (e.get("algo", "gemv"), cfg)
    return _TUNED


def partial_config(n_tiles: int, rows: int, k: int = 4096) -> Optional[tuple]:
    """(tnw, nw, kf, sk, kw, d) when a residual decode projection of ``rows`` rows is measured
    faster as coop EPI_PARTIAL (splits store fp32 tiles) + lsa_resid_rmsnorm_partials than with
    the in-kernel split reduction + residual epilogue (scripts/tune_coop_partial.py), else None."""
    t = _tuned().get((n_tiles * 16, k, row_blocks(rows), False, "partial"))
    if t is None or rows <= 16:
        return None
    cfg = tuple(t[1])
    return cfg if cfg in coop_candidates(n_tiles, k, rows) and 1 <= cfg[3] <= 8 else None


def proj_config(n_tiles: int, rows: int, need_even: bool = False, k: int = 4096) -> tuple:
    """("gemv", (tn, nw, u)) or ("coop", (tnw, nw, kf, sk, kw, d)) for a decode projection of ``rows``
    rows. The tuning table (measured on MI355X) wins; otherwise rows <= 16 use the
    weight-streaming GEMV and larger row counts the cooperative split-K kernel with the
    smallest split that fills the 256 CUs."""
    t = _tuned().get((n_tiles * 16, k, row_blocks(rows), bool(need_even)))
    if t is not None:
        algo, cfg = t
        if (algo == "coop" and cfg in coop_candidates(n_tiles, k, rows, need_even)) or \
           (algo == "gemv" and cfg in gemv_candidates(n_tiles, k, rows, need_even)):
            return t
    if rows > 16:
        allc = coop_candidates(n_tiles, k, rows, need_even)
        cands = []
        for pref in ((1, 8, 8), (1, 8, 4), (1, 8, 2)):
            cands = [c for c in allc if c[:3] == pref and c[3] >= 1 and c[4] == 1 and c[5] == 3]
            if cands:
                break
        cands = cands or [c for c in allc if c[3] >= 1]
        for c in cands:
            if (n_tiles // 8) * c[3] >= N_CU:
                return ("coop", c)
        if cands:
            return ("coop", cands[-1])
    if rows > 64:
        raise ValueError(f"no projection config for {n_tiles * 16}x{k} at {rows} rows")
    return ("gemv", gemv_config(n_tiles, rows, need_even, k))


def gemv_config(n_tiles: int, rows: int, need_even: bool = False, k: int = 4096) -> tuple:
    """(tn, nw, u) for the decode GEMV. Uses the on-device tuning table measured on MI355X
    (scripts/bench_kernels.py --tune) when the shape is in it, else a cost model:
    time ~ (weight bytes + A re-reads / 5) / grid efficiency, where each workgroup re-reads
    the whole A (rows x K) from L2 (~5x the HBM rate) and grid efficiency =
    workgroups / (256 CUs x rounds)."""
    t = _tuned().get((n_tiles * 16, k, row_blocks(rows), bool(need_even)))
    cands = gemv_candidates(n_tiles, k, rows, need_even)
    if t is not None and t[0] == "gemv" and t[1] in cands:
        return t[1]
    best, best_cost = None, float("inf")
    for tn, nw, u in cands:
        g = n_tiles // tn
        eff = g / (N_CU * -(-g // N_CU))
        cost = (1.0 + 0.2 * rows / (16.0 * tn)) / eff - 0.01 * (nw * u / 32.0)
        if cost < best_cost - 1e-9:
            best, best_cost = (tn, nw, u), cost
    if best is None:
        raise ValueError(f"no GEMV config for {n_tiles} tiles, K={k}, rows={rows}")
    return best


