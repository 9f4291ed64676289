"""Which kernel runs a projection: ONE route table keyed by (N, K, row range), with one fallback rule.

The reference runs every projection through ``nn.Linear`` (cuBLAS; /root/reference/utils/shard_loader.py:66-74).
Here three hand-written kernel families compete, and which wins depends on the shape and the row
count. Measured winners that differ from the fallback are listed in ``ROUTES``; everything else
follows ``FALLBACK``:

* rows <= 128 (decode): the weight-streaming GEMVs (gemv.hip up to 16 rows, gemv_coop.hip 17-128)
  with the RMSNorm fused in (``norm=True``); their launch parameters per shape come from
  ops/gemv_tuning.json, or the analytic default (ops/packing.py) for an unlisted shape;
* rows > 128: the stream-K LDS-DMA MFMA GEMM (gemm_sk.hip), decomposition from
  ops/gemm_sk_tuning.json, or the analytic planner (ops/hip.gemm_sk_plan) for an unlisted shape.

So a new model runs correctly and reasonably fast with no entry at all; an entry only records a
measured improvement, with the profile that measured it. The tuning JSONs hold the PARAMETERS of
the chosen kernel; this table chooses the kernel.

The row-count decision of a whole layer (GEMV family vs GEMM family) is made once per forward,
because the fused RMSNorm chain differs between the families (GEMV: norm inside the kernel; GEMM:
per-64-column sums of squares from the residual epilogues, ``ss_in`` / ``ss_out``):
``layer_family`` sends a layer to the GEMM family when any of its projection shapes routes there.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Optional

GEMV_MAX_ROWS = 128  # = packing.GEMV_MAX_ROWS: the largest decode batch the GEMV kernels and decode graphs take


@dataclass(frozen=True)
class Route:
    N: int
    K: int
    lo: int             # row range [lo, hi] (inclusive)
    hi: int
    kernel: str         # "gemm_wr" | "gemm_sk" | "gemv"
    params: dict = field(default_factory=dict)
    epis: tuple = ()    # epilogues the route applies to (empty: any)
    evidence: str = ""


# EPI codes (= ops/hip.EPI_*; not imported to keep this module free of the ctypes library)
EPI_STORE, EPI_RESID, EPI_SWIGLU, EPI_QKV = 0, 1, 2, 3
_WR_EPIS = (EPI_STORE, EPI_QKV, EPI_SWIGLU)

ROUTES = (
    # ---- gemm_wr (weights straight to MFMA registers): where one round of whole 128 x bn tiles
    # fills the chip. Llama-2-7B qkv
    Route(12288, 4096, 193, 256, "gemm_wr", {"bn": 128}, _WR_EPIS, "profiles/r4_gemm_wr_shapes.jsonl"),
    Route(12288, 4096, 320, 512, "gemm_wr", {"bn": 192}, _WR_EPIS,
          "README: 7B qkv at 512 rows 57 vs 68 us on gemm_sk; profiles/r5_gemm_pmc.md"),
    # Llama-2-13B qkv
    Route(15360, 5120, 193, 256, "gemm_wr", {"bn": 128}, _WR_EPIS, "profiles/r4_gemm_wr_shapes.jsonl"),
    Route(15360, 5120, 320, 384, "gemm_wr", {"bn": 192}, _WR_EPIS, "profiles/r4_gemm_wr_shapes.jsonl"),
    Route(15360, 5120, 448, 512, "gemm_wr", {"bn": 256}, _WR_EPIS, "profiles/r4_gemm_wr_shapes.jsonl"),
    # Llama-3.2-3B qkv and gate_up (SwiGLU epilogue)
    Route(5120, 3072, 193, 512, "gemm_wr", {"bn": 128}, _WR_EPIS, "profiles/r4_gemm_wr_engine_ab.txt"),
    Route(16384, 3072, 193, 256, "gemm_wr", {"bn": 128}, _WR_EPIS, "profiles/r4_gemm_wr_engine_ab.txt"),
    Route(16384, 3072, 320, 512, "gemm_wr", {"bn": 256}, _WR_EPIS, "profiles/r4_gemm_wr_engine_ab.txt"),
    # 7B / 13B gate_up at 193-256 rows
    Route(22016, 4096, 193, 256, "gemm_wr", {"bn": 256}, _WR_EPIS, "profiles/r4_gemm_wr_shapes.jsonl"),
    Route(27648, 5120, 193, 256, "gemm_wr", {"bn": 256}, _WR_EPIS, "profiles/r4_gemm_wr_shapes.jsonl"),
    # ---- the MFMA GEMMs below the GEMV limit: Llama-2-13B's 65-128-row decode (-4.6..5.6 % per
    # step on three boxes); the 7B (+6 %), 3B (+65 %) and 70B stage (+6-10 %) measured slower there
    Route(15360, 5120, 65, 128, "gemm_sk", {}, (), "profiles/r5_gemv_max_rows_ab.md"),
    Route(5120, 5120, 65, 128, "gemm_sk", {}, (), "profiles/r5_gemv_max_rows_ab.md"),
    Route(27648, 5120, 65, 128, "gemm_sk", {}, (), "profiles/r5_gemv_max_rows_ab.md"),
    Route(5120, 13824, 65, 128, "gemm_sk", {}, (), "profiles/r5_gemv_max_rows_ab.md"),
)


def fallback(M: int) -> Route:
    """The kernel family of a shape the table does not list."""
    return Route(0, 0, 1, GEMV_MAX_ROWS, "gemv") if M <= GEMV_MAX_ROWS else Route(0, 0, GEMV_MAX_ROWS + 1, 1 << 30,
                                                                                    "gemm_sk")


def route(M: int, N: int, K: int, epi: Optional[int] = None) -> Route:
    """The kernel for an [M, K] x [K, N] projection with epilogue ``epi``."""
    for r in ROUTES:
        if r.N == N and r.K == K and r.lo <= M <= r.hi and (epi is None or not r.epis or epi in r.epis):
            return r
    return fallback(M)


def layer_family(M: int, shapes) -> str:
    """'gemv' or 'gemm' for a layer whose projections are ``shapes`` [(N, K), ...] at M rows.
    LSA_GEMV_MAX_ROWS (diagnostic) overrides: GEMV up to that many rows."""
    env = os.environ.get("LSA_GEMV_MAX_ROWS")
    if env:
        return "gemv" if M <= int(env) else "gemm"
    if M > GEMV_MAX_ROWS:
        return "gemm"
    return "gemm" if any(route(M, N, K).kernel != "gemv" for N, K in shapes) else "gemv"


def gemv_max_rows(shapes) -> int:
    """The largest row count <= GEMV_MAX_ROWS at which a layer of ``shapes`` still runs the GEMVs
    (StageEngine.GEMV_MAX_ROWS per model)."""
    m = GEMV_MAX_ROWS
    while m > 0 and layer_family(m, shapes) == "gemm":
        m -= 1
    return m
