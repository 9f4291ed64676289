"""Error metrics for comparing a kernel's output against an fp32 reference.

One global Frobenius relative error ``||a - b|| / ||b||`` cannot see a localized bug: at 512 x 12288
one fully zeroed 16 x 16 output tile (what a stream-K fix-up or a split-K ticket bug produces) moves
it by only sqrt(256 / 6.3 M) = 6.4e-3, under the 8e-3 gate of a bf16 GEMM test, and one row of a
1024-row output that is 5 % off moves it by 1.6e-3. So every comparison here measures three things:

* ``global_``: the Frobenius relative error of the whole tensor;
* ``tile``: the worst relative error of any 16 x 16 tile of the tensor viewed as
  ``[-1, last_dim]`` (GEMM output tiles, attention head blocks);
* ``row``: the worst relative error of any row of that view (GEMV / attention outputs, one
  sequence per row).

Each local error is ``||a - b||_T / sqrt(||b||_T^2 + floor)``, where ``floor`` is 1 % of the squared
norm of an average tile / row of the reference, so tiles whose reference is (near) zero are measured
against a typical magnitude instead of dividing by zero.

``rel_err(a, b) < tol`` passes only when the global error is below ``tol`` AND both local errors are
below ``local_factor * tol`` (default 3: bf16 output rounding puts the worst of ~25k tiles at about
1.5x the global error, ``tests/test_numerics.py`` measures it). The object also behaves as a float
(its global error) for logging.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

LOCAL_FACTOR = 3.0
TILE = (16, 16)


def _as_2d(t: torch.Tensor) -> torch.Tensor:
    t = t.detach().float()
    if t.dim() == 0:
        return t.reshape(1, 1)
    if t.dim() == 1:
        return t.reshape(1, -1)
    return t.reshape(-1, t.shape[-1])


def _block_sums(x2: torch.Tensor, tr: int, tc: int) -> torch.Tensor:
    """Sum of x2 over [tr, tc] blocks (zero-padded at the edges)."""
    R, C = x2.shape
    pr, pc = (-R) % tr, (-C) % tc
    if pr or pc:
        x2 = torch.nn.functional.pad(x2, (0, pc, 0, pr))
    R2, C2 = x2.shape
    return x2.reshape(R2 // tr, tr, C2 // tc, tc).sum(dim=(1, 3))


def _local(d2: torch.Tensor, n2: torch.Tensor, tr: int, tc: int):
    """Worst block relative error and its block index from squared diffs / squared refs."""
    ds = _block_sums(d2, tr, tc)
    ns = _block_sums(n2, tr, tc)
    floor = 1e-2 * float(n2.mean()) * tr * tc
    e = (ds / (ns + floor + 1e-30)).sqrt()
    k = int(torch.argmax(e))
    return float(e.reshape(-1)[k]), divmod(k, e.shape[1])


@dataclass
class Err:
    global_: float
    tile: float
    tile_at: tuple
    row: float
    row_at: int
    local_factor: float = LOCAL_FACTOR

    @property
    def local(self) -> float:
        return max(self.tile, self.row)

    def ok(self, tol: float) -> bool:
        return self.global_ < tol and self.local < self.local_factor * tol

    # ``assert rel_err(a, b) < tol`` checks the global AND the local errors
    def __lt__(self, tol) -> bool:
        return self.ok(float(tol))

    def __le__(self, tol) -> bool:
        return self.ok(float(tol))

    def __gt__(self, tol) -> bool:
        return not self.ok(float(tol))

    def __float__(self) -> float:
        return self.global_

    def __format__(self, spec: str) -> str:
        return format(self.global_, spec or ".3e")

    def __repr__(self) -> str:
        return (f"Err(global={self.global_:.3e}, worst 16x16 tile={self.tile:.3e} at tile {self.tile_at}, "
                f"worst row={self.row:.3e} at row {self.row_at}, local gate {self.local_factor:g}x)")


def rel_err(a: torch.Tensor, b: torch.Tensor, *, local_factor: float = LOCAL_FACTOR, tile=TILE) -> Err:
    """Global + per-tile + per-row relative error of ``a`` against the reference ``b``."""
    a2 = _as_2d(a)
    b2 = _as_2d(b).to(a2.device)
    if a2.shape != b2.shape:
        raise ValueError(f"shape mismatch {tuple(a.shape)} vs {tuple(b.shape)}")
    d2 = (a2 - b2).pow(2)
    n2 = b2.pow(2)
    g = math.sqrt(float(d2.sum())) / (math.sqrt(float(n2.sum())) + 1e-12)
    R, C = a2.shape
    tr, tc = min(tile[0], R), min(tile[1], C)
    te, tat = _local(d2, n2, tr, tc)
    re, (rat, _) = _local(d2, n2, 1, C)
    if not (math.isfinite(g) and math.isfinite(te) and math.isfinite(re)):
        g = te = re = float("inf")
    return Err(g, te, tat, re, rat, local_factor)


def assert_close(a: torch.Tensor, b: torch.Tensor, tol: float, what: str = "", **kw) -> Err:
    e = rel_err(a, b, **kw)
    assert e < tol, f"{what} {e!r} vs tol {tol:g}"
    return e
