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


def pick_tn(n_tiles: int, need_even: bool = False, prefer: tuple = (4, 2, 1)) -> int:
    for tn in prefer:
        if n_tiles % tn == 0 and (not need_even or tn % 2 == 0):
            return tn
    raise ValueError(f"no tile factor for {n_tiles} tiles")
