"""StageEngine: one pipeline stage (layers ``[start, end)``) resident on one device.

This is the MI355X-native replacement for the reference's per-stage forward
(``NodeWorker.pass_through_shard`` -> ``LlamaShardPart.forward`` -> HF ``LlamaDecoderLayer``,
``/root/reference/utils/node_worker.py:226-272``, ``utils/shard_loader.py:57-78``):

* weights are loaded once (reference ``.pth`` shard files, or deterministic random init on
  the device) and **pre-packed** into the MFMA fragment layout, with q/k/v and gate/up fused;
* the KV cache is a **static** preallocated ``[slots, n_kv, max_seq, head_dim]`` tensor per
  layer (no ``DynamicCache`` ``torch.cat`` growth), written in place by the QKV epilogue;
* a row-batch of tokens (any mix of sequences: row r -> cache ``slot[r]`` at position
  ``pos[r]``) runs through 5 fused HIP launches per layer for decode
  (QKV+norm+RoPE+KV-append, split-KV attention(+combine), o-proj+residual,
  gate/up+norm+SwiGLU, down+residual) or the MFMA GEMM path for prefill;
* the last stage runs final-norm + lm_head + greedy argmax fused, on the device;
* ``DecodeGraph`` captures a whole decode step into a hipGraph (device-side position
  counters, so one capture serves every step).

On a CPU device the same engine runs plain torch ops on unpacked weights (the
"plumbing" configuration of BASELINE.json config 1); it is not used on the GPU.
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn.functional as F

from ..config import LlamaConfig, ceil_div
from ..models import gpt2 as G2
from ..models import weights as W
from ..models.rope import rope_table
from ..ops import packing


# ---------------------------------------------------------------------------- weight sources
class WeightSource:
    """Where a stage's weights come from."""

    def layer(self, i: int, device, dtype) -> dict:
        raise NotImplementedError

    def embedding(self, device, dtype) -> torch.Tensor:
        raise NotImplementedError

    def final_norm(self, device, dtype) -> torch.Tensor:
        raise NotImplementedError

    def lm_head(self, device, dtype) -> torch.Tensor:
        raise NotImplementedError

    def pos_embedding(self, device, dtype) -> Optional[torch.Tensor]:
        """Learned absolute position table (GPT-2 ``wpe``); None for RoPE models."""
        return None

    def final_norm_bias(self, device, dtype) -> Optional[torch.Tensor]:
        """Final LayerNorm bias (GPT-2 ``ln_f.bias``); None for RMSNorm models."""
        return None


class ShardFolderSource(WeightSource):
    """Reference on-disk format (``block_{i}.pth`` ...), read with ``weights_only=True``."""

    def __init__(self, shards_path: str, cfg: Optional[LlamaConfig] = None):
        self.path = shards_path
        self.cfg = cfg or LlamaConfig.from_pretrained(shards_path)

    def layer(self, i, device, dtype):
        if self.cfg.is_gpt2:
            return G2.load_block(self.path, i, device, dtype)
        return W.load_block(self.path, i, device, dtype)

    def embedding(self, device, dtype):
        if self.cfg.is_gpt2:
            return G2.load_embedding(self.path, device, dtype)[0]
        return W.load_single(self.path, "embedding.pth", device, dtype)

    def final_norm(self, device, dtype):
        if self.cfg.is_gpt2:
            return G2.load_ln_f(self.path, device, dtype)[0]
        return W.load_single(self.path, "final_norm.pth", device, dtype)

    def lm_head(self, device, dtype):
        if self.cfg.is_gpt2:
            return G2.load_lm_head(self.path, device, dtype)
        return W.load_lm_head(self.path, self.cfg, device, dtype)

    def pos_embedding(self, device, dtype):
        return G2.load_embedding(self.path, device, dtype)[1] if self.cfg.is_gpt2 else None

    def final_norm_bias(self, device, dtype):
        return G2.load_ln_f(self.path, device, dtype)[1] if self.cfg.is_gpt2 else None


class RandomSource(WeightSource):
    """Deterministic random init generated directly on the target device (no disk)."""

    def __init__(self, cfg: LlamaConfig, seed: int = 0):
        self.cfg, self.seed = cfg, seed

    def layer(self, i, device, dtype):
        if self.cfg.is_gpt2:
            return G2.random_layer(self.cfg, i, dtype, device, self.seed)
        return W.random_layer(self.cfg, i, dtype, device, self.seed)

    def embedding(self, device, dtype):
        if self.cfg.is_gpt2:
            return G2.random_wte(self.cfg, dtype, device, self.seed)
        return W.random_embedding(self.cfg, dtype, device, self.seed)

    def final_norm(self, device, dtype):
        if self.cfg.is_gpt2:
            return G2.random_ln_f(self.cfg, dtype, device, self.seed)[0]
        return W.random_final_norm(self.cfg, dtype, device, self.seed)

    def lm_head(self, device, dtype):
        if self.cfg.is_gpt2:  # tied to wte
            return G2.random_wte(self.cfg, dtype, device, self.seed)
        return W.random_lm_head(self.cfg, dtype, device, self.seed)

    def pos_embedding(self, device, dtype):
        return G2.random_wpe(self.cfg, dtype, device, self.seed) if self.cfg.is_gpt2 else None

    def final_norm_bias(self, device, dtype):
        return G2.random_ln_f(self.cfg, dtype, device, self.seed)[1] if self.cfg.is_gpt2 else None


@dataclass
class LayerWeights:
    qkv: torch.Tensor      # packed (GPU) or fused-unpacked (CPU) [qkv, H]
    o: torch.Tensor
    gate_up: torch.Tensor
    down: torch.Tensor
    ln_in: torch.Tensor
    ln_post: torch.Tensor
    raw: Optional[dict] = None  # CPU path keeps the reference state dict
    # fp8 weights (weight_dtype="fp8"): per-output-row fp32 scales of the packed e4m3 tensors
    qkv_s: Optional[torch.Tensor] = None
    o_s: Optional[torch.Tensor] = None
    gate_up_s: Optional[torch.Tensor] = None
    down_s: Optional[torch.Tensor] = None
    # GPT-2: LayerNorm biases (bf16) and projection biases (fp32, packed column order);
    # gate_up / down hold c_fc / mlp.c_proj
    ln_in_b: Optional[torch.Tensor] = None
    ln_post_b: Optional[torch.Tensor] = None
    qkv_b: Optional[torch.Tensor] = None
    o_b: Optional[torch.Tensor] = None
    gate_up_b: Optional[torch.Tensor] = None
    down_b: Optional[torch.Tensor] = None


def _is_gpu(device: torch.device) -> bool:
    return device.type == "cuda"


_I64_MIN = -(1 << 63)


def argmax_keys_torch(v: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """CPU mirror of common.h ``argmax_key``: (order-preserving fp32 bits << 32) |
    (0xffffffff - index), as the int64 bit pattern of the unsigned 64-bit key."""
    u = v.float().contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    k = torch.where(u >= 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)
    return (k << 32) | (0xFFFFFFFF - idx.to(torch.int64))


def keys_max_torch(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Elementwise UNSIGNED max of int64-stored 64-bit keys."""
    return torch.where((a ^ _I64_MIN) >= (b ^ _I64_MIN), a, b)


class StageEngine:
    DECODE_MAX_ROWS = packing.GEMV_MAX_ROWS  # rows handled by the decode attention / graph paths (128)
    # rows above which the projections run on the MFMA GEMMs instead of the weight-streaming GEMVs
    # (per instance: the route table, ops/routes.py, may send a model's 65-128-row decode to the
    # MFMA GEMMs - Llama-2-13B, profiles/r5_gemv_max_rows_ab.md; LSA_GEMV_MAX_ROWS overrides)
    GEMV_MAX_ROWS = int(os.environ.get("LSA_GEMV_MAX_ROWS", str(packing.GEMV_MAX_ROWS)))
    # split-KV chunks never shorter than this many keys: below ~256 keys per split the merge
    # costs more than the extra parallelism buys (profiles/r1_bench_kernels_sweep.jsonl, attn)
    ATTN_MIN_CHUNK = int(os.environ.get("LSA_ATTN_MIN_CHUNK", "256"))  # keys per decode split, at least
    # batch-1 decode: attention and the o projection in one launch, the o weights streamed while
    # the attention runs (attn_oproj.hip). Off: measured 6 % slower at batch 1 than the two
    # launches (profiles/r6_attn_oproj.md); LSA_ATTN_OPROJ=1 turns it on
    ATTN_OPROJ = os.environ.get("LSA_ATTN_OPROJ", "0") == "1"

    def __init__(self, cfg: LlamaConfig, start: int, end: int, device="cpu",
                 dtype=torch.bfloat16, *, has_embed: bool = False, has_head: bool = False,
                 source: Optional[WeightSource] = None, max_slots: int = 1, max_seq: int = 2048,
                 max_prefill_rows: int = 2048, causal: bool = True, load: bool = True,
                 verbose: bool = False, head_cols: Optional[tuple] = None, weight_dtype: str = "bf16"):
        if not (0 <= start < end <= cfg.num_hidden_layers):
            raise ValueError(f"[ERROR] invalid layer range [{start}, {end})")
        self.cfg = cfg
        self.start, self.end = start, end
        self.n_layers = end - start
        if "LSA_GEMV_MAX_ROWS" not in os.environ:  # the class value (env / tests) bounds the route table's
            from ..ops import routes
            self.GEMV_MAX_ROWS = min(type(self).GEMV_MAX_ROWS, routes.gemv_max_rows(self.proj_shapes(cfg)))
        self.device = torch.device(device)
        self.gpu = _is_gpu(self.device)
        if self.gpu and dtype != torch.bfloat16:
            raise ValueError("the HIP path computes in bfloat16 (pass dtype=torch.bfloat16)")
        self.dtype = dtype
        self.has_embed, self.has_head = has_embed, has_head
        if weight_dtype not in ("bf16", "fp8"):
            raise ValueError(f"weight_dtype must be bf16 or fp8, got {weight_dtype!r}")
        # fp8: projection + lm_head weights kept as OCP e4m3 with per-row scales (W8A16); decode
        # batches <= 64 stream them natively (gemv_fp8.hip), larger row counts dequantise one
        # projection at a time into a scratch buffer for the bf16 coop / GEMM kernels
        self.fp8 = weight_dtype == "fp8" and self.gpu
        self.lm_head_s = None
        # vocab rows [v0, v1) of the lm_head held here (a pipeline may split the head between its
        # last and first stage so that neither carries the whole 0.4-layer lm_head)
        self.head_v0, self.head_v1 = head_cols if head_cols is not None else (0, cfg.head_rows)
        if not (0 <= self.head_v0 < self.head_v1 <= cfg.head_rows) or (self.head_v1 - self.head_v0) % 16:
            raise ValueError(f"bad head_cols {head_cols}")
        self.source = source
        self.max_slots = int(max_slots)
        self.max_seq = int(min(max_seq, cfg.max_position_embeddings))
        self.max_prefill_rows = int(max_prefill_rows)
        self.causal = causal
        self.verbose = verbose
        self.layers: list = []
        self.embed_w = self.final_norm = self.lm_head = None
        self.head_bias = None  # fp32 [head_v1 - head_v0]: -huge on vocab padding columns
        self.pos_emb = self.final_norm_b = None
        self.k_cache: list = []
        self.v_cache: list = []
        self.seq_len = [0] * self.max_slots  # host-side KV length per slot
        self._graphs: dict = {}
        self._scratch: dict = {}  # decode scratch sets of concurrent graphs (decode_scratch)
        if self.gpu:
            from ..ops import hip as _hip  # noqa: F401  (fail loudly if the .so is missing)
            _hip.lib()
        if load:
            self.load()

    # ------------------------------------------------------------------------- loading
    @staticmethod
    def proj_shapes(cfg: LlamaConfig) -> list:
        """(N, K) of a layer's four projections: qkv, o, gate_up (or GPT-2's c_fc), down."""
        return [(cfg.qkv_size, cfg.hidden_size), (cfg.hidden_size, cfg.q_size),
                (cfg.mlp_in_size, cfg.hidden_size), (cfg.hidden_size, cfg.intermediate_size)]

    def _log(self, msg: str) -> None:
        if self.verbose:
            print(msg, flush=True)

    def load(self) -> None:
        cfg, dev, dt = self.cfg, self.device, self.dtype
        src = self.source
        if src is None:
            raise ValueError("StageEngine needs a WeightSource")
        self.layers = []
        for i in range(self.start, self.end):
            self._log(f"[INFO] loading hidden layer {i}")
            lw = src.layer(i, dev, dt)
            self.layers.append(self._prepare_layer(lw))
            del lw
        if self.has_embed:
            self._log("[INFO] loading embedding layer...")
            self.embed_w = src.embedding(dev, dt).contiguous()
        if cfg.is_gpt2 and self.start == 0:  # wpe is added in front of layer 0 (fused into ln_1)
            self.pos_emb = src.pos_embedding(dev, dt).contiguous()
        if self.has_head:
            self._log("[INFO] loading final norm / lm_head...")
            self.final_norm = src.final_norm(dev, dt).contiguous()
            fb = src.final_norm_bias(dev, dt)
            self.final_norm_b = fb.contiguous() if fb is not None else None
            lm = src.lm_head(dev, dt)
            if lm.shape[0] < cfg.head_rows:  # pad to whole 16-row tiles with copies of row 0
                lm = torch.cat([lm, lm[:1].expand(cfg.head_rows - lm.shape[0], -1)])
            if (self.head_v0, self.head_v1) != (0, lm.shape[0]):
                lm = lm[self.head_v0:self.head_v1]
            # GPU: final RMSNorm weight folded into the packed lm_head (fused norm+GEMV+argmax);
            # GPT-2's LayerNorm (mean + bias) runs as its own kernel in front of a plain GEMV
            if self.gpu and not cfg.is_gpt2:
                lm = packing.fold_norm(lm, self.final_norm)
            if self.fp8:
                q, self.lm_head_s = packing.quantize_fp8_rows(lm)
                self.lm_head = packing.pack_b_fp8(q)
            else:
                self.lm_head = packing.pack_b(lm) if self.gpu else lm.contiguous()
            del lm
            # padding columns (copies of row 0) tie with token 0 up to rounding: a -huge bias
            # keeps them out of the fused argmax
            n_pad = self.head_v1 - max(self.head_v0, cfg.vocab_size)
            if n_pad > 0:
                hb = torch.zeros(self.head_v1 - self.head_v0, dtype=torch.float32, device=dev)
                hb[hb.numel() - n_pad:] = -3.0e38
                self.head_bias = hb
        self._alloc_runtime()

    def _prepare_layer(self, lw: dict) -> LayerWeights:
        cfg = self.cfg
        if cfg.is_gpt2:
            return self._prepare_layer_gpt2(lw)
        qkv = packing.fuse_qkv(lw["self_attn.q_proj.weight"], lw["self_attn.k_proj.weight"],
                               lw["self_attn.v_proj.weight"], cfg.num_attention_heads,
                               cfg.num_key_value_heads, cfg.head_dim)
        gu = packing.fuse_gate_up(lw["mlp.gate_proj.weight"], lw["mlp.up_proj.weight"])
        if self.gpu and self.fp8:
            ln_in, ln_post = lw["input_layernorm.weight"], lw["post_attention_layernorm.weight"]
            parts = []
            for wt in (packing.fold_norm(qkv, ln_in), lw["self_attn.o_proj.weight"], packing.fold_norm(gu, ln_post),
                       lw["mlp.down_proj.weight"]):
                q, sc = packing.quantize_fp8_rows(wt)
                parts.append((packing.pack_b_fp8(q), sc))
            return LayerWeights(parts[0][0], parts[1][0], parts[2][0], parts[3][0], ln_in.contiguous(),
                                ln_post.contiguous(), qkv_s=parts[0][1], o_s=parts[1][1], gate_up_s=parts[2][1],
                                down_s=parts[3][1])
        if self.gpu:
            # RMSNorm weights are folded into the projections that consume the normed input
            ln_in, ln_post = lw["input_layernorm.weight"], lw["post_attention_layernorm.weight"]
            mats = (packing.fold_norm(qkv, ln_in), lw["self_attn.o_proj.weight"], packing.fold_norm(gu, ln_post),
                    lw["mlp.down_proj.weight"])
            return LayerWeights(*(packing.pack_b(m) for m in mats), ln_in.contiguous(), ln_post.contiguous())
        return LayerWeights(None, None, None, None, lw["input_layernorm.weight"],
                            lw["post_attention_layernorm.weight"], raw=lw)

    def _prepare_layer_gpt2(self, lw: dict) -> LayerWeights:
        t = G2.to_linear(lw)
        if not self.gpu:
            return LayerWeights(None, None, None, None, t["ln1_w"], t["ln2_w"], raw=t, ln_in_b=t["ln1_b"],
                                ln_post_b=t["ln2_b"])
        mats, scales = [], []
        for k in ("qkv_w", "o_w", "fc_w", "proj_w"):
            if self.fp8:
                q, sc = packing.quantize_fp8_rows(t[k])
                mats.append(packing.pack_b_fp8(q))
                scales.append(sc)
            else:
                mats.append(packing.pack_b(t[k]))
                scales.append(None)
        fb = {k: t[k].float().contiguous() for k in ("qkv_b", "o_b", "fc_b", "proj_b")}
        return LayerWeights(*mats, t["ln1_w"].contiguous(), t["ln2_w"].contiguous(), qkv_s=scales[0], o_s=scales[1],
                            gate_up_s=scales[2], down_s=scales[3], ln_in_b=t["ln1_b"].contiguous(),
                            ln_post_b=t["ln2_b"].contiguous(), qkv_b=fb["qkv_b"], o_b=fb["o_b"],
                            gate_up_b=fb["fc_b"], down_b=fb["proj_b"])

    def _alloc_runtime(self) -> None:
        cfg, dev = self.cfg, self.device
        nkv, hd = cfg.num_key_value_heads, cfg.head_dim
        shape = (self.max_slots, nkv, self.max_seq, hd)
        self.k_cache = [torch.zeros(shape, dtype=self.dtype, device=dev) for _ in range(self.n_layers)]
        self.v_cache = [torch.zeros(shape, dtype=self.dtype, device=dev) for _ in range(self.n_layers)]
        self.cos, self.sin = (None, None) if cfg.is_gpt2 else rope_table(cfg, self.max_seq, dev)
        R = max(self.max_prefill_rows, self.DECODE_MAX_ROWS)
        H, I = cfg.hidden_size, cfg.intermediate_size
        if self.gpu:
            bf = torch.bfloat16
            self.buf_h = torch.zeros((R, H), dtype=bf, device=dev)
            self.buf_xn = torch.zeros((R, H), dtype=bf, device=dev)
            self.buf_q = torch.zeros((R, cfg.q_size), dtype=bf, device=dev)
            self.buf_attn = torch.zeros((R, cfg.q_size), dtype=bf, device=dev)
            self.buf_act = torch.zeros((R, I), dtype=bf, device=dev)
            self.max_decode_nsplit = int(min(16, max(1, ceil_div(self.max_seq, self.ATTN_MIN_CHUNK))))
            ws_rows = max(self.DECODE_MAX_ROWS * self.max_decode_nsplit, R * 4)
            self.part_o = torch.zeros(ws_rows * cfg.num_attention_heads * hd, dtype=torch.float32, device=dev)
            self.part_lse = torch.zeros(ws_rows * cfg.num_attention_heads, dtype=torch.float32, device=dev)
            # per-(row, kv-head) arrival tickets of the in-kernel split-KV merge (self-resetting)
            self.attn_cnt = torch.zeros(ws_rows * cfg.num_key_value_heads, dtype=torch.int32, device=dev)
            self.ao_sync = torch.zeros(4, dtype=torch.int32, device=dev)  # attn_oproj arrival counters
            self.ws_rows = ws_rows
            self.keys = torch.zeros(R, dtype=torch.int64, device=dev)
            self.tokens = torch.zeros(R, dtype=torch.int32, device=dev)
            # split-K workspace of the cooperative decode GEMV (gemv_coop.hip), owned by the
            # stage and allocated before any graph capture
            from ..ops import hip
            shapes = [(cfg.qkv_size, H), (H, cfg.q_size), (cfg.mlp_in_size, H), (H, I)]
            if self.has_head:
                shapes.append((self.head_v1 - self.head_v0, H))
            even = () if cfg.is_gpt2 else ((2 * I, H),)
            floats, groups = packing.coop_workspace_need(shapes, self.DECODE_MAX_ROWS, even_n=even)
            # the prefill GEMM's split-K slabs (small-M grids only) share it: <= 64 MB
            self.coop_ws = hip.CoopWorkspace(dev, slab_floats=max(floats, 1 << 24), groups=max(groups, 4096))
            # stream-K / split-K partial slabs + tickets of the > 128-row GEMM (gemm_sk.hip)
            self.sk_ws = hip.SkWorkspace(dev) if R > self.DECODE_MAX_ROWS else None
            # split-K partials of the residual projections (gemm_sk EPI_PARTIAL), summed by the
            # following norm kernel, for >128-row forwards of up to PARTIAL_MAX_ROWS rows
            self.part_k = self._alloc_part_k(R)
            # row sums of squares per 64 columns of h: RMSNorm fused across the >128-row GEMMs
            self.ss_buf = self._alloc_ss(R)
            self.w_scratch = None
            if self.fp8:  # one projection's bf16 weights, for the >64-row paths
                self.w_scratch = torch.empty(max(n * k for n, k in shapes), dtype=torch.bfloat16, device=dev)

    def _alloc_ss(self, R: int):
        if R <= self.DECODE_MAX_ROWS or self.cfg.is_gpt2 or self.cfg.hidden_size % 256:
            return None
        return torch.zeros((R, self.cfg.hidden_size // 64), dtype=torch.float32, device=self.device)

    def _alloc_part_k(self, R: int):
        from ..ops import hip
        if R <= self.DECODE_MAX_ROWS or self.cfg.is_gpt2:
            return None
        rows = min(R, hip.PARTIAL_MAX_ROWS)
        return torch.empty((hip.PARTIAL_MAX_SPLIT, rows, self.cfg.hidden_size), dtype=torch.float32,
                           device=self.device)

    # buffers a forward pass writes besides the KV cache: one set per concurrently running graph
    SCRATCH_ATTRS = ("buf_h", "buf_xn", "buf_q", "buf_attn", "buf_act", "part_o", "part_lse", "attn_cnt",
                     "ao_sync", "coop_ws", "sk_ws", "part_k", "ss_buf", "w_scratch", "keys", "tokens", "ws_rows")

    def decode_scratch(self, k: int, rows: Optional[int] = None) -> dict:
        """Scratch set ``k`` for forward passes that run CONCURRENTLY on different streams (a
        hipGraph bakes in its buffer addresses, so two graphs replayed at once must not share
        activations, attention partials or split-K tickets). Set 0 is the engine's own; sets
        k >= 1 are allocated on first use for ``rows`` rows (default: a decode graph's
        DECODE_MAX_ROWS; a server that also prefills on the set asks for its prefill budget)."""
        if k == 0:
            return {a: getattr(self, a) for a in self.SCRATCH_ATTRS}
        R = max(self.DECODE_MAX_ROWS, rows or 0)
        if k in self._scratch and self._scratch[k]["buf_h"].shape[0] < R:
            raise ValueError(f"scratch set {k} was allocated for fewer than {R} rows")
        if k not in self._scratch:
            from ..ops import hip
            cfg, dev, bf = self.cfg, self.device, torch.bfloat16
            H, I, nh, hd = cfg.hidden_size, cfg.intermediate_size, cfg.num_attention_heads, cfg.head_dim
            ws_rows = max(self.DECODE_MAX_ROWS * self.max_decode_nsplit, R * 4 if R > self.DECODE_MAX_ROWS else 0)
            self._scratch[k] = {
                "buf_h": torch.zeros((R, H), dtype=bf, device=dev),
                "buf_xn": torch.zeros((R, H), dtype=bf, device=dev),
                "buf_q": torch.zeros((R, cfg.q_size), dtype=bf, device=dev),
                "buf_attn": torch.zeros((R, cfg.q_size), dtype=bf, device=dev),
                "buf_act": torch.zeros((R, I), dtype=bf, device=dev),
                "part_o": torch.zeros(ws_rows * nh * hd, dtype=torch.float32, device=dev),
                "part_lse": torch.zeros(ws_rows * nh, dtype=torch.float32, device=dev),
                "attn_cnt": torch.zeros(ws_rows * cfg.num_key_value_heads, dtype=torch.int32, device=dev),
                "ao_sync": torch.zeros(4, dtype=torch.int32, device=dev),
                "coop_ws": hip.CoopWorkspace(dev, slab_floats=self.coop_ws.slab.numel(),
                                             groups=self.coop_ws.counters.numel()),
                "sk_ws": hip.SkWorkspace(dev) if R > self.DECODE_MAX_ROWS else None,
                "part_k": self._alloc_part_k(R),
                "ss_buf": self._alloc_ss(R),
                "w_scratch": None if self.w_scratch is None else torch.empty_like(self.w_scratch),
                "keys": torch.zeros(R, dtype=torch.int64, device=dev),
                "tokens": torch.zeros(R, dtype=torch.int32, device=dev),
                "ws_rows": ws_rows,
            }
        return self._scratch[k]

    @contextmanager
    def use_scratch(self, k: int):
        """Run (capture) forward passes against scratch set ``k``."""
        saved = {a: getattr(self, a) for a in self.SCRATCH_ATTRS}
        for a, v in self.decode_scratch(k).items():
            setattr(self, a, v)
        try:
            yield
        finally:
            for a, v in saved.items():
                setattr(self, a, v)

    def memory_bytes(self) -> int:
        """Bytes of weights + KV cache (tensors that share storage are counted once)."""
        ts = []
        for lw in self.layers:
            ts += [lw.qkv, lw.o, lw.gate_up, lw.down, lw.ln_in, lw.ln_post, lw.qkv_s, lw.o_s, lw.gate_up_s,
                   lw.down_s, lw.ln_in_b, lw.ln_post_b, lw.qkv_b, lw.o_b, lw.gate_up_b, lw.down_b]
            if lw.raw is not None:
                ts += list(lw.raw.values())
        ts += [self.embed_w, self.final_norm, self.lm_head, self.pos_emb, self.final_norm_b, self.lm_head_s]
        ts += self.k_cache + self.v_cache
        seen, n = set(), 0
        for t in ts:
            if t is None:
                continue
            key = (t.untyped_storage().data_ptr(), t.storage_offset(), t.numel())
            if key not in seen:
                seen.add(key)
                n += t.numel() * t.element_size()
        return n

    # ------------------------------------------------------------------------- state
    def reset(self, slots=None) -> None:
        """Forget the KV contents of ``slots`` (all by default). The static cache is not
        zeroed: attention only ever reads positions < the row's length."""
        for s in (range(self.max_slots) if slots is None else slots):
            self.seq_len[s] = 0

    # ------------------------------------------------------------------------- helpers
    def _i32(self, x) -> torch.Tensor:
        if isinstance(x, torch.Tensor):
            return x.to(device=self.device, dtype=torch.int32).contiguous()
        return torch.tensor(list(x), dtype=torch.int32, device=self.device)

    # ------------------------------------------------------------------------- forward (eager)
    def embed(self, ids: torch.Tensor) -> torch.Tensor:
        """ids [rows] -> hidden [rows, H] (dtype)."""
        if self.embed_w is None:
            raise RuntimeError("[ERROR] this stage has no embedding layer")
        ids = ids.reshape(-1)
        if self.gpu:
            from ..ops import hip
            rows = ids.numel()
            out = torch.empty((rows, self.cfg.hidden_size), dtype=torch.bfloat16, device=self.device)
            hip.embed(self._i32(ids), self.embed_w, out)
            return out
        return F.embedding(ids.to(self.device, torch.long), self.embed_w)

    def forward(self, h: torch.Tensor, slot, pos, kv_len=None) -> torch.Tensor:
        """Run this stage's layers on ``h`` [rows, H]. Row r is a token of the sequence in
        cache ``slot[r]`` at position ``pos[r]``. Returns the new hidden [rows, H]."""
        rows = h.shape[0]
        slot_t, pos_t = self._i32(slot), self._i32(pos)
        kvl_t = None if kv_len is None else self._i32(kv_len)
        if self.gpu:
            tiles = None
            if rows > self.DECODE_MAX_ROWS:
                # prefill: flash attention over per-sequence tiles (host-built table)
                from ..ops import hip
                th = hip.build_prefill_tiles(slot, pos, kv_len, tile_rows=hip.prefill_tile_rows(
                    self.cfg.num_attention_heads, self.cfg.num_key_value_heads, rows))
                tiles = (th, th.to(self.device, non_blocking=True))
            return self._forward_hip(h, slot_t, pos_t, kvl_t, rows, tiles=tiles)
        return self._forward_torch(h, slot_t.long(), pos_t.long(), None if kvl_t is None else kvl_t.long())

    def head(self, h: torch.Tensor, rows_idx=None) -> torch.Tensor:
        """final RMSNorm -> lm_head -> greedy argmax for the selected rows. Returns int64 [n]."""
        if self.lm_head is None:
            raise RuntimeError("[ERROR] this stage has no lm_head")
        if rows_idx is None:
            rows_idx = list(range(h.shape[0]))
        if self.gpu:
            from ..ops import hip
            if (self.head_v0, self.head_v1) != (0, self.cfg.head_rows):
                raise RuntimeError("head(): this stage holds only part of the lm_head (use head_keys)")
            keys = self.head_keys(h, rows_idx)
            n = keys.numel()
            out = torch.empty(n, dtype=torch.int64, device=self.device)
            for c0 in range(0, n, self.DECODE_MAX_ROWS):
                c = min(self.DECODE_MAX_ROWS, n - c0)
                hip.argmax_finalize(keys[c0:c0 + c], c, self.tokens)
                out[c0:c0 + c] = self.tokens[:c].long()
            return out
        hs = h[torch.as_tensor(rows_idx, device=h.device, dtype=torch.long)]
        lg = self.logits_torch(hs)
        return torch.argmax(lg, dim=-1)

    def head_keys(self, h: torch.Tensor, rows_idx=None, keys: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Fused final-norm + (partial) lm_head + argmax KEYS of the selected rows over this
        stage's vocab slice [head_v0, head_v1): the 64-bit (ordered logit, inverted index) keys of
        common.h ``argmax_key``, so two slices combine by an unsigned max. ``keys`` (int64 [n]:
        pass the other slice's keys to complete them) defaults to zeros. Returns keys."""
        if rows_idx is None:
            rows_idx = list(range(h.shape[0]))
        if not self.gpu:
            hs = h[torch.as_tensor(rows_idx, device=h.device, dtype=torch.long)]
            v, i = self.logits_torch(hs).max(-1)
            new = argmax_keys_torch(v, i + self.head_v0)
            return new if keys is None else keys_max_torch(keys, new)
        from ..ops import hip
        idx = self._i32(rows_idx)
        n = idx.numel()
        if keys is None:
            keys = torch.zeros(n, dtype=torch.int64, device=self.device)
        # one call: head_gemv picks the same kernel path (and numerics) for n rows as a decode
        # graph of n rows does, so a split head's re-derived first token matches the prefill's
        self.head_gemv(h, n, keys, a_rows=idx)
        return keys

    def head_gemv(self, h: torch.Tensor, rows: int, keys: torch.Tensor, a_rows=None) -> None:
        """Fused final RMSNorm + lm_head slice + argmax keys (atomicMax into ``keys``).
        GPT-2: ln_f (LayerNorm kernel, rows gathered first) then the plain GEMV + argmax."""
        from ..ops import hip
        N0 = self.head_v1 - self.head_v0
        if (rows > self.DECODE_MAX_ROWS and not self.cfg.is_gpt2 and self.lm_head_s is None and self.sk_ws is not None
                and N0 % 128 == 0 and rows <= self.buf_xn.shape[0]):
            # big batches: RMSNorm kernel (final norm folded into lm_head) -> gemm_sk with the
            # fused argmax epilogue (one launch instead of 128-row GEMV chunks)
            xn = self.buf_xn[:rows]
            src = h[:rows] if a_rows is None else h.index_select(0, a_rows.long())
            hip.rmsnorm(src, None, xn, rows, self.cfg.rms_norm_eps, self.cfg.hidden_size)
            ep = hip.make_epi(keys=keys, col_offset=self.head_v0, bias=self.head_bias)
            hip.gemm_sk(xn, self.lm_head, rows, N0, self.cfg.hidden_size, hip.EPI_ARGMAX, ep, ws=self.sk_ws)
            return
        if rows > self.DECODE_MAX_ROWS:  # the fused head kernels take <= 128 rows per launch
            for c0 in range(0, rows, self.DECODE_MAX_ROWS):
                c = min(self.DECODE_MAX_ROWS, rows - c0)
                if a_rows is None:
                    self.head_gemv(h[c0:c0 + c], c, keys[c0:c0 + c])
                else:
                    self.head_gemv(h, c, keys[c0:c0 + c], a_rows=a_rows[c0:c0 + c])
            return
        ep = hip.make_epi(keys=keys, col_offset=self.head_v0, bias=self.head_bias)
        N, H, eps = self.head_v1 - self.head_v0, self.cfg.hidden_size, self.cfg.rms_norm_eps
        if self.cfg.is_gpt2:
            xn = self.buf_xn[:rows]
            src = h if a_rows is None else h.index_select(0, a_rows.long())
            hip.layernorm(src, xn, self.final_norm, self.final_norm_b, rows, eps)
            if self.lm_head_s is not None:
                hip.proj_fp8(xn, self.lm_head.view(-1), self.lm_head_s, rows, N, H, hip.EPI_ARGMAX, ep, ws=self.coop_ws)
            else:
                hip.gemv(xn, self.lm_head, rows, N, H, hip.EPI_ARGMAX, ep, ws=self.coop_ws)
            return
        if self.lm_head_s is not None:
            hip.proj_fp8(h, self.lm_head.view(-1), self.lm_head_s, rows, N, H, hip.EPI_ARGMAX, ep, norm=True, eps=eps,
                         a_rows=a_rows, ws=self.coop_ws)
        else:
            hip.gemv(h, self.lm_head, rows, N, H, hip.EPI_ARGMAX, ep, ws=self.coop_ws, norm=True, eps=eps,
                     a_rows=a_rows)

    def finalize_keys(self, keys: torch.Tensor) -> torch.Tensor:
        """argmax keys -> token ids (int32, device); resets ``keys``."""
        if not self.gpu:
            tok = (0xFFFFFFFF - (keys & 0xFFFFFFFF)).to(torch.int32)
            keys.zero_()
            return tok
        from ..ops import hip
        n = keys.numel()
        out = torch.empty(n, dtype=torch.int32, device=self.device)
        for c0 in range(0, n, self.DECODE_MAX_ROWS):
            c = min(self.DECODE_MAX_ROWS, n - c0)
            hip.argmax_finalize(keys[c0:c0 + c], c, out[c0:c0 + c])
        return out

    def logits_torch(self, hs: torch.Tensor) -> torch.Tensor:
        from ..models.reference import rmsnorm
        if self.cfg.is_gpt2:
            x = G2.layer_norm(hs, self.final_norm, self.final_norm_b, self.cfg.rms_norm_eps)
        else:
            x = rmsnorm(hs, self.final_norm, self.cfg.rms_norm_eps)
        lg = F.linear(x, self.lm_head.float())
        if self.head_bias is not None:
            lg = lg + self.head_bias.to(lg.device)
        return lg

    # ------------------------------------------------------------------------- HIP path
    def decode_nsplit(self, rows: int) -> int:
        """Split-KV factor for a decode batch, fixed at graph capture: no split once the batch
        alone gives >= 512 attention workgroups (measured: splitting then only adds the combine
        launch), else aim for ~512 workgroups, chunks of >= 256 keys at max_seq."""
        wgs = rows * self.cfg.num_key_value_heads
        return int(max(1, min(self.max_decode_nsplit, ceil_div(512, wgs))))

    def _attn_nsplit(self, rows: int, kv_max: int) -> int:
        if rows <= self.DECODE_MAX_ROWS:
            return self.decode_nsplit(rows)
        want = max(1, min(8, ceil_div(kv_max, 512), ceil_div(1024, rows * self.cfg.num_key_value_heads)))
        return max(1, min(want, self.ws_rows // rows))

    def _forward_hip(self, h, slot, pos, kv_len, rows, nsplit: Optional[int] = None, tiles=None) -> torch.Tensor:
        from ..ops import hip
        cfg = self.cfg
        H, I, eps = cfg.hidden_size, cfg.intermediate_size, cfg.rms_norm_eps
        nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        if rows > self.max_prefill_rows and rows > self.DECODE_MAX_ROWS:
            raise ValueError(f"{rows} rows exceed max_prefill_rows={self.max_prefill_rows}")
        if h.dtype != torch.bfloat16 or not h.is_contiguous():
            h = h.to(torch.bfloat16).contiguous()
        hbuf = self.buf_h[:rows]
        if h.data_ptr() != hbuf.data_ptr():
            hbuf.copy_(h)
        decode = rows <= self.DECODE_MAX_ROWS
        if nsplit is None and tiles is None:
            kv_max = self.max_seq if decode else (int(pos.max().item()) + 1 if kv_len is None else int(kv_len.max().item()))
            nsplit = self._attn_nsplit(rows, kv_max)
        q, attn_o, act, xn = self.buf_q[:rows], self.buf_attn[:rows], self.buf_act[:rows], self.buf_xn[:rows]
        ws = self.coop_ws
        native_fp8 = self.fp8 and rows <= packing.GEMV_MAX_ROWS
        if cfg.is_gpt2:
            return self._forward_hip_gpt2(hbuf, slot, pos, kv_len, rows, nsplit, tiles, decode, native_fp8)

        def wbf(w, s, N, K):  # packed bf16 weights (fp8 -> scratch for the >64-row kernels)
            return w if s is None else hip.dequant_fp8_packed(w.view(-1), s, self.w_scratch, N, K)

        def dec(x, w, s, N, K, epi, ep, norm=False):
            if native_fp8:
                hip.proj_fp8(x, w.view(-1), s, rows, N, K, epi, ep, norm=norm, eps=eps, ws=ws)
            else:
                hip.gemv(x, wbf(w, s, N, K), rows, N, K, epi, ep, norm=norm, eps=eps, ws=ws)

        def dec_resid(x, w, s, N, K, ep):
            # 17..128 rows: split-K partials + one residual-add kernel where measured faster than
            # the coop kernel's in-kernel split reduction (ops/gemv_tuning.json "coop_partial")
            pc = None if (native_fp8 or s is not None or cfg.is_gpt2 or N not in (2048, 4096, 6144, 8192)) \
                else packing.partial_config(N // 16, rows, k=K)
            if pc is None or ws.slab.numel() < pc[3] * rows * N:
                dec(x, w, s, N, K, hip.EPI_RESID, ep)
                return
            part = ws.slab[:pc[3] * rows * N].view(pc[3], rows, N)
            hip.gemv(x, w, rows, N, K, hip.EPI_PARTIAL, hip.make_epi(out=part, ldo=N), coop=pc, ws=ws,
                     out_numel=part.numel())
            hip.resid_rmsnorm_partials(hbuf, part, pc[3], rows, eps)

        def pre(x, w, s, N, K, epi, ep):
            hip.gemm(x, wbf(w, s, N, K), rows, N, K, epi, ep, ws=ws, sk_ws=self.sk_ws)

        # residual projections as split-K partials summed by the next norm kernel, where measured
        # faster than the fused residual epilogue (ops/gemm_sk_tuning.json "partial" entries)
        # the projection kernel family: the weight-streaming GEMVs up to GEMV_MAX_ROWS rows, the
        # LDS-DMA MFMA GEMMs (gemm_sk / gemm_wr) above - independent of the attention's decode mode
        proj_gemm = (not decode) or (rows > self.GEMV_MAX_ROWS and not native_fp8 and self.sk_ws is not None)
        part_ok = proj_gemm and self.part_k is not None and rows <= self.part_k.shape[1]

        def resid_proj(x, w, s, N, K, ep):
            # returns the split count of partials left in part_k (0: residual applied in-GEMM)
            pp = hip.gemm_sk_partial_plan(rows, N, K) if part_ok else None
            if pp is None:
                pre(x, w, s, N, K, hip.EPI_RESID, ep)
                return 0
            bn, sp = pp
            hip.gemm_sk(x, wbf(w, s, N, K), rows, N, K, hip.EPI_PARTIAL, hip.make_epi(out=self.part_k, ldo=N),
                        bn=bn, grid=hip.N_CU, dp=0, split=sp, ws=self.sk_ws, out_numel=self.part_k.numel())
            return sp

        # RMSNorm fused across the GEMMs: residual GEMMs write per-64-column sums of squares of
        # their outputs (ss), the qkv / gate_up GEMMs read the raw residual stream and scale each
        # row by its rstd in the epilogue - no standalone norm kernel between projections
        fuse = proj_gemm and self.ss_buf is not None and rows <= self.ss_buf.shape[0]
        ss = self.ss_buf[:rows] if fuse else None
        # one decode row, one split: attention + o projection + residual in one launch
        ao = (self.ATTN_OPROJ and rows == 1 and tiles is None and nsplit == 1 and not proj_gemm and not native_fp8
              and self.ao_sync is not None)
        ss_valid = False  # ss holds the partials of hbuf's current values
        pending = 0  # down-projection partials not yet added to hbuf
        for li, lw in enumerate(self.layers):
            kc, vc = self.k_cache[li], self.v_cache[li]
            ep_qkv = hip.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, cos=self.cos, sin=self.sin,
                                  ldo=q.stride(0), n_heads=nh, n_kv=nkv, head_dim=hd, t_max=self.max_seq)
            if not proj_gemm:
                dec(hbuf, lw.qkv, lw.qkv_s, cfg.qkv_size, H, hip.EPI_QKV, ep_qkv, norm=True)
            else:
                if pending and not fuse:
                    hip.resid_rmsnorm_partials(hbuf, self.part_k, pending, rows, eps, out=xn)
                    pending = 0
                    pre(xn, lw.qkv, lw.qkv_s, cfg.qkv_size, H, hip.EPI_QKV, ep_qkv)
                elif fuse:
                    if pending:  # the previous down projection left K-split partials: add them
                        hip.resid_rmsnorm_partials(hbuf, self.part_k, pending, rows, eps)
                        pending = 0
                    if not ss_valid:
                        # (also at a stage's first layer: the same partials, in the same order, as
                        # a residual GEMM epilogue writes - a layer range computes the same bits
                        # whichever stage it starts)
                        hip.row_ss(hbuf, rows, ss)
                    ep_qkv = hip.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, cos=self.cos,
                                          sin=self.sin, ldo=q.stride(0), n_heads=nh, n_kv=nkv, head_dim=hd,
                                          t_max=self.max_seq, ss_in=ss, ss_eps=eps)
                    pre(hbuf, lw.qkv, lw.qkv_s, cfg.qkv_size, H, hip.EPI_QKV, ep_qkv)
                else:
                    hip.rmsnorm(hbuf, None, xn, rows, eps, H)
                    pre(xn, lw.qkv, lw.qkv_s, cfg.qkv_size, H, hip.EPI_QKV, ep_qkv)
            ep_o = hip.make_epi(out=hbuf, resid=hbuf, ldo=hbuf.stride(0), ldr=hbuf.stride(0))
            fused_o = ao and lw.o_s is None and hip.attn_oproj(q, kc, vc, slot, pos, nh, nkv, hd, attn_o, lw.o, H, ep_o,
                                                               self.ao_sync, kv_len=kv_len)
            if tiles is not None:
                hip.attn_prefill(q, kc, vc, tiles[1], nh, nkv, hd, attn_o, causal=kv_len is None, tiles_host=tiles[0])
            elif not fused_o:
                hip.attn(q, kc, vc, slot, pos, rows, nh, nkv, hd, nsplit, self.part_o, self.part_lse, attn_o,
                         kv_len=kv_len, counters=self.attn_cnt, min_chunk=self.ATTN_MIN_CHUNK)
            ep_gu = hip.make_epi(out=act, ldo=act.stride(0))
            if not proj_gemm:
                if not fused_o:
                    dec_resid(attn_o, lw.o, lw.o_s, H, cfg.q_size, ep_o)
                dec(hbuf, lw.gate_up, lw.gate_up_s, 2 * I, H, hip.EPI_SWIGLU, ep_gu, norm=True)
                dec_resid(act, lw.down, lw.down_s, H, I, ep_o)
            else:
                ep_r = hip.make_epi(out=hbuf, resid=hbuf, ldo=hbuf.stride(0), ldr=hbuf.stride(0), ss_out=ss) \
                    if fuse else ep_o
                sp = resid_proj(attn_o, lw.o, lw.o_s, H, cfg.q_size, ep_r)
                if sp:
                    hip.resid_rmsnorm_partials(hbuf, self.part_k, sp, rows, eps, out=xn)
                    pre(xn, lw.gate_up, lw.gate_up_s, 2 * I, H, hip.EPI_SWIGLU, ep_gu)
                elif fuse:
                    pre(hbuf, lw.gate_up, lw.gate_up_s, 2 * I, H, hip.EPI_SWIGLU,
                        hip.make_epi(out=act, ldo=act.stride(0), ss_in=ss, ss_eps=eps))
                else:
                    hip.rmsnorm(hbuf, None, xn, rows, eps, H)
                    pre(xn, lw.gate_up, lw.gate_up_s, 2 * I, H, hip.EPI_SWIGLU, ep_gu)
                pending = resid_proj(act, lw.down, lw.down_s, H, I, ep_r)
                ss_valid = fuse and not pending
        if pending:  # the stage's output residual stream
            hip.resid_rmsnorm_partials(hbuf, self.part_k, pending, rows, eps)
        return hbuf

    def _forward_hip_gpt2(self, hbuf, slot, pos, kv_len, rows, nsplit, tiles, decode, native_fp8) -> torch.Tensor:
        """GPT-2 layer on the HIP path: LayerNorm kernel (ln_1, with the wpe add fused in front
        of layer 0) -> QKV projection + bias + KV-cache append (no RoPE) -> attention ->
        c_proj + bias + residual -> LayerNorm (ln_2) -> c_fc + bias + GELU -> mlp.c_proj + bias
        + residual. Decode rows use the GEMV / coop / fp8 kernels, prefill rows the MFMA GEMM."""
        from ..ops import hip
        cfg = self.cfg
        H, I, eps = cfg.hidden_size, cfg.intermediate_size, cfg.rms_norm_eps
        nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        q, attn_o, act, xn = self.buf_q[:rows], self.buf_attn[:rows], self.buf_act[:rows], self.buf_xn[:rows]
        ws = self.coop_ws

        def proj(x, w, s, N, K, epi, ep):
            if decode and native_fp8:
                hip.proj_fp8(x, w.view(-1), s, rows, N, K, epi, ep, ws=ws)
                return
            wb = w if s is None else hip.dequant_fp8_packed(w.view(-1), s, self.w_scratch, N, K)
            if decode:
                hip.gemv(x, wb, rows, N, K, epi, ep, ws=ws)
            else:
                hip.gemm(x, wb, rows, N, K, epi, ep, ws=ws, sk_ws=self.sk_ws)

        for li, lw in enumerate(self.layers):
            kc, vc = self.k_cache[li], self.v_cache[li]
            pe = self.pos_emb if (li == 0 and self.start == 0) else None
            hip.layernorm(hbuf, xn, lw.ln_in, lw.ln_in_b, rows, eps, pos_emb=pe, pos=pos)
            ep_qkv = hip.make_epi(out=q, k_cache=kc, v_cache=vc, slot=slot, pos=pos, ldo=q.stride(0), n_heads=nh,
                                  n_kv=nkv, head_dim=hd, t_max=self.max_seq, bias=lw.qkv_b)
            proj(xn, lw.qkv, lw.qkv_s, cfg.qkv_size, H, hip.EPI_QKV, ep_qkv)
            if tiles is not None:
                hip.attn_prefill(q, kc, vc, tiles[1], nh, nkv, hd, attn_o, causal=kv_len is None, tiles_host=tiles[0])
            else:
                hip.attn(q, kc, vc, slot, pos, rows, nh, nkv, hd, nsplit, self.part_o, self.part_lse, attn_o,
                         kv_len=kv_len, counters=self.attn_cnt, min_chunk=self.ATTN_MIN_CHUNK)
            proj(attn_o, lw.o, lw.o_s, H, cfg.q_size, hip.EPI_RESID,
                 hip.make_epi(out=hbuf, resid=hbuf, ldo=hbuf.stride(0), ldr=hbuf.stride(0), bias=lw.o_b))
            hip.layernorm(hbuf, xn, lw.ln_post, lw.ln_post_b, rows, eps)
            proj(xn, lw.gate_up, lw.gate_up_s, I, H, hip.EPI_STORE,
                 hip.make_epi(out=act, ldo=act.stride(0), bias=lw.gate_up_b, act=hip.ACT_GELU))
            proj(act, lw.down, lw.down_s, H, I, hip.EPI_RESID,
                 hip.make_epi(out=hbuf, resid=hbuf, ldo=hbuf.stride(0), ldr=hbuf.stride(0), bias=lw.down_b))
        return hbuf

    # ------------------------------------------------------------------------- torch path (CPU)
    def _attend_torch(self, q, kc, vc, slot, T) -> torch.Tensor:
        """Per-slot causal attention over the cache (fp32). q [rows, nh, hd] -> [rows, nh*hd]."""
        cfg = self.cfg
        nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        g = nh // nkv
        rows = q.shape[0]
        o = torch.empty((rows, nh, hd), dtype=torch.float32, device=self.device)
        for s_ in torch.unique(slot).tolist():
            sel = (slot == s_).nonzero().flatten()
            tmax = int(T[sel].max())
            K = kc[s_, :, :tmax].float().repeat_interleave(g, dim=0)  # [nh, t, hd]
            V = vc[s_, :, :tmax].float().repeat_interleave(g, dim=0)
            qs = q[sel].float().transpose(0, 1)  # [nh, n, hd]
            sc = torch.matmul(qs, K.transpose(1, 2)) * (hd ** -0.5)  # [nh, n, t]
            mask = torch.arange(tmax, device=self.device)[None, :] >= T[sel][:, None]
            sc = sc.masked_fill(mask[None], float("-inf"))
            o[sel] = torch.matmul(torch.softmax(sc, dim=-1), V).transpose(0, 1)
        return o.reshape(rows, nh * hd)

    def _forward_torch_gpt2(self, h, slot, pos, kv_len) -> torch.Tensor:
        cfg = self.cfg
        nh, hd, eps, dt = cfg.num_attention_heads, cfg.head_dim, cfg.rms_norm_eps, self.dtype
        rows = h.shape[0]
        h = h.to(self.device, dt)
        if self.start == 0:
            h = (h.float() + self.pos_emb[pos].float()).to(dt)
        T = (pos + 1) if kv_len is None else kv_len
        for li, lw in enumerate(self.layers):
            w = lw.raw
            x = G2.layer_norm(h, w["ln1_w"], w["ln1_b"], eps).to(dt).float()
            qkv = F.linear(x, w["qkv_w"].float(), w["qkv_b"].float())
            q, k, v = (t.reshape(rows, nh, hd) for t in qkv.split(cfg.hidden_size, dim=-1))
            kc, vc = self.k_cache[li], self.v_cache[li]
            kc[slot, :, pos] = k.to(dt)
            vc[slot, :, pos] = v.to(dt)
            o = self._attend_torch(q.to(dt), kc, vc, slot, T).to(dt)
            h = (h.float() + F.linear(o.float(), w["o_w"].float(), w["o_b"].float())).to(dt)
            x = G2.layer_norm(h, w["ln2_w"], w["ln2_b"], eps).to(dt).float()
            a = G2.gelu_new(F.linear(x, w["fc_w"].float(), w["fc_b"].float())).to(dt)
            h = (h.float() + F.linear(a.float(), w["proj_w"].float(), w["proj_b"].float())).to(dt)
        return h

    def _forward_torch(self, h, slot, pos, kv_len) -> torch.Tensor:
        from ..models.reference import rmsnorm
        cfg = self.cfg
        if cfg.is_gpt2:
            return self._forward_torch_gpt2(h, slot, pos, kv_len)
        nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        dt = self.dtype
        rows = h.shape[0]
        h = h.to(self.device, dt)
        half = hd // 2
        cos = self.cos[pos]  # [rows, half]
        sin = self.sin[pos]
        T = (pos + 1) if kv_len is None else kv_len
        for li, lw in enumerate(self.layers):
            w = lw.raw
            x = rmsnorm(h, lw.ln_in, cfg.rms_norm_eps).to(dt)
            q = F.linear(x.float(), w["self_attn.q_proj.weight"].float()).view(rows, nh, hd)
            k = F.linear(x.float(), w["self_attn.k_proj.weight"].float()).view(rows, nkv, hd)
            v = F.linear(x.float(), w["self_attn.v_proj.weight"].float()).view(rows, nkv, hd)

            def rope(t):
                t1, t2 = t[..., :half], t[..., half:]
                c, s = cos[:, None, :], sin[:, None, :]
                return torch.cat([t1 * c - t2 * s, t2 * c + t1 * s], dim=-1)

            q, k = rope(q).to(dt), rope(k).to(dt)
            kc, vc = self.k_cache[li], self.v_cache[li]
            kc[slot, :, pos] = k
            vc[slot, :, pos] = v.to(dt)
            o = self._attend_torch(q, kc, vc, slot, T).to(dt)
            h = (h.float() + F.linear(o.float(), w["self_attn.o_proj.weight"].float())).to(dt)
            x = rmsnorm(h, lw.ln_post, cfg.rms_norm_eps).to(dt).float()
            a = (F.silu(F.linear(x, w["mlp.gate_proj.weight"].float())) *
                 F.linear(x, w["mlp.up_proj.weight"].float())).to(dt)
            h = (h.float() + F.linear(a.float(), w["mlp.down_proj.weight"].float())).to(dt)
        return h

    # ------------------------------------------------------------------------- sequence API
    def prefill_rows(self, slot_ids: list, lengths: list) -> tuple:
        """Build (slot, pos) row vectors for appending ``lengths[i]`` tokens to ``slot_ids[i]``."""
        slot, pos = [], []
        for s, n in zip(slot_ids, lengths):
            p0 = self.seq_len[s]
            if p0 + n > self.max_seq:
                raise ValueError(f"[ERROR] sequence in slot {s} would exceed max_seq={self.max_seq}")
            slot += [s] * n
            pos += list(range(p0, p0 + n))
        return slot, pos

    def advance(self, slot_ids: list, lengths: list) -> None:
        for s, n in zip(slot_ids, lengths):
            self.seq_len[s] += n

    def graph(self, key) -> Optional["DecodeGraph"]:
        return self._graphs.get(key)


class DecodeGraph:
    """A hipGraph-captured decode step for a fixed set of ``rows`` (row r -> slot r).

    ``mode``:
      * ``"full"``  embed(tokens) -> layers -> head argmax -> tokens (single-stage loop)
      * ``"first"`` embed(tokens) -> layers -> out hidden
      * ``"mid"``   hidden in -> layers -> out hidden
      * ``"last"``  hidden in -> layers -> head argmax -> tokens
    Positions live on the device (``self.pos``) and are advanced inside the graph, so the
    same graph is replayed every step. ``sync_pos()`` copies the host view after replays.
    """

    def __init__(self, eng: StageEngine, rows: int, mode: str, slots: Optional[list] = None,
                 history_len: int = 0, split_head: bool = False, scratch: int = 0):
        from ..ops import hip
        if not eng.gpu:
            raise RuntimeError("DecodeGraph needs a GPU stage")
        # above DECODE_MAX_ROWS the step runs the >128-row projections (gemm_sk.hip stream-K GEMM
        # pass, or gemm.hip) on buffers sized by max_prefill_rows; argmax_finalize takes <= 1024
        cap = min(1024, max(eng.DECODE_MAX_ROWS, eng.max_prefill_rows))
        if rows > cap:
            raise ValueError(f"decode graph supports <= {cap} rows")
        self.eng, self.rows, self.mode = eng, rows, mode
        dev = eng.device
        # scratch set (StageEngine.decode_scratch): graphs replayed concurrently need distinct sets
        self.scratch = scratch
        self._out = eng.decode_scratch(scratch, rows)["buf_h"][:rows]
        self.slots = list(range(rows)) if slots is None else list(slots)
        self.slot = torch.tensor(self.slots, dtype=torch.int32, device=dev)
        self.pos = torch.tensor([eng.seq_len[s] for s in self.slots], dtype=torch.int32, device=dev)
        self.tokens = torch.zeros(rows, dtype=torch.int32, device=dev)
        self.keys = torch.zeros(rows, dtype=torch.int64, device=dev)
        self.h_in = torch.zeros((rows, eng.cfg.hidden_size), dtype=torch.bfloat16, device=dev)
        self.history = torch.zeros((max(1, history_len), rows), dtype=torch.int32, device=dev) if history_len else None
        self.step_ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        self.graph = None
        self._hip = hip
        # stage hand-off captured INTO the graph (pipeline over a graph-capturable transport,
        # parallel/ipc_ring.py): receive into h_in before the step, send the step's output after
        self.pre_comm = None
        self.post_comm = None
        # split lm_head (pipeline): "last" leaves partial keys over its vocab slice + the raw
        # final hidden; "first" completes the PREVIOUS step's keys over its slice from
        # (h_fin, keys_in), finalises the token ids (and history) and then embeds them
        self.split_head = split_head
        if split_head:
            if mode not in ("first", "last"):
                raise ValueError("split_head needs mode 'first' or 'last'")
            self.h_fin = torch.zeros((rows, eng.cfg.hidden_size), dtype=torch.bfloat16, device=dev)
            self.keys_in = torch.zeros(rows, dtype=torch.int64, device=dev)

    def _body(self) -> None:
        with self.eng.use_scratch(self.scratch):
            self._step()

    def _step(self) -> None:
        hip, eng, rows = self._hip, self.eng, self.rows
        h = eng.buf_h[:rows]
        if self.split_head and self.mode == "first":
            self.keys.copy_(self.keys_in)
            eng.head_gemv(self.h_fin, rows, self.keys)
            hip.argmax_finalize(self.keys, rows, self.tokens, None, 1, self.history,
                                self.step_ctr if self.history is not None else None)
        if self.mode in ("full", "first"):
            hip.embed(self.tokens, eng.embed_w, h)
        else:
            h.copy_(self.h_in)
        eng._forward_hip(h, self.slot, self.pos, None, rows, nsplit=eng.decode_nsplit(rows))
        if self.split_head and self.mode == "last":
            self.keys.zero_()
            eng.head_gemv(h, rows, self.keys)
            hip.pos_advance(self.pos, rows, 1)
        elif self.mode in ("full", "last"):
            eng.head_gemv(h, rows, self.keys)
            hip.argmax_finalize(self.keys, rows, self.tokens, self.pos, 1, self.history,
                                self.step_ctr if self.history is not None else None)
        else:
            hip.pos_advance(self.pos, rows, 1)

    @property
    def out_hidden(self) -> torch.Tensor:
        return self._out

    def capture(self, warmup: bool = True) -> "DecodeGraph":
        """Capture the step (with ``pre_comm`` / ``post_comm`` around it when set). The warm-up
        run (if any) is undone (positions restored) and never communicates."""
        pos0, tok0 = self.pos.clone(), self.tokens.clone()
        kin0 = self.keys_in.clone() if self.split_head else None
        s = torch.cuda.Stream(device=self.eng.device)
        s.wait_stream(torch.cuda.current_stream(self.eng.device))
        with torch.cuda.stream(s):
            if warmup:
                self._body()
        torch.cuda.current_stream(self.eng.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            if self.pre_comm is not None:
                self.pre_comm()
            self._body()
            if self.post_comm is not None:
                self.post_comm()
        self.graph = g
        self.pos.copy_(pos0)
        self.tokens.copy_(tok0)
        self.keys.zero_()
        self.step_ctr.zero_()
        if kin0 is not None:
            self.keys_in.copy_(kin0)
        if self.history is not None:
            self.history.zero_()
        return self

    def replay(self) -> None:
        self.graph.replay()

    def set_positions(self) -> None:
        self.pos.copy_(torch.tensor([self.eng.seq_len[s] for s in self.slots], dtype=torch.int32))

    def sync_positions(self) -> None:
        p = self.pos.tolist()
        for s, v in zip(self.slots, p):
            self.eng.seq_len[s] = int(v)


class EagerDecode:
    """Same interface as :class:`DecodeGraph` for devices without graphs (the CPU torch path
    used by the multi-process gloo tests): one decode step per ``_body()`` call."""

    def __init__(self, eng: StageEngine, rows: int, mode: str, slots: Optional[list] = None,
                 history_len: int = 0, split_head: bool = False):
        self.eng, self.rows, self.mode = eng, rows, mode
        self.slots = list(range(rows)) if slots is None else list(slots)
        self.tokens = torch.zeros(rows, dtype=torch.int32)
        self.h_in = torch.zeros((rows, eng.cfg.hidden_size), dtype=eng.dtype)
        self.history = torch.zeros((history_len, rows), dtype=torch.int32) if history_len else None
        self.step = 0
        self._out = None
        self.split_head = split_head
        self.keys = torch.zeros(rows, dtype=torch.int64)
        self.h_fin = torch.zeros((rows, eng.cfg.hidden_size), dtype=eng.dtype)
        self.keys_in = torch.zeros(rows, dtype=torch.int64)

    def _body(self) -> None:
        eng = self.eng
        if self.split_head and self.mode == "first":  # complete the previous step's argmax
            self.tokens.copy_(eng.finalize_keys(eng.head_keys(self.h_fin, None, keys=self.keys_in.clone())))
            if self.history is not None and self.step < self.history.shape[0]:
                self.history[self.step] = self.tokens
            self.step += 1
        h = eng.embed(self.tokens) if self.mode in ("full", "first") else self.h_in
        slot, pos = eng.prefill_rows(self.slots, [1] * self.rows)
        h = eng.forward(h, slot, pos)
        eng.advance(self.slots, [1] * self.rows)
        if self.split_head and self.mode == "last":
            self.keys.copy_(eng.head_keys(h))
        elif self.mode in ("full", "last"):
            self.tokens.copy_(eng.head(h).to(torch.int32))
            if self.history is not None and self.step < self.history.shape[0]:
                self.history[self.step] = self.tokens
            self.step += 1
        self._out = h

    replay = _body

    def capture(self, warmup: bool = True) -> "EagerDecode":
        return self

    @property
    def out_hidden(self) -> torch.Tensor:
        return self._out

    def sync_positions(self) -> None:
        pass
