"""Master-side placement scheduler.

The reference README describes a scheduling algorithm on the master node that calls
``ConfigSender`` (``/root/reference/README.md:7-8``) but the repo ships none - placement is
hand-written in ``send_config.py:5-44``. Its profiler produces the inputs such a scheduler
needs: per-token compute capability ``c_k``, max layers per device, cold-start latency
(``utils/node_profiler.py:46-62,368-476,1138-1172``).

``plan_stages`` implements it: split the ``L`` decoder layers into contiguous ranges, one per
device in chain order, minimising the bottleneck stage time

    t(stage) = sum(layer_cost) * speed_factor(device) + extras (embedding / lm_head)

subject to a per-device memory cap (weights + KV cache + workspace), by exact dynamic
programming over (layer, stage). Default costs are the bytes streamed per decode token
(batch-1 decode is HBM-bound on MI355X), which is what the profiler's ``c_k`` measures.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence

from ..config import LlamaConfig


@dataclass
class DeviceSpec:
    name: str = "mi355x"
    mem_bytes: float = 288e9          # HBM3E per MI355X
    reserve_bytes: float = 8e9        # runtime / workspace headroom
    speed: float = 1.0                # relative time multiplier (profiled c_k ratio)
    host: str = "127.0.0.1"
    config_port: int = 40700
    data_port: int = 40800


@dataclass
class StagePlan:
    index: int
    start: int
    end: int
    device: DeviceSpec
    has_embed: bool
    has_head: bool
    est_time: float
    weight_bytes: float
    kv_bytes: float

    @property
    def n_layers(self) -> int:
        return self.end - self.start


@dataclass
class Plan:
    stages: List[StagePlan] = field(default_factory=list)

    @property
    def bottleneck(self) -> float:
        return max(s.est_time for s in self.stages)

    def ranges(self) -> list:
        return [(s.start, s.end) for s in self.stages]

    def summary(self) -> str:
        return " | ".join(f"s{s.index}[{s.start},{s.end}){'E' if s.has_embed else ''}"
                          f"{'H' if s.has_head else ''} {s.est_time:.3g}" for s in self.stages)


def default_costs(cfg: LlamaConfig, elem_bytes: int = 2) -> tuple:
    layer = [float(cfg.layer_bytes(elem_bytes))] * cfg.num_hidden_layers
    head = float((cfg.vocab_size * cfg.hidden_size + cfg.hidden_size) * elem_bytes)
    embed = float(cfg.hidden_size * elem_bytes)  # one row gathered per token
    return layer, embed, head


def plan_stages(cfg: LlamaConfig, devices: Sequence[DeviceSpec] | int, *,
                layer_costs: Optional[Sequence[float]] = None, embed_cost: Optional[float] = None,
                head_cost: Optional[float] = None, kv_tokens: int = 0, elem_bytes: int = 2,
                min_layers: int = 1, head_split: bool = False, scratch: float = 0.0,
                stage_overhead: float = 0.0) -> Plan:
    """Exact min-max contiguous partition. ``devices`` is a list (chain order) or a count.
    ``head_split``: the lm_head is shared by the last and the first stage (pipeline.py), so each
    carries half of its cost and memory. ``scratch``: per-stage engine scratch bytes
    (:func:`scratch_bytes`), counted against every device's memory next to weights and KV.
    ``stage_overhead``: fixed cost of one stage step (measured costs:
    node_profiler.costs_for_planner), added to every stage before its device's speed factor."""
    if isinstance(devices, int):
        devices = [DeviceSpec() for _ in range(devices)]
    n, L = len(devices), cfg.num_hidden_layers
    if n < 1 or n * min_layers > L:
        raise ValueError(f"cannot place {L} layers on {n} stages (min {min_layers} each)")
    lc, ec, hc = default_costs(cfg, elem_bytes)
    lc = list(layer_costs) if layer_costs is not None else lc
    ec = ec if embed_cost is None else embed_cost
    hc = hc if head_cost is None else head_cost
    lbytes = float(cfg.layer_bytes(elem_bytes))
    kv_per_layer = float(cfg.kv_bytes_per_token_per_layer(elem_bytes)) * kv_tokens
    emb_bytes = float(cfg.vocab_size * cfg.hidden_size * elem_bytes)
    head_bytes = emb_bytes if not cfg.tie_word_embeddings else 0.0

    pre = [0.0]
    for c in lc:
        pre.append(pre[-1] + c)

    split = head_split and n > 1
    hfrac_last = 0.5 if split else 1.0

    def stage_cost(k: int, a: int, b: int) -> float:
        t = pre[b] - pre[a] + stage_overhead
        if k == 0:
            t += ec + (hc * 0.5 if split else 0.0)
        if k == n - 1:
            t += hc * hfrac_last
        return t * devices[k].speed

    def stage_mem(k: int, a: int, b: int) -> float:
        m = (b - a) * (lbytes + kv_per_layer) + scratch
        if k == 0:
            m += emb_bytes + (emb_bytes * 0.5 if split else 0.0)
        if k == n - 1:
            m += (emb_bytes * hfrac_last if not cfg.tie_word_embeddings or split else head_bytes) \
                + cfg.hidden_size * elem_bytes
        return m

    def fits(k: int, a: int, b: int) -> bool:
        d = devices[k]
        return stage_mem(k, a, b) <= d.mem_bytes - d.reserve_bytes

    INF = float("inf")
    # best[k][i] = min bottleneck placing layers [0, i) on stages 0..k-1 (stage k-1 ends at i)
    best = [[INF] * (L + 1) for _ in range(n + 1)]
    arg = [[-1] * (L + 1) for _ in range(n + 1)]
    best[0][0] = 0.0
    for k in range(1, n + 1):
        for i in range(k * min_layers, L - (n - k) * min_layers + 1):
            for j in range((k - 1) * min_layers, i - min_layers + 1):
                if best[k - 1][j] == INF or not fits(k - 1, j, i):
                    continue
                v = max(best[k - 1][j], stage_cost(k - 1, j, i))
                if v < best[k][i] - 1e-9:
                    best[k][i], arg[k][i] = v, j
    if best[n][L] == INF:
        raise ValueError("model does not fit on the given devices")
    cuts = [L]
    i = L
    for k in range(n, 0, -1):
        i = arg[k][i]
        cuts.append(i)
    cuts = cuts[::-1]
    plan = Plan()
    for k in range(n):
        a, b = cuts[k], cuts[k + 1]
        plan.stages.append(StagePlan(k, a, b, devices[k], k == 0, k == n - 1, stage_cost(k, a, b),
                                     stage_mem(k, a, b) - (b - a) * kv_per_layer - scratch,
                                     (b - a) * kv_per_layer))
    return plan


def kv_slots_for_memory(cfg: LlamaConfig, n_layers: int, max_seq: int, mem_bytes: float,
                        weight_bytes: float, reserve_bytes: float = 8e9, elem_bytes: int = 2,
                        microbatches: int = 1, max_per_microbatch: int = 128) -> int:
    """KV slots (sequences of ``max_seq`` tokens) per micro-batch that fit a stage of
    ``n_layers`` layers next to its weights: the static KV cache is sized from the device's
    HBM (288 GB on MI355X) instead of a fixed guess. Capped at
    ``max_per_microbatch`` (the largest hipGraph decode batch)."""
    per_slot = float(cfg.kv_bytes_per_token_per_layer(elem_bytes)) * n_layers * max_seq
    free = mem_bytes - reserve_bytes - weight_bytes
    if per_slot <= 0 or free < per_slot * microbatches:
        raise ValueError(f"no room for a KV cache of {max_seq} tokens x {n_layers} layers "
                         f"({free / 1e9:.1f} GB free after weights)")
    return int(min(max_per_microbatch, free // (per_slot * microbatches)))


def scratch_bytes(cfg: LlamaConfig, rows: int, sets: int = 1, max_seq: int = 4096,
                  head_rows: int = 0) -> float:
    """Device bytes a stage engine allocates besides weights and KV cache, per ``sets``
    concurrently replayed scratch sets sized for ``rows`` rows - the same formulas as
    StageEngine._alloc_runtime / decode_scratch: activations, attention split partials and
    their tickets, the coop-GEMV workspace, the gemm_sk slabs and split-K partials (> 128 rows)."""
    from ..ops import packing
    H, I, nh, hd = cfg.hidden_size, cfg.intermediate_size, cfg.num_attention_heads, cfg.head_dim
    dmr = packing.GEMV_MAX_ROWS
    R = max(rows, dmr)
    act = R * (2 * H + 2 * cfg.q_size + I) * 2 + R * (8 + 4)        # buffers + keys + tokens
    nsplit = int(min(16, max(1, -(-max_seq // 256))))
    ws_rows = max(dmr * nsplit, 4 * R)
    attn = ws_rows * (nh * hd * 4 + nh * 4 + cfg.num_key_value_heads * 4)
    shapes = [(cfg.qkv_size, H), (H, cfg.q_size), (cfg.mlp_in_size, H), (H, I)]
    if head_rows:
        shapes.append((head_rows, H))
    even = () if cfg.is_gpt2 else ((2 * I, H),)
    floats, groups = packing.coop_workspace_need(shapes, dmr, even_n=even)
    coop = max(floats, 1 << 24) * 4 + max(groups, 4096) * 4
    sk = (2 * 256 * 256 * 256 * 4 + 4 * 256 * 4) if R > dmr else 0
    # split-K partials of the residual projections (hip.PARTIAL_MAX_SPLIT x <= 1024 rows x H fp32)
    part = 8 * min(R, 1024) * H * 4 if (R > dmr and not cfg.is_gpt2) else 0
    ssb = R * (H // 64) * 4 if (R > dmr and not cfg.is_gpt2 and H % 256 == 0) else 0  # fused-norm sums
    return float(sets * (act + attn + coop + sk + part + ssb))


def stage_memory(cfg: LlamaConfig, n_layers: int, *, slots: int, max_seq: int, prefill_rows: int,
                 has_embed: bool = False, head_rows: int = 0, scratch_sets: int = 1,
                 io_rows: int = 0, elem_bytes: int = 2) -> dict:
    """Device bytes of one pipeline stage as the engine allocates them (weights, static KV cache,
    scratch) - the memory table the bench's stage sizing relies on (profiles/memory_table.md).
    ``head_rows``: lm_head rows held on this stage (split head: a part of the vocabulary);
    ``io_rows``: per-micro-batch hidden/token hand-off buffers (PipelineStage.h_out/tok_out)."""
    H = cfg.hidden_size
    w = n_layers * cfg.layer_bytes(elem_bytes)
    if has_embed:
        w += cfg.vocab_size * H * elem_bytes
    if head_rows:
        w += head_rows * H * elem_bytes + H * elem_bytes          # lm_head part + final norm
    kv = n_layers * cfg.kv_bytes_per_token_per_layer(elem_bytes) * slots * max_seq
    scratch = scratch_bytes(cfg, prefill_rows, scratch_sets, max_seq, head_rows)
    io = io_rows * (H * elem_bytes + 4 + 8)
    return {"weights": float(w), "kv": float(kv), "scratch": float(scratch), "io": float(io),
            "total": float(w + kv + scratch + io)}


def build_chain_configs(plan: Plan, ingress_stage: int = 0) -> list:
    """ConfigSender payloads (reference schema, config_sender.py:33-40) for a ring chain."""
    n = len(plan.stages)
    out = []
    for k, st in enumerate(plan.stages):
        nxt = plan.stages[(k + 1) % n]
        first = plan.stages[0]
        out.append({
            "src_addr": f"tcp://*:{st.device.data_port}",
            "dst_addr": f"tcp://{nxt.device.host}:{nxt.device.data_port}",
            "can_receive_user_request": k == ingress_stage,
            "first_node_addr": f"tcp://{first.device.host}:{first.device.data_port}" if k == ingress_stage else "",
            "shards_start": st.start,
            "shards_end": st.end,
        })
    return out
