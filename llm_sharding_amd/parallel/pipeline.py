"""Micro-batched pipeline-parallel decode over RCCL (one process per GPU).

The reference chain passes ONE token around the ring at a time: stage i receives a pickled
``next_state_info`` over ZMQ, runs its layers, pushes the result on (SURVEY.md §3.2,
``/root/reference/utils/node_worker.py:493-559``), so at most 1/N of the devices ever work.

Here each rank is one stage (a contiguous layer range from the master scheduler, resident on
its own MI355X). M micro-batches of B sequences are in flight; for every (step, micro-batch)
a rank:

    irecv(hidden | token ids)  ->  stream-wait  ->  replay the micro-batch's hipGraph
    (layers [+ embed] [+ final-norm/lm_head/argmax])  ->  isend(hidden | token ids)

The RCCL p2p ops run on the NCCL streams (one communicator per ring edge) and are ordered
against the compute streams by events - no host synchronisation per token; the host runs
ahead until the HIP queues fill. Micro-batch mb runs on compute stream mb % S (S concurrent
streams per stage, each with its own engine scratch set), so S decode graphs share a GPU at
once. Hidden states go rank r -> r+1 over xGMI, token ids go last -> 0 (the ring back-edge,
``receive_next_token`` with the embedding co-located on the first stage).
"""
from __future__ import annotations

import contextlib
import os
import time
from typing import Optional

import torch

from ..config import get_preset
from ..runtime.engine import DecodeGraph, EagerDecode, RandomSource, StageEngine
from ..utils import tracing
from .scheduler import plan_stages, scratch_bytes, stage_memory


class DistP2P:
    """Point-to-point over torch.distributed (RCCL on GPUs, gloo on CPU), with one process group
    - i.e. one RCCL communicator and one communication stream - per directed ring edge
    ``r -> r+1`` (the back-edge ``N-1 -> 0`` included).

    Why: RCCL executes the p2p ops of a communicator in issue order on one stream, and an
    ``ncclSend`` may wait for its matching ``ncclRecv`` to be running. On a single shared
    communicator stage 0's stream holds ``send(mb1 -> 1)`` ahead of ``recv(back-edge mb0)``
    while the last stage's holds ``send(back-edge mb0)`` ahead of ``recv(mb1)``: a cycle that
    only the transport's eager buffering breaks (small messages), not the API contract. With a
    communicator per edge each stream carries one direction in FIFO order, so the pipeline's
    dataflow order alone guarantees progress, and sends / receives on different edges overlap.
    Must be constructed on every rank at the same point (``new_group`` is collective).

    ``ranks``: the global ranks of THIS pipeline's stages in stage order (stage indices passed
    to isend/recv are translated through it; default: every rank, one pipeline). ``rings``: the
    rank lists of every pipeline replica of a data-parallel job (each process must create every
    replica's edge groups, in the same order)."""

    def __init__(self, ranks: Optional[list] = None, rings: Optional[list] = None):
        import torch.distributed as dist
        self.groups = {}
        self.ranks = ranks
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            n = dist.get_world_size()
            for ring in (rings if rings is not None else [list(range(n))]):
                for i in range(len(ring) if len(ring) > 1 else 0):
                    a, b = ring[i], ring[(i + 1) % len(ring)]
                    self.groups[(a, b)] = dist.new_group([a, b])
            if self.ranks is None:
                self.ranks = list(range(n))

    def _global(self, stage: int) -> int:
        return self.ranks[stage] if self.ranks is not None else stage

    def _group(self, src: int, dst: int):
        return self.groups.get((src, dst))  # non-ring edges (none in the pipeline): default group

    def isend(self, t: torch.Tensor, dst: int):
        import torch.distributed as dist
        dst = self._global(dst)
        return dist.isend(t, dst, group=self._group(dist.get_rank(), dst))

    def recv(self, t: torch.Tensor, src: int) -> None:
        self.irecv(t, src).wait()

    def irecv(self, t: torch.Tensor, src: int):
        import torch.distributed as dist
        src = self._global(src)
        return dist.irecv(t, src, group=self._group(src, dist.get_rank()))


PREFLIGHT_EXIT = 75  # a rank whose ring edge failed the preflight exits with this code


def _parse_fault(spec: str):
    """``LSA_PREFLIGHT_FAULT="a->b"``: test hook - global rank a never sends on edge a -> b."""
    if not spec:
        return None
    a, b = spec.split("->")
    return int(a), int(b)


def _startup_watchdog(rank: int, timeout_s: Optional[float] = None):
    """Started before the RCCL process group is created, cancelled after the ring preflight's
    results are gathered: if RCCL's own setup (eager communicator init, the world all-gather)
    has not finished within ``timeout_s`` (``LSA_STARTUP_TIMEOUT_S``, default 180) the rank says
    so and exits with :data:`PREFLIGHT_EXIT`."""
    import sys
    import threading
    timeout_s = float(os.environ.get("LSA_STARTUP_TIMEOUT_S", "180")) if timeout_s is None else timeout_s

    def _fail():
        print(f"[bench] PREFLIGHT FAILED on rank {rank}: RCCL process-group setup did not complete within "
              f"{timeout_s:.0f} s; exiting {PREFLIGHT_EXIT}", file=sys.stderr, flush=True)
        os._exit(PREFLIGHT_EXIT)

    wd = threading.Timer(timeout_s, _fail)
    wd.daemon = True
    wd.start()
    return wd


def preflight_edges(p2p: "DistP2P", srank: int, pp: int, dev, timeout_s: Optional[float] = None,
                    iters: int = 5, inject: bool = True) -> dict:
    """First-light check of this rank's two ring edges before anything heavy runs: one small
    tensor goes ``stage -> stage+1`` on the outgoing edge's communicator while one arrives from
    ``stage-1`` on the incoming one, ``iters`` times (the first round, which may build the
    communicators lazily, is not timed). Returns ``{"a->b": us}`` for the INCOMING edge (global
    ranks; median round time). A watchdog bounds the whole check: if either edge has not
    completed within ``timeout_s`` (``LSA_PREFLIGHT_TIMEOUT_S``, default 30) the rank prints which
    edge and exits with :data:`PREFLIGHT_EXIT` at once (``os._exit``: a communicator stuck on a
    dead peer cannot be torn down) - the bench's per-rank supervisor then decides on a fallback."""
    import sys
    import threading
    if pp < 2:
        return {}
    timeout_s = float(os.environ.get("LSA_PREFLIGHT_TIMEOUT_S", "30")) if timeout_s is None else timeout_s
    me, nxt, prv = p2p._global(srank), p2p._global((srank + 1) % pp), p2p._global((srank - 1) % pp)
    fault = _parse_fault(os.environ.get("LSA_PREFLIGHT_FAULT", "")) if inject else None
    state = {"pending": f"{prv}->{me} (receive) and {me}->{nxt} (send)"}

    def _fail():
        print(f"[bench] PREFLIGHT FAILED on rank {me}: edge {state['pending']} did not complete within "
              f"{timeout_s:.0f} s; exiting {PREFLIGHT_EXIT}", file=sys.stderr, flush=True)
        os._exit(PREFLIGHT_EXIT)

    wd = threading.Timer(timeout_s, _fail)
    wd.daemon = True
    wd.start()
    out = torch.empty(64, dtype=torch.float32, device=dev)
    inp = torch.empty(64, dtype=torch.float32, device=dev)
    times = []
    for it in range(iters + 1):
        out.fill_(float(me * 1000 + it))
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        state["pending"] = f"{prv}->{me} (receive) and {me}->{nxt} (send)"
        try:
            sw = None if fault == (me, nxt) else p2p.isend(out, (srank + 1) % pp)
            rw = p2p.irecv(inp, (srank - 1) % pp)
            rw.wait()
            state["pending"] = f"{me}->{nxt} (send)"
            if sw is not None:
                sw.wait()
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
        except Exception as e:  # noqa: BLE001 - an edge that FAILS fast is as dead as one that hangs
            wd.cancel()
            print(f"[bench] PREFLIGHT FAILED on rank {me}: edge {state['pending']} raised "
                  f"{type(e).__name__}: {e}; exiting {PREFLIGHT_EXIT}", file=sys.stderr, flush=True)
            os._exit(PREFLIGHT_EXIT)
        times.append(time.perf_counter() - t0)
        if float(inp[0]) != float(prv * 1000 + it):
            wd.cancel()
            raise RuntimeError(f"preflight: edge {prv}->{me} delivered {float(inp[0])}, expected {prv * 1000 + it}")
    wd.cancel()
    t = sorted(times[1:])
    return {f"{prv}->{me}": round(t[len(t) // 2] * 1e6, 1)}


class LocalP2P:
    """In-process device-copy transport: several stages in ONE process (e.g. N stages on one
    GPU, SURVEY.md §4 'local device-copy backend'). Messages are snapshot copies queued per
    (src, dst); stages must be driven in pipeline order (see :func:`drive_local_pipeline`)."""

    class _Done:
        def wait(self):
            return None

    def __init__(self):
        self.boxes: dict = {}

    def bind(self, rank: int) -> "LocalP2P._Endpoint":
        return LocalP2P._Endpoint(self, rank)

    class _Endpoint:
        def __init__(self, hub, rank):
            self.hub, self.rank = hub, rank

        def isend(self, t, dst):
            # snapshot on the sender's current stream, then an event behind the copy: the
            # receiver's stream waits on it before reading the snapshot
            snap, ev = t.clone(), None
            if t.is_cuda:
                ev = torch.cuda.Event()
                ev.record()
            self.hub.boxes.setdefault((self.rank, dst), []).append((snap, ev))
            return LocalP2P._Done()

        def recv(self, t, src):
            box = self.hub.boxes.get((src, self.rank))
            if not box:
                raise RuntimeError(f"local p2p: no message from stage {src} to {self.rank} (drive order?)")
            snap, ev = box.pop(0)
            if ev is not None:
                cur = torch.cuda.current_stream(t.device)
                cur.wait_event(ev)
                t.copy_(snap)
                snap.record_stream(cur)  # the allocator must not recycle it before this copy ran
            else:
                t.copy_(snap)


def _percentile(xs, q):
    if not xs:
        return float("nan")
    s = sorted(xs)
    k = (len(s) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(s) - 1)
    return s[lo] + (s[hi] - s[lo]) * (k - lo)


class PipelineStage:
    """One rank's share of a pipelined decode: engine + per-micro-batch graphs and buffers."""

    def __init__(self, cfg, rank: int, world: int, start: int, end: int, device, batch: int,
                 microbatches: int, max_seq: int, source, use_graph: bool = True,
                 max_prefill_rows: int = 2048, dtype=torch.bfloat16, p2p=None,
                 split_head: Optional[bool] = None, weight_dtype: str = "bf16", streams: int = 1,
                 pp_streams: Optional[bool] = None, engine: Optional[StageEngine] = None):
        """``engine``: reuse a loaded StageEngine (its weights, KV cache and scratch) instead of
        building one - e.g. a batch-1 latency pass after a throughput pass; it must cover this
        stage's layers and hold >= batch x microbatches KV slots."""
        self.cfg, self.rank, self.world = cfg, rank, world
        self.p2p = p2p if p2p is not None else DistP2P()
        self.first, self.last = rank == 0, rank == world - 1
        self.B, self.M = batch, microbatches
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.use_graph = use_graph and self.gpu
        self.dtype = torch.bfloat16 if self.gpu else dtype
        # Split lm_head (GPU pipelines of >= 2 stages): the last stage covers vocab [0, V1), the
        # first stage [V1, V). The ring back-edge then carries the raw final hidden + partial
        # argmax keys instead of token ids, and the first stage completes the argmax at the
        # start of its next step - the ~0.4-layer lm_head no longer sits on one stage only.
        V = cfg.head_rows
        v1 = (V // 2) // 128 * 128
        self.split = (world > 1 and v1 > 0) if split_head is None else split_head
        head_cols = None
        if self.split and self.last:
            head_cols = (0, v1)
        elif self.split and self.first:
            head_cols = (v1, V)
        if engine is not None:
            ok = (engine.start, engine.end) == (start, end) and engine.max_slots >= batch * microbatches
            if engine.has_head:
                ok = ok and (engine.head_v0, engine.head_v1) == (head_cols or (0, cfg.head_rows))
            if not ok:
                raise ValueError("PipelineStage: the shared engine does not match this stage")
            self.eng = engine
        else:
            self.eng = StageEngine(cfg, start, end, device, self.dtype, has_embed=self.first,
                                   has_head=self.last or (self.split and self.first), source=source,
                                   max_slots=batch * microbatches, max_seq=max_seq,
                                   max_prefill_rows=max(max_prefill_rows, batch), head_cols=head_cols,
                                   weight_dtype=weight_dtype)
        H = cfg.hidden_size
        self.h_out = [torch.zeros((batch, H), dtype=self.dtype, device=self.device) for _ in range(microbatches)]
        self.tok_out = [torch.zeros(batch, dtype=torch.int32, device=self.device) for _ in range(microbatches)]
        if self.split:
            self.keys_out = [torch.zeros(batch, dtype=torch.int64, device=self.device) for _ in range(microbatches)]
            self.seed = [None] * microbatches   # stage 0: (h_fin, keys) of each micro-batch's prefill
            self.final_tokens = [None] * microbatches
        self.graphs: list = []
        self.send_works: dict = {}
        self.tokens_ready = [True] * microbatches  # stage 0: next-step token ids are in place
        self.tl = tracing.from_env(rank, self.device if self.gpu else "cpu")  # LSA_TRACE=dir
        # Concurrent micro-batches (single-stage GPU pipelines only): micro-batch mb replays on
        # stream mb % S with its own scratch set, so up to S decode graphs share the GPU at once.
        # A Llama-2-7B decode graph alone leaves CUs idle (its projections have too few tiles to
        # fill 256 CUs), and S graphs side by side raise throughput (scripts/concurrency_probe.py).
        # Multi-stage pipelines do the same (``pp_streams``; LSA_PP_STREAMS=0 keeps one compute
        # stream per stage): every GPU enqueues its p2p and compute work in one global (step,
        # micro-batch) order on every stream, and each op waits only on ops of an equal or
        # earlier (step, micro-batch) on any GPU, so the waits-for relation stays acyclic however
        # streams share hardware queues. Exercised in-process (LocalP2P + stream events, GPU tests)
        # and over gloo; RCCL between GPUs adds per-edge FIFO ordering, which the same order meets.
        if pp_streams is None:
            pp_streams = os.environ.get("LSA_PP_STREAMS", "1") == "1"
        multi = world == 1 or pp_streams
        self.S = max(1, min(streams, microbatches)) if (self.gpu and self.use_graph and multi) else 1
        self.streams = [torch.cuda.Stream(self.device) for _ in range(self.S)] if self.S > 1 else []

    # ---------------------------------------------------------------- p2p helpers
    def _send(self, t: torch.Tensor, dst: int, key):
        self.send_works[key] = self.p2p.isend(t, dst)

    def _wait_send(self, key):
        w = self.send_works.pop(key, None)
        if w is not None:
            w.wait()

    def _recv(self, t: torch.Tensor, src: int):
        self.p2p.recv(t, src)

    # ---------------------------------------------------------------- prefill
    def slots(self, mb: int) -> list:
        return list(range(mb * self.B, (mb + 1) * self.B))

    def prefill(self, prompts: Optional[torch.Tensor], prompt_len: int) -> Optional[list]:
        """Prefill every micro-batch through the pipeline. ``prompts``: [M, B, P] int (rank 0).
        Returns (on rank 0) the first generated token per micro-batch ([B] int32 tensors)."""
        firsts = []
        for mb in range(self.M):
            tok = self.prefill_mb(mb, prompts, prompt_len, recv_token=True)
            if tok is not None:
                firsts.append(tok)
        return firsts if self.first else None

    def prefill_mb(self, mb: int, prompts, prompt_len: int, recv_token: bool = True):
        """Prefill one micro-batch on this stage. Returns the first generated ids on the stage
        that ends up holding them (rank 0 after the back-edge, or a single-stage pipeline)."""
        eng, B, P, H = self.eng, self.B, prompt_len, self.cfg.hidden_size
        sl = self.slots(mb)
        slot, pos = eng.prefill_rows(sl, [P] * B)
        if self.first:
            h = eng.embed(prompts[mb].reshape(-1).to(self.device))
        else:
            h = torch.empty((B * P, H), dtype=self.dtype, device=self.device)
            self._recv(h, self.rank - 1)
        with self.tl.span("prefill", mb=mb, rows=B * P):
            h = eng.forward(h, slot, pos)
        eng.advance(sl, [P] * B)
        if self.last:
            last_rows = [i * P + P - 1 for i in range(B)]
            if self.split:
                keys = eng.head_keys(h, last_rows)
                hl = h[torch.tensor(last_rows, device=h.device)].contiguous()
                self._send(hl, 0, ("pfh", mb))
                self._send(keys, 0, ("pf", mb))
                self._wait_send(("pfh", mb))
                self._wait_send(("pf", mb))
            else:
                tok = eng.head(h, last_rows).to(torch.int32)
                if self.world == 1:
                    return tok
                self._send(tok, 0, ("pf", mb))
                self._wait_send(("pf", mb))
        else:
            self._send(h.clone(), self.rank + 1, ("pf", mb))
            self._wait_send(("pf", mb))
        if self.first and recv_token:
            return self.recv_first_token(mb)
        return None

    def recv_first_token(self, mb: int = 0) -> torch.Tensor:
        if self.split:
            hf = torch.zeros((self.B, self.cfg.hidden_size), dtype=self.dtype, device=self.device)
            keys = torch.zeros(self.B, dtype=torch.int64, device=self.device)
            self._recv(hf, self.world - 1)
            self._recv(keys, self.world - 1)
            self.seed[mb] = (hf, keys.clone())  # the decode graph recomputes token 0 from these
            return self._complete(hf, keys)
        tok = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        self._recv(tok, self.world - 1)
        return tok

    def _complete(self, h_fin: torch.Tensor, keys: torch.Tensor) -> torch.Tensor:
        """Stage 0 (split head): finish the argmax over its vocab slice -> token ids."""
        k = self.eng.head_keys(h_fin, None, keys=keys.clone())
        return self.eng.finalize_keys(k)

    # ---------------------------------------------------------------- decode
    @property
    def history_stage(self) -> bool:
        """Does this stage hold the generated-token history (last stage, or stage 0 when the
        lm_head is split)?"""
        return self.first if self.split else self.last

    def build_graphs(self, first_tokens: Optional[list], history_len: int) -> None:
        mode = "full" if self.world == 1 else ("first" if self.first else ("last" if self.last else "mid"))
        self.mode = mode
        self.graphs = []
        for mb in range(self.M):
            # micro-batches that share a stream replay one after another: one scratch set each
            extra = {"scratch": mb % self.S} if self.gpu else {}
            cls = DecodeGraph if self.gpu else EagerDecode
            if self.split and mode in ("first", "last"):
                # stage 0 re-derives token s at step s: one more history row than the last stage keeps
                g = cls(self.eng, self.B, mode, slots=self.slots(mb),
                        history_len=history_len + 1 if self.first else 0, split_head=True, **extra)
                if self.first and self.seed[mb] is not None:
                    g.h_fin.copy_(self.seed[mb][0])
                    g.keys_in.copy_(self.seed[mb][1])
            else:
                g = cls(self.eng, self.B, mode, slots=self.slots(mb),
                        history_len=history_len if self.last else 0, **extra)
                if first_tokens is not None and mode in ("full", "first"):
                    g.tokens.copy_(first_tokens[mb])
            if self.use_graph:
                if self.graph_comm:
                    self._attach_comm(g)
                g.capture()
            self.graphs.append(g)

    @property
    def graph_comm(self) -> bool:
        """Hand-offs captured inside the decode graphs: a graph-capturable transport (IPC ring),
        one compute stream (graphs of one edge must not run concurrently: the ring's device
        counters order its messages) and every decode message small enough for the ring. The
        first stage's back-edge receive stays outside (it is skipped after a drain)."""
        if not (self.gpu and self.use_graph and self.world > 1 and self.S == 1
                and getattr(self.p2p, "graph_capturable", False)
                and os.environ.get("LSA_GRAPH_COMM", "1") == "1"):
            return False
        H = self.cfg.hidden_size
        probe = [torch.empty((self.B, H), dtype=self.dtype, device=self.device),
                 torch.empty(self.B, dtype=torch.int64, device=self.device),
                 torch.empty(self.B, dtype=torch.int32, device=self.device)]
        return all(self.p2p.fits(t) for t in probe)

    def _attach_comm(self, g: DecodeGraph) -> None:
        p2p, r = self.p2p, self.rank
        if self.mode in ("mid", "last"):
            g.pre_comm = lambda: p2p.recv(g.h_in, r - 1)
        if self.mode == "last" and self.split:
            def post():
                p2p.isend(g.out_hidden, 0)
                p2p.isend(g.keys, 0)
        elif self.mode == "last":
            def post():
                p2p.isend(g.tokens, 0)
        else:
            def post():
                p2p.isend(g.out_hidden, r + 1)
        g.post_comm = post
        g.in_graph_comm = True

    def _run_mb(self, g: DecodeGraph):
        if self.use_graph:
            g.replay()
        else:
            g._body()

    def step(self, s: int, events: Optional[list] = None) -> None:
        """One decode step for every micro-batch (the host never blocks on the GPU here)."""
        for mb in range(self.M):
            self.step_mb(s, mb, events)

    def _mb_stream(self, mb: int):
        """Stream context of micro-batch ``mb`` (concurrent mode), ordered after whatever the
        caller enqueued on its current stream before."""
        if self.S == 1:
            return contextlib.nullcontext()
        st = self.streams[mb % self.S]
        if mb < self.S:
            st.wait_stream(torch.cuda.current_stream(self.device))
        return torch.cuda.stream(st)

    def join_streams(self) -> None:
        """Make the current stream wait for the concurrent micro-batch streams."""
        cur = torch.cuda.current_stream(self.device) if self.gpu else None
        for st in self.streams:
            cur.wait_stream(st)

    def step_mb(self, s: int, mb: int, events: Optional[list] = None) -> None:
        with self._mb_stream(mb):
            self._step_mb(s, mb, events)

    def _step_mb(self, s: int, mb: int, events: Optional[list] = None) -> None:
        g = self.graphs[mb]
        tl = self.tl
        in_graph = getattr(g, "in_graph_comm", False)
        if self.world > 1 and not (in_graph and not self.first):
            with tl.span("recv", mb=mb, step=s):
                if self.first:
                    if not self.tokens_ready[mb]:
                        if self.split:
                            self._recv(g.h_fin, self.world - 1)
                            self._recv(g.keys_in, self.world - 1)
                        else:
                            self._recv(g.tokens, self.world - 1)
                    self.tokens_ready[mb] = False
                else:
                    self._recv(g.h_in, self.rank - 1)
        with tl.span("decode", mb=mb, step=s):
            self._run_mb(g)
        if events is not None and self.gpu:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            events.append((s, mb, ev))
        if self.world > 1 and not in_graph:
            if self.last and self.split:
                # private copies: the next replay rewrites the engine's hidden buffer / keys
                self._wait_send(("hb", mb))
                self._wait_send(("tok", mb))
                self.h_out[mb].copy_(g.out_hidden.reshape(self.h_out[mb].shape))
                self.keys_out[mb].copy_(g.keys)
                self._send(self.h_out[mb], 0, ("hb", mb))
                self._send(self.keys_out[mb], 0, ("tok", mb))
            elif self.last:
                # the next replay rewrites g.tokens: send from a private copy, reused only
                # after the previous send of this micro-batch completed
                self._wait_send(("tok", mb))
                self.tok_out[mb].copy_(g.tokens)
                self._send(self.tok_out[mb], 0, ("tok", mb))
            else:
                self._wait_send(("h", mb))
                self.h_out[mb].copy_(g.out_hidden.reshape(self.h_out[mb].shape))
                self._send(self.h_out[mb], self.rank + 1, ("h", mb))

    def drain(self):
        """End of a phase: stage 0 collects the token ids the last stage produced in the final
        step (the ring back-edge), then every outstanding send is waited for."""
        if self.world > 1 and self.first:
            for mb, g in enumerate(self.graphs):
                if not self.tokens_ready[mb]:
                    with self._mb_stream(mb), (self.eng.use_scratch(mb % self.S) if self.S > 1
                                               else contextlib.nullcontext()):
                        self._drain_mb(mb, g)
        for k in list(self.send_works):
            self._wait_send(k)
        self.join_streams()
        chk = getattr(self.p2p, "check", None)
        if chk is not None:  # a transport with device-side timeouts (IPC ring): surface them here
            chk()

    def _drain_mb(self, mb: int, g) -> None:
        if self.split:
            # the last step's keys: complete them eagerly; the inputs stay in place, so a later
            # replay re-derives the same token first
            self._recv(g.h_fin, self.world - 1)
            self._recv(g.keys_in, self.world - 1)
            self.final_tokens[mb] = self._complete(g.h_fin, g.keys_in)
        else:
            self._recv(g.tokens, self.world - 1)
        self.tokens_ready[mb] = True


def run_pipeline_generate(cfg, source, prompts: Optional[torch.Tensor], n_new: int, rank: int, world: int,
                          device="cpu", batch: int = 1, microbatches: int = 1, max_seq: int = 256,
                          plan=None, dtype=torch.float32, streams: int = 1, p2p=None) -> Optional[torch.Tensor]:
    """Greedy generation through the micro-batched pipeline (torch.distributed already
    initialised; gloo on CPU or nccl/RCCL on GPUs). ``prompts`` [M, B, P] on rank 0.
    ``p2p``: the stage hand-off transport (default DistP2P; e.g. ipc_ring.IpcRingP2P).
    Returns [n_new, M, B] generated ids on rank 0 (gathered from the last stage)."""
    import torch.distributed as dist
    plan = plan or plan_stages(cfg, world, head_split=world > 1)
    st = plan.stages[rank]
    P = int(prompts.shape[-1]) if prompts is not None else 0
    if world > 1:
        pl = torch.tensor([P], dtype=torch.int64)
        dist.broadcast(pl, 0)
        P = int(pl[0])
    stage = PipelineStage(cfg, rank, world, st.start, st.end, device, batch, microbatches, max_seq, source,
                          use_graph=True, max_prefill_rows=batch * P, dtype=dtype, streams=streams, p2p=p2p)
    firsts = stage.prefill(prompts, P)
    stage.build_graphs(firsts, history_len=n_new - 1)
    for s in range(n_new - 1):
        stage.step(s)
    stage.drain()
    if stage.gpu:
        torch.cuda.synchronize()
    out = None
    if stage.split:
        if rank == 0:  # history rows: token s re-derived at step s (s = 0 .. n_new-2) + drained last
            hist = torch.stack([g.history[:n_new - 1] for g in stage.graphs], dim=1).cpu()
            last = torch.stack([t.cpu() for t in stage.final_tokens], dim=0)[None]
            return torch.cat([hist, last], dim=0) if n_new > 1 else hist[:1]
        return None
    if stage.last:
        hist = torch.stack([g.history for g in stage.graphs], dim=1).cpu()  # [n_new-1, M, B]
        out = hist
    if world > 1:
        if stage.last:
            dist.send(out.contiguous(), 0) if rank != 0 else None
        if rank == 0 and not stage.last:
            out = torch.zeros((n_new - 1, microbatches, batch), dtype=torch.int32)
            dist.recv(out, world - 1)
    if rank == 0:
        first = torch.stack([f.cpu() for f in firsts], dim=0)[None]  # [1, M, B]
        return torch.cat([first, out], dim=0)
    return None


def drive_local_pipeline(cfg, source, prompts: torch.Tensor, n_new: int, n_stages: int, device,
                         batch: int = 1, microbatches: int = 1, max_seq: int = 256, plan=None,
                         dtype=torch.bfloat16, use_graph: bool = True, streams: int = 1) -> torch.Tensor:
    """All stages of a pipeline in ONE process (one device), connected by :class:`LocalP2P`
    and driven in pipeline order. Same PipelineStage code as the multi-process RCCL path."""
    if n_stages < 2:
        raise ValueError("drive_local_pipeline needs >= 2 stages (use run_pipeline_generate for 1)")
    plan = plan or plan_stages(cfg, n_stages)
    hub = LocalP2P()
    P = int(prompts.shape[-1])
    stages = [PipelineStage(cfg, r, n_stages, st.start, st.end, device, batch, microbatches, max_seq, source,
                            use_graph=use_graph, max_prefill_rows=batch * P, dtype=dtype, p2p=hub.bind(r),
                            streams=streams, pp_streams=streams > 1)
              for r, st in enumerate(plan.stages)]
    firsts = []
    for mb in range(microbatches):
        for st in stages:
            st.prefill_mb(mb, prompts if st.first else None, P, recv_token=False)
        firsts.append(stages[0].recv_first_token(mb))
    for st in stages:
        st.build_graphs(firsts if st.first else None, history_len=n_new - 1)
    for s in range(n_new - 1):
        for mb in range(microbatches):
            for st in stages:
                st.step_mb(s, mb)
    for st in stages:
        st.drain()
    if stages[0].gpu:
        torch.cuda.synchronize()
    if stages[0].split:
        hist = torch.stack([g.history[:n_new - 1] for g in stages[0].graphs], dim=1).cpu()
        last = torch.stack([t.cpu() for t in stages[0].final_tokens], dim=0)[None]
        return torch.cat([hist, last], dim=0)
    hist = torch.stack([g.history for g in stages[-1].graphs], dim=1).cpu()
    first = torch.stack([f.cpu() for f in firsts], dim=0)[None]
    return torch.cat([first, hist], dim=0)


LAT_WARMUP = 4  # untimed steps of the batch-1 latency pass


def _tpot_from_events(events: list) -> list:
    """Per-token latencies (ms) between consecutive decode replays of each micro-batch."""
    by_mb: dict = {}
    for s, mb, ev in events:
        by_mb.setdefault(mb, []).append(ev)
    out = []
    for evs in by_mb.values():
        for a, b in zip(evs, evs[1:]):
            out.append(a.elapsed_time(b))
    return out


def _latency_pass(cfg, stage: "PipelineStage", srank: int, pp: int, st, dev, max_seq: int, prompts,
                  prompt_len: int, steps: int, dist, sync, p2p, rows: int = 1) -> tuple:
    """Batch-``rows`` decode through the pipeline on the already loaded stage engine (KV slots
    0..rows-1 are reused): prefill ``rows`` prompts, LAT_WARMUP untimed steps, ``steps`` timed
    ones. Returns (p50 per-token latency in ms on the last stage - 0.0 elsewhere -, timed wall
    seconds)."""
    eng = stage.eng
    eng.reset(list(range(rows)))
    b1 = PipelineStage(cfg, srank, pp, st.start, st.end, dev, rows, 1, max_seq, None,
                       use_graph=stage.use_graph, dtype=stage.dtype, p2p=p2p, engine=eng)
    b1.tl = stage.tl
    p1 = prompts[:1, :rows].contiguous() if prompts is not None else None
    firsts = b1.prefill(p1, prompt_len)
    b1.build_graphs(firsts, history_len=LAT_WARMUP + steps)
    for s in range(LAT_WARMUP):
        b1.step(s)
    b1.drain()
    sync()
    if dist:
        dist.barrier()
    sync()
    events: list = []
    t0 = time.perf_counter()
    for s in range(steps):
        b1.step(LAT_WARMUP + s, events if b1.last else None)
    b1.drain()
    sync()
    if dist:
        dist.barrier()
    sync()
    el = time.perf_counter() - t0
    tp = _tpot_from_events(events) if b1.last else []
    return (_percentile(tp, 0.5) if tp else 0.0), el


def rank_identity(rank: int, dev: torch.device) -> dict:
    """Which device this rank really runs on: host, pid, visibility env and, on a GPU, the
    device's UUID and PCI address (from the HIP runtime, not from the rank number) - so a
    multi-GPU JSON line proves that its N ranks ran on N distinct GPUs."""
    import socket
    info = {"rank": rank, "host": socket.gethostname(), "pid": os.getpid(),
            "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
            "visible": next((os.environ[k] for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                                      "CUDA_VISIBLE_DEVICES") if os.environ.get(k)), None)}
    if dev.type == "cuda":
        p = torch.cuda.get_device_properties(dev)
        info.update(device=f"{p.name} ({getattr(p, 'gcnArchName', '?')})", device_index=dev.index,
                    uuid=str(getattr(p, "uuid", "")),
                    pci_bus_id="%04x:%02x:%02x" % (getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", 0),
                                                   getattr(p, "pci_device_id", 0)))
    else:
        info.update(device="cpu", device_index=None, uuid=f"cpu:{info['host']}:{info['pid']}", pci_bus_id=None)
    return info


def gather_topology(dist, rank: int, dev: torch.device, rings: list, transport: str, gpu: bool,
                    p2p=None) -> dict:
    """World size / backend of the process group, every rank's identity and the transport of
    every ring edge, gathered to all ranks. Raises when RCCL ranks share a device (a mis-set
    HIP_VISIBLE_DEVICES would otherwise pass as an N-GPU measurement)."""
    me = rank_identity(rank, dev)
    if dist is not None:
        allr = [None] * dist.get_world_size()
        dist.all_gather_object(allr, me)
        world, backend = dist.get_world_size(), str(dist.get_backend())
    else:
        allr, world, backend = [me], 1, None
    edges = {}
    for ring in rings:
        for i in range(len(ring) if len(ring) > 1 else 0):
            a, b = ring[i], ring[(i + 1) % len(ring)]
            kind = "ipc" if transport == "ipc" and gpu else ("rccl" if gpu else "gloo")
            edges[f"{a}->{b}"] = kind
    if p2p is not None and getattr(p2p, "alloc_kinds", None):
        edges["ipc_alloc"] = sorted(set(str(v) for v in p2p.alloc_kinds.values()))
    # a device is named by its PCI address where the runtime reports one, else by its UUID; a rank
    # with neither (some runtimes report zeros) is not judged (distinct_devices: None)
    def ident(r):
        if r.get("pci_bus_id") and r["pci_bus_id"] != "0000:00:00":
            return (r["host"], r["pci_bus_id"])
        u = str(r.get("uuid") or "")
        return (r["host"], u) if u.strip("0-") else None
    ids = [ident(r) for r in allr]
    distinct = None if any(i is None for i in ids) else len(set(ids)) == len(ids)
    shared_ok = gpu and transport == "ipc" and torch.cuda.device_count() < world  # 1-GPU IPC rehearsal
    if gpu and distinct is False and not shared_ok:
        dup = sorted({str(i) for i in ids if ids.count(i) > 1})
        raise RuntimeError(f"[ERROR] {world} ranks but only {len(set(ids))} distinct GPUs (shared: {dup}); "
                           f"check HIP_VISIBLE_DEVICES / LOCAL_RANK")
    return {"world_size": world, "backend": backend, "distinct_devices": distinct,
            "shared_gpu_rehearsal": bool(shared_ok and distinct is False),
            "ranks": [{k: r[k] for k in ("rank", "host", "device_index", "uuid", "pci_bus_id", "visible")} for r in allr],
            "edges": edges}


def run_decode_benchmark(model: str = "llama2-7b", n_gpus: int = 1, steps: int = 64, warmup: int = 8,
                         batch: int = 16, prompt_len: int = 128, max_seq: int = 0,
                         microbatches: int = 0, seed: int = 0, use_graph: bool = True,
                         verbose: bool = True, weight_dtype: str = "bf16", streams: int = 1,
                         device: str = "cuda", dp: int = 1, latency_steps: int = 0,
                         stage_layers: int = 0, transport: str = "rccl", mid_batch: int = 0) -> Optional[dict]:
    """``microbatches`` 0 = ``streams`` x stages (every GPU holds ``streams`` micro-batches of
    ``batch`` sequences: weak scaling); ``max_seq`` 0 = what the run needs, rounded up to 64.

    ``dp`` > 1: data parallel x pipeline parallel - the ranks form ``dp`` independent pipelines
    of ``n_gpus / dp`` stages each (replica ``rank // pp``, stage ``rank % pp``), each on its own
    prompts; the numbers are whole-job aggregates (tokens of all replicas over the slowest
    rank's time). The pipelines share no communicator, so a replica's ring stays on its own
    xGMI links (adjacent ranks) and a 7B model fits one GPU many times over: dp8 trades the
    pipeline's per-token latency for none of its bubbles.

    ``mid_batch`` > 0: after the batch-1 pass, the same latency pass with ``mid_batch`` sequences
    (<= 128: the fused-GEMV decode regime of a latency-oriented serving batch or a pipeline
    micro-batch) -> ``mid_p50_tpot_ms`` / ``mid_tok_s``.

    ``stage_layers`` > 0: a STAGE PROFILE, not the headline number - the model's architecture
    cut to that many decoder layers (embedding and lm_head kept), e.g. one 10-layer stage of
    Llama-2-70B's 8-stage plan on one GPU with ``microbatches=8`` to hold that stage's KV.

    ``transport`` "ipc": every stage hand-off (decode hidden states, argmax keys, token ids, and
    the prompt prefill's hidden states as slot-sized chunks) goes through IPC-mapped rings in the
    receiver's HBM (parallel/ipc_ring.py: one kernel per send / receive, device flags, no
    communicator); the process group is then gloo (barriers and the final statistics only), so
    N ranks may also share ONE GPU (``LOCAL_RANK % device_count``) - a multi-process rehearsal
    of the exact N-stage pipeline on a 1-GPU box. A timed-out hand-off raises (exit non-zero)."""
    cfg = get_preset(model)
    if stage_layers:
        import dataclasses
        cfg = dataclasses.replace(cfg, num_hidden_layers=stage_layers)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if n_gpus != world:
        raise ValueError(f"n_gpus={n_gpus} but WORLD_SIZE={world}")
    if dp < 1 or world % dp:
        raise ValueError(f"dp={dp} must divide the world size {world}")
    pp = world // dp
    replica, srank = divmod(rank, pp)
    # device "cpu": the same flow on gloo + the torch CPU path (rehearsal of the multi-rank
    # schedule in CPU tests); otherwise one rank per GPU over RCCL
    gpu = device != "cpu"
    if gpu:
        local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    dist = None
    ipc_only = transport == "ipc" and gpu and pp > 1
    if transport not in ("rccl", "ipc"):
        raise ValueError(f"transport {transport!r}: rccl or ipc")
    startup_wd = None
    if world > 1:
        import datetime

        import torch.distributed as dist
        # a stuck peer surfaces as an error after 5 minutes instead of the 10-minute default
        tmo = datetime.timedelta(seconds=int(os.environ.get("LSA_DIST_TIMEOUT_S", "300")))
        if gpu and not ipc_only:
            # the eager RCCL init (device_id) and the preflight's result gather run on the world
            # communicator: bound them too, so a rank that never gets through RCCL's own setup
            # exits legibly with PREFLIGHT_EXIT (the bench supervisor's fallback signal) instead of
            # hanging until the launcher's timeout
            startup_wd = _startup_watchdog(rank)
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group("gloo", timeout=tmo)

    def sync():
        if gpu:
            torch.cuda.synchronize()
    M = microbatches or streams * pp
    need = prompt_len + max(warmup + steps, (LAT_WARMUP + latency_steps) if latency_steps else 0) + 1
    max_seq = max_seq or -(-need // 64) * 64
    S_sets = max(1, min(streams, M))
    plan = plan_stages(cfg, pp, kv_tokens=max_seq * batch * M, head_split=pp > 1,
                       scratch=scratch_bytes(cfg, batch * prompt_len, S_sets, max_seq))
    st = plan.stages[srank]
    # this stage's device bytes as the engine will allocate them (profiles/memory_table.md)
    V = cfg.head_rows
    v1 = (V // 2) // 128 * 128 if pp > 1 else V
    head_rows = (v1 if st.has_head else 0) + (V - v1 if (pp > 1 and st.has_embed) else 0)
    mem_pred = stage_memory(cfg, st.n_layers, slots=batch * M, max_seq=max_seq, prefill_rows=batch * prompt_len,
                            has_embed=st.has_embed, head_rows=head_rows, scratch_sets=S_sets, io_rows=batch * M)
    if need > max_seq:
        raise ValueError(f"prompt+warmup+steps ({need}) exceeds max_seq {max_seq}")
    if verbose and rank == 0:
        print(f"[bench] {cfg.name} {'dp%d x ' % dp if dp > 1 else ''}pp{pp} plan: {plan.summary()}", flush=True)
    rings = [list(range(d * pp, (d + 1) * pp)) for d in range(dp)]
    if ipc_only:
        from .ipc_ring import IpcRingP2P
        edges = [(r[i], r[(i + 1) % pp]) for r in rings for i in range(pp)]
        p2p = IpcRingP2P(rank, slot_bytes=batch * cfg.hidden_size * 2, slots=min(64, max(2, M)),
                         ranks=rings[replica], edges=edges)
    else:
        p2p = DistP2P(ranks=rings[replica], rings=rings)
    preflight = {}
    if dist is not None and not ipc_only and pp > 1:
        # every ring edge carries a message before the weights load: a dead edge ends this rank
        # within LSA_PREFLIGHT_TIMEOUT_S with the edge named (exit PREFLIGHT_EXIT), not after the
        # LSA_DIST_TIMEOUT_S watchdog in the middle of the prefill
        mine = preflight_edges(p2p, srank, pp, dev, inject=transport == "rccl")
        got = [None] * world
        dist.all_gather_object(got, mine)
        for g in got:
            preflight.update(g)
        if verbose and rank == 0:
            print(f"[bench] preflight (us per ring edge): {preflight}", flush=True)
    if startup_wd is not None:
        startup_wd.cancel()
    # which devices the ranks really hold (asserted distinct for RCCL before anything is timed)
    topology = gather_topology(dist, rank, dev, rings, transport if pp > 1 else "local", gpu,
                               p2p if ipc_only else None)
    if verbose and rank == 0 and world > 1:
        print(f"[bench] ranks on devices: {[(r['rank'], r['pci_bus_id'] or r['uuid']) for r in topology['ranks']]} "
              f"edges {topology['edges']}", flush=True)
    t0 = time.perf_counter()
    stage = PipelineStage(cfg, srank, pp, st.start, st.end, dev, batch, M, max_seq,
                          RandomSource(cfg, seed), use_graph=use_graph,
                          max_prefill_rows=batch * prompt_len, weight_dtype=weight_dtype, streams=streams,
                          dtype=torch.bfloat16 if gpu else torch.float32, p2p=p2p)
    if dp > 1:  # trace files are named by rank: use the global one
        stage.tl = tracing.from_env(rank, dev if gpu else "cpu")
    sync()
    load_s = time.perf_counter() - t0
    if dist:
        dist.barrier()

    prompts = None
    if stage.first:
        g = torch.Generator().manual_seed(seed + 1 + replica)
        prompts = torch.randint(3, cfg.vocab_size, (M, batch, prompt_len), generator=g, dtype=torch.int32)
    sync()
    tp0 = time.perf_counter()
    firsts = stage.prefill(prompts, prompt_len)
    sync()
    ttft_ms = (time.perf_counter() - tp0) * 1e3 / M  # per micro-batch prefill through the pipeline
    stage.build_graphs(firsts, history_len=warmup + steps)
    sync()
    if dist:
        dist.barrier()

    for s in range(warmup):
        stage.step(s)
    stage.drain()
    sync()
    if dist:
        dist.barrier()
    sync()
    stage.tl.spans.clear()
    stage.tl.start()  # ranks aligned on the barrier above
    events: list = []
    t_start = time.perf_counter()
    for s in range(steps):
        stage.step(warmup + s, events if stage.last else None)
    stage.drain()
    sync()
    if dist:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t_start

    # per-token latency of each sequence = time between its consecutive tokens (last stage)
    tpot = _tpot_from_events(events) if stage.last else []
    # the first warmup + steps generated ids of micro-batch 0 (for parity checks across layouts)
    tokens_mb0 = None
    if stage.history_stage and stage.graphs[0].history is not None:
        n_tok = warmup + steps
        hist = stage.graphs[0].history.cpu()
        if stage.split:  # row k = generated token k (re-derived at step k)
            tokens_mb0 = hist[:n_tok].T.tolist()
        else:  # row k = token produced at decode step k, after the prefill's first token
            tokens_mb0 = torch.cat([firsts[0].cpu()[None].to(hist.dtype), hist[:n_tok - 1]]).T.tolist() \
                if firsts else None

    # batch-1 latency pass (the reference's only mode, node_worker.py:493-559): ONE sequence
    # through the same pipeline and weights, a 1-row decode graph per stage
    lat_p50 = lat_el = 0.0
    if latency_steps > 0:
        lat_p50, lat_el = _latency_pass(cfg, stage, srank, pp, st, dev, max_seq, prompts, prompt_len,
                                        latency_steps, dist, sync, p2p)
    mid_p50 = mid_el = 0.0
    mid_batch = mid_batch if 0 < mid_batch <= min(batch, 128) else 0
    if mid_batch and latency_steps > 0:
        mid_p50, mid_el = _latency_pass(cfg, stage, srank, pp, st, dev, max_seq, prompts, prompt_len,
                                        latency_steps, dist, sync, p2p, rows=mid_batch)
    mem_peak = float(torch.cuda.max_memory_allocated(dev)) if gpu else 0.0
    chk = getattr(p2p, "check", None)
    if chk is not None:
        chk()  # a timed-out IPC hand-off ends the run with an error, never with poisoned tokens
    stats = torch.tensor([elapsed, ttft_ms, _percentile(tpot, 0.5) if tpot else 0.0,
                          _percentile(tpot, 0.9) if tpot else 0.0, load_s, lat_el, lat_p50,
                          mem_pred["total"], mem_peak, mid_el, mid_p50], dtype=torch.float64,
                         device="cpu" if ipc_only else dev)  # gloo gathers host tensors
    if not gpu and stage.last:  # no device events on CPU: wall-clock step time stands in for TPOT
        stats[2] = stats[3] = elapsed * 1e3 / steps
    if dist:
        gathered = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(gathered, stats)
        allst = torch.stack(gathered).cpu()
        elapsed = float(allst[:, 0].max())
        ttft_ms = float(allst[0, 1])
        p50, p90 = float(allst[pp - 1, 2]), float(allst[pp - 1, 3])  # replica 0's last stage
        load_s = float(allst[:, 4].max())
        lat_el, lat_p50 = float(allst[:, 5].max()), float(allst[pp - 1, 6])
        mem_pred_max, mem_peak_max = float(allst[:, 7].max()), float(allst[:, 8].max())
        mid_el, mid_p50 = float(allst[:, 9].max()), float(allst[pp - 1, 10])
    else:
        mem_pred_max, mem_peak_max = float(stats[7]), float(stats[8])
        p50, p90 = float(stats[2]), float(stats[3])
        lat_el, lat_p50 = float(stats[5]), float(stats[6])
        mid_el, mid_p50 = float(stats[9]), float(stats[10])
    if latency_steps > 0 and not gpu:
        lat_p50 = lat_el * 1e3 / latency_steps
        mid_p50 = mid_el * 1e3 / latency_steps if mid_batch else 0.0
    tokens = dp * steps * M * batch
    res = {
        "tok_s": tokens / elapsed,
        "ms_per_step": elapsed * 1e3 / steps,
        "p50_tpot_ms": p50,
        "p90_tpot_ms": p90,
        "ttft_ms": ttft_ms,
        "global_batch": dp * M * batch,
        "microbatches": M,
        "dp": dp,
        "pp": pp,
        "streams": stage.S,
        "max_seq": max_seq,
        "model_name": ("Llama-2-7B" if model == "llama2-7b" else cfg.name)
        + (f" stage profile ({stage_layers} layers)" if stage_layers else ""),
        "load_s": load_s,
        "plan": plan.ranges(),
        "tokens_mb0": tokens_mb0,  # rank 0 only when it holds the history (1 stage or split head)
        "transport": transport if pp > 1 else None,
        "preflight_us": preflight or None,
        "topology": topology,
        "b1_p50_tpot_ms": lat_p50 if latency_steps > 0 else None,
        "b1_tok_s": (dp * latency_steps / lat_el) if latency_steps > 0 and lat_el > 0 else None,
        "mid_batch": mid_batch or None,
        "mid_p50_tpot_ms": mid_p50 if mid_batch and latency_steps > 0 else None,
        "mid_tok_s": (dp * mid_batch * latency_steps / mid_el) if mid_batch and latency_steps > 0 and mid_el > 0
        else None,
        # max over ranks: the memory model's stage bytes and torch's measured peak allocation
        "mem_pred_gb": round(mem_pred_max / 1e9, 2),
        "mem_peak_gb": round(mem_peak_max / 1e9, 2) if gpu else None,
    }
    trace = tracing.export_env(stage.tl)
    if trace and verbose:
        print(f"[bench] rank {rank} timeline -> {trace}  {stage.tl.summary()}", flush=True)
    if stage.history_stage and verbose:
        hist = stage.graphs[0].history[:8, :4].cpu().tolist() if stage.graphs[0].history is not None else []
        print(f"[bench] rank {rank} sample tokens (step x seq): {hist}", flush=True)
    if ipc_only:
        p2p.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if rank != 0:
        return None
    if verbose:
        print(f"[bench] load {load_s:.1f}s  ttft/mb {ttft_ms:.1f}ms  step {res['ms_per_step']:.3f}ms  "
              f"p50 tpot {p50:.3f}ms  {res['tok_s']:.1f} tok/s", flush=True)
    return res
