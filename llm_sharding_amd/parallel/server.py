"""Continuous-batching serving over the layer-sharded pipeline (one process per GPU).

The reference serves one request at a time around a ZMQ ring, and in serve mode never even
reads requests (``/root/reference/utils/node_worker.py:493-559``). Here the
stages are the ranks of one ``torch.distributed`` job (RCCL over xGMI on GPUs, gloo on CPU)
and rank 0 - the stage that owns the embedding - is also the ingress and the scheduler:

* ``M`` micro-batches of ``B`` KV-cache slots; each micro-batch has at most ONE command in
  flight, so with ``M >= world`` every stage always has work (the same schedule as
  :mod:`.pipeline`).
* Per visit of a micro-batch, rank 0 first collects the token ids the last stage returned for
  its previous command (ring back-edge), updates the requests (streaming output, EOS /
  ``max_new_tokens``), frees finished slots, then issues the next command:
  ``PREFILL`` (admit waiting requests into free slots; long prompts are prefilled in chunks
  under a token budget, only the final chunk emits the first token) or ``DECODE`` (one step of
  every slot of the micro-batch: the captured hipGraph of :class:`DecodeGraph` on GPUs,
  positions on the device, eager active rows on CPU).
* Commands are small int32 headers sent by rank 0 to every rank over a separate gloo (CPU)
  group, so no stage ever blocks its GPU to learn what to do next; activations go rank r ->
  r+1 and token ids last -> 0 over the data group (RCCL).

A slot whose request finished is re-armed (device position reset) with the next command of
its micro-batch; a free slot still rides along in graph replays (its outputs are ignored),
which keeps the graph static.

Live re-sharding (the reference's hot re-configuration, ``/root/reference/utils/node_worker.py
:445-474``, on the deployed pipeline): :meth:`request_replan` (rank 0; the master's ``replan``
command arrives through the ingress) stops admitting requests, lets every request in flight
finish on the current layer split, then broadcasts ``REPLAN`` with the new stage boundaries in
the same ordered command stream; every rank drains its sends, frees its engine, loads its new
``[start, end)`` range, rebuilds KV cache and decode graphs, and rank 0 resumes admission. The
ring edges (and their communicators) are unchanged - only the layer ranges move.
"""
from __future__ import annotations

import contextlib
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch

from ..runtime.engine import DecodeGraph, StageEngine
from ..utils import tracing
from .pipeline import DistP2P, _percentile

CMD_DECODE, CMD_PREFILL, CMD_STOP, CMD_REPLAN = 1, 2, 3, 4
WAITING, PREFILLING, DECODING, DONE = "waiting", "prefilling", "decoding", "done"


@dataclass
class Request:
    rid: int
    input_ids: List[int]
    max_new_tokens: int
    eos_ids: tuple
    on_token: Optional[Callable] = None
    reply_to: Optional[str] = None
    state: str = WAITING
    slot: int = -1
    prefilled: int = 0
    output_ids: List[int] = field(default_factory=list)
    t_submit: float = 0.0
    t_first: float = 0.0
    t_done: float = 0.0

    @property
    def ttft_ms(self) -> float:
        return (self.t_first - self.t_submit) * 1e3

    @property
    def tpot_ms(self) -> float:
        n = len(self.output_ids)
        return (self.t_done - self.t_first) * 1e3 / (n - 1) if n > 1 else 0.0


class _Header:
    """int32 command header: [cmd, mb, n_items, n_resets, items (slot, p0, n, emit)..., resets...];
    REPLAN: [cmd, 0, world + 1, 0, stage boundaries...]."""

    def __init__(self, batch: int, world: int = 1):
        self.size = 4 + max(4 * batch + batch, world + 1)

    def pack(self, cmd, mb, items=(), resets=()) -> torch.Tensor:
        t = torch.zeros(self.size, dtype=torch.int32)
        t[0], t[1], t[2], t[3] = cmd, mb, len(items), len(resets)
        o = 4
        for it in items:
            t[o:o + 4] = torch.tensor(it, dtype=torch.int32)
            o += 4
        for s in resets:
            t[o] = s
            o += 1
        return t

    @staticmethod
    def unpack(t: torch.Tensor):
        v = t.tolist()
        cmd, mb, ni, nr = v[:4]
        items = [tuple(v[4 + 4 * i: 8 + 4 * i]) for i in range(ni)]
        resets = v[4 + 4 * ni: 4 + 4 * ni + nr]
        return cmd, mb, items, resets


class PipelineServer:
    """One rank of a continuous-batching pipeline server. Rank 0 additionally owns the
    request queue (:meth:`submit`, :meth:`serve`); the other ranks run :meth:`serve` too and
    follow rank 0's commands until ``STOP``."""

    def __init__(self, cfg, source, rank: int = 0, world: int = 1, start: int = 0, end: Optional[int] = None,
                 device="cpu", batch: int = 8, microbatches: int = 1, max_seq: int = 2048,
                 prefill_budget: int = 2048, use_graph: bool = True, dtype=torch.bfloat16,
                 ctrl_group=None, p2p=None, causal: bool = True, verbose: bool = False, streams: int = 1):
        self.cfg, self.rank, self.world = cfg, rank, world
        end = cfg.num_hidden_layers if end is None else end
        self.first, self.last = rank == 0, rank == world - 1
        self.B, self.M = batch, microbatches
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.graph_mode = use_graph and self.gpu
        self.dtype = torch.bfloat16 if self.gpu else dtype
        self.budget = int(prefill_budget)
        self.verbose = verbose
        self.source, self.causal, self.max_seq = source, causal, max_seq
        self.start, self.end = start, end
        self.eng = self._build_engine(start, end)
        self.p2p = p2p if p2p is not None else DistP2P()
        self.ctrl = ctrl_group
        self.hdr = _Header(batch, world)
        self.graphs: List = []
        # Concurrent micro-batches (one GPU, graph mode): every command of micro-batch mb -
        # prefill, decode replay, result collection - runs on stream mb % S against engine
        # scratch set mb % S (sized for the prefill budget), so up to S micro-batches share the
        # GPU at once (see pipeline.PipelineStage); a micro-batch's own commands stay ordered.
        self.S = max(1, min(streams, microbatches)) if (self.graph_mode and world == 1) else 1
        self.streams = [torch.cuda.Stream(self.device) for _ in range(self.S)] if self.S > 1 else []
        self._build_graphs()
        # rank 0 state
        self.incoming: "queue.Queue[Request]" = queue.Queue()
        self.waiting: List[Request] = []
        self.by_slot: Dict[int, Request] = {}
        self.requests: Dict[int, Request] = {}
        self.finished: List[Request] = []
        self.outstanding: List = [None] * microbatches
        self.pending_resets: List[list] = [[] for _ in range(microbatches)]
        self.cur_tok: Dict[int, int] = {}  # eager mode: next input token per slot
        self._next_id = 0
        self._ctrl_works: list = []
        self._send_works: list = []
        self._lock = threading.Lock()
        self._replan: Optional[list] = None  # rank 0: stage boundaries waiting for a drained pipeline
        self.replans = 0
        self.tokens_generated = 0
        self.t_start = None
        self.tl = tracing.from_env(rank, self.device)  # LSA_TRACE=dir -> per-rank Chrome trace

    # ------------------------------------------------------------------ engine (re)build
    def _build_engine(self, start: int, end: int) -> StageEngine:
        return StageEngine(self.cfg, start, end, self.device, self.dtype, has_embed=self.first, has_head=self.last,
                           source=self.source, max_slots=self.B * self.M, max_seq=self.max_seq,
                           max_prefill_rows=max(self.budget, self.B), causal=self.causal)

    def _build_graphs(self) -> None:
        for k in range(1, self.S):
            self.eng.decode_scratch(k, rows=self.eng.max_prefill_rows)
        self.graphs = []
        if self.graph_mode:
            mode = "full" if self.world == 1 else ("first" if self.first else ("last" if self.last else "mid"))
            for mb in range(self.M):
                self.graphs.append(DecodeGraph(self.eng, self.B, mode, slots=self._slots(mb),
                                               scratch=mb % self.S).capture())
        for st in self.streams:  # after weight loading and graph capture on the current stream
            st.wait_stream(torch.cuda.current_stream(self.device))

    def _reshard(self, start: int, end: int) -> None:
        """Every rank, pipeline drained: free this stage's engine, load layers [start, end),
        rebuild the KV cache and the decode graphs (same slots, micro-batches and streams)."""
        self._flush_sends()
        if self.gpu:
            torch.cuda.synchronize(self.device)
        with self.tl.span("replan", start=start, end=end):
            self.graphs = []
            self.eng = None
            if self.gpu:
                torch.cuda.empty_cache()
            self.eng = self._build_engine(start, end)
            self.start, self.end = start, end
            self._build_graphs()
            if self.gpu:
                torch.cuda.synchronize(self.device)
        self.cur_tok.clear()
        self.pending_resets = [[] for _ in range(self.M)]
        self.replans += 1
        if self.verbose:
            print(f"[INFO] rank {self.rank}: re-sharded to layers [{start}, {end})", flush=True)

    def request_replan(self, stages) -> None:
        """Rank 0 (thread-safe): move the layer split to ``stages`` ([[start, end], ...] per rank,
        contiguous from 0 to num_hidden_layers). New requests wait; requests in flight finish
        on the current split first (:meth:`serve` applies it once the pipeline is drained)."""
        if not self.first:
            raise RuntimeError("re-plans are requested on rank 0 (the pipeline's command stream)")
        st = [(int(a), int(b)) for a, b in stages]
        L = self.cfg.num_hidden_layers
        ok = (len(st) == self.world and st[0][0] == 0 and st[-1][1] == L
              and all(a < b for a, b in st) and all(x[1] == y[0] for x, y in zip(st, st[1:])))
        if not ok:
            raise ValueError(f"replan: {st} is not a contiguous split of {L} layers over {self.world} stages")
        with self._lock:
            self._replan = [a for a, _ in st] + [L]

    def _apply_replan(self) -> None:
        with self._lock:
            bounds, self._replan = self._replan, None
        t = torch.zeros(self.hdr.size, dtype=torch.int32)
        t[0], t[2] = CMD_REPLAN, len(bounds)
        t[4:4 + len(bounds)] = torch.tensor(bounds, dtype=torch.int32)
        self._bcast_header(t)
        self._reshard(bounds[0], bounds[1])

    # ------------------------------------------------------------------ helpers
    def _mb_ctx(self, mb: int):
        """Stream + engine scratch set of micro-batch ``mb`` (no-op with one stream)."""
        if self.S == 1:
            return contextlib.nullcontext()
        es = contextlib.ExitStack()
        es.enter_context(torch.cuda.stream(self.streams[mb % self.S]))
        es.enter_context(self.eng.use_scratch(mb % self.S))
        return es

    def _slots(self, mb: int) -> list:
        return list(range(mb * self.B, (mb + 1) * self.B))

    def _set_pos(self, slot: int, p: int) -> None:
        self.eng.seq_len[slot] = p
        if self.graph_mode:
            mb, i = divmod(slot, self.B)
            self.graphs[mb].pos[i] = p

    def _to_host(self, t: torch.Tensor):
        """Token ids -> host without serialising the host behind later GPU work: a pinned
        non-blocking copy enqueued right behind the producing kernels, plus an event."""
        if not self.gpu:
            return t.tolist()
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        h.copy_(t, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return (h, ev)

    @staticmethod
    def _host_list(local):
        if isinstance(local, tuple):
            h, ev = local
            ev.synchronize()
            return h.tolist()
        return local

    def _send(self, t, dst):
        self._send_works.append((self.p2p.isend(t, dst), t))
        if len(self._send_works) > 4 * self.M:
            w, _ = self._send_works.pop(0)
            w.wait()

    def _flush_sends(self):
        for w, _ in self._send_works:
            w.wait()
        self._send_works.clear()

    def _bcast_header(self, hdr: torch.Tensor) -> None:
        if self.world == 1:
            return
        import torch.distributed as dist
        for r in range(1, self.world):
            self._ctrl_works.append((dist.isend(hdr, r, group=self.ctrl), hdr))
        while len(self._ctrl_works) > 8 * self.world:
            w, _ = self._ctrl_works.pop(0)
            w.wait()

    # ------------------------------------------------------------------ command execution (every rank)
    def _exec(self, cmd, mb, items, resets, ids=None):
        """Run one command on this stage. Returns the last stage's token ids (world == 1)."""
        name = {CMD_PREFILL: "prefill", CMD_DECODE: "decode"}.get(cmd, "cmd")
        with self.tl.span(name, mb=mb, items=len(items)), self._mb_ctx(mb):
            return self._exec_body(cmd, mb, items, resets, ids)

    def _exec_body(self, cmd, mb, items, resets, ids=None):
        eng, H = self.eng, self.cfg.hidden_size
        for s in resets:
            self._set_pos(s, 0)
        if cmd == CMD_PREFILL:
            slot, pos, emit_rows = [], [], []
            for (s, p0, n, emit) in items:
                eng.seq_len[s] = p0
                slot += [s] * n
                pos += list(range(p0, p0 + n))
                if emit:
                    emit_rows.append(len(pos) - 1)
            rows = len(slot)
            if self.first:
                h = eng.embed(torch.tensor(ids, dtype=torch.int64))
            else:
                h = torch.empty((rows, H), dtype=self.dtype, device=self.device)
                self.p2p.recv(h, self.rank - 1)
            h = eng.forward(h, slot, pos)
            for (s, p0, n, emit) in items:
                self._set_pos(s, p0 + n)
            if self.last:
                if not emit_rows:
                    return []
                tok = eng.head(h, emit_rows).to(torch.int32)
                if self.world == 1:
                    return self._to_host(tok)
                self._send(tok.contiguous(), 0)
            else:
                self._send(h.contiguous(), self.rank + 1)
            return None
        if cmd == CMD_DECODE:
            if self.graph_mode:
                g = self.graphs[mb]
                if not self.first:
                    self.p2p.recv(g.h_in, self.rank - 1)
                g.replay()
                if self.last:
                    if self.world == 1:
                        return self._to_host(g.tokens)
                    out = g.tokens.clone()
                    self._send(out, 0)
                else:
                    self._send(g.out_hidden.clone(), self.rank + 1)
                return None
            # eager: only the listed rows (slot, p0) run
            slots = [it[0] for it in items]
            n = len(slots)
            if self.first:
                h = eng.embed(torch.tensor(ids, dtype=torch.int64))
            else:
                h = torch.empty((n, H), dtype=self.dtype, device=self.device)
                self.p2p.recv(h, self.rank - 1)
            pos = [it[1] for it in items]
            for s, p in zip(slots, pos):
                eng.seq_len[s] = p
            h = eng.forward(h, slots, pos)
            for s, p in zip(slots, pos):
                eng.seq_len[s] = p + 1
            if self.last:
                tok = eng.head(h).to(torch.int32)
                if self.world == 1:
                    return self._to_host(tok)
                self._send(tok.contiguous(), 0)
            else:
                self._send(h.contiguous(), self.rank + 1)
            return None
        return None

    # ------------------------------------------------------------------ rank 0: requests
    def submit(self, input_ids, max_new_tokens: int = 64, eos_ids=None, on_token=None,
               reply_to: Optional[str] = None) -> int:
        """Queue a request (thread-safe). ``input_ids``: list of token ids."""
        if not self.first:
            raise RuntimeError("requests are submitted on rank 0 (the ingress stage)")
        ids = [int(x) for x in input_ids]
        if not ids:
            raise ValueError("empty prompt")
        if len(ids) + max_new_tokens > self.eng.max_seq:
            raise ValueError(f"prompt ({len(ids)}) + max_new_tokens ({max_new_tokens}) exceeds max_seq "
                             f"{self.eng.max_seq}")
        with self._lock:
            rid = self._next_id
            self._next_id += 1
        eos = tuple(self.cfg.eos_ids if eos_ids is None else eos_ids)
        r = Request(rid, ids, int(max_new_tokens), eos, on_token=on_token, reply_to=reply_to,
                    t_submit=time.perf_counter())
        self.incoming.put(r)
        return rid

    def unfinished(self) -> List[Request]:
        """Rank 0, after :meth:`serve` has returned: every request that will never finish here
        (queued, waiting or in flight) - the controller answers them with an error when the
        pipeline is dropped (a lost rank), instead of leaving their clients waiting."""
        self._intake()
        return [r for r in self.requests.values() if r.state != DONE]

    def _intake(self) -> None:
        while True:
            try:
                r = self.incoming.get_nowait()
            except queue.Empty:
                break
            self.requests[r.rid] = r
            self.waiting.append(r)

    def _free_slots(self, mb: int) -> list:
        return [s for s in self._slots(mb) if s not in self.by_slot]

    def _emit(self, r: Request, tok: int, now: float) -> None:
        if not r.output_ids:
            r.t_first = now
        r.output_ids.append(tok)
        self.tokens_generated += 1
        if r.on_token is not None:
            r.on_token(r, tok)
        if tok in r.eos_ids or len(r.output_ids) >= r.max_new_tokens:
            r.state, r.t_done = DONE, now
            mb = r.slot // self.B
            del self.by_slot[r.slot]
            self.cur_tok.pop(r.slot, None)
            self.pending_resets[mb].append(r.slot)
            self.finished.append(r)
        else:
            self.cur_tok[r.slot] = tok

    def _collect(self, mb: int) -> None:
        """Receive/process the return of micro-batch ``mb``'s outstanding command."""
        with self._mb_ctx(mb):
            self._collect_body(mb)

    def _collect_body(self, mb: int) -> None:
        o = self.outstanding[mb]
        if o is None:
            return
        self.outstanding[mb] = None
        kind, info, local = o
        if kind == CMD_PREFILL:
            emitted = [r for r in info if r is not None]
            if not emitted:
                return
            if local is None:
                buf = torch.zeros(len(emitted), dtype=torch.int32, device=self.device)
                self.p2p.recv(buf, self.world - 1)
                toks = buf.tolist()
            else:
                toks = self._host_list(local)
            now = time.perf_counter()
            for r, t in zip(emitted, toks):
                r.state = DECODING
                if self.graph_mode:
                    self.graphs[mb].tokens[r.slot - mb * self.B] = t
                self._emit(r, int(t), now)
        elif kind == CMD_DECODE:
            if local is None:
                if self.graph_mode:
                    g = self.graphs[mb]
                    self.p2p.recv(g.tokens, self.world - 1)  # next step's input ids, in place
                    toks = g.tokens.tolist()
                else:
                    buf = torch.zeros(len(info), dtype=torch.int32, device=self.device)
                    self.p2p.recv(buf, self.world - 1)
                    toks = buf.tolist()
            else:
                toks = self._host_list(local)
            now = time.perf_counter()
            if self.graph_mode:
                for i, s in enumerate(self._slots(mb)):
                    r = self.by_slot.get(s)
                    if r is not None and r.state == DECODING and r.rid in info:
                        self._emit(r, int(toks[i]), now)
            else:
                for (s, rid), t in zip(info, toks):
                    r = self.by_slot.get(s)
                    if r is not None and r.rid == rid:
                        self._emit(r, int(t), now)

    def _schedule(self, mb: int) -> bool:
        """Issue the next command for ``mb``. Returns False if it has nothing to do."""
        resets = self.pending_resets[mb]
        # admission: waiting requests into free slots (held back while a re-plan drains)
        for s in self._free_slots(mb):
            if not self.waiting or self._replan is not None:
                break
            r = self.waiting.pop(0)
            r.slot, r.state, r.prefilled = s, PREFILLING, 0
            self.by_slot[s] = r
            if s in resets:
                resets.remove(s)
        pre = [self.by_slot[s] for s in self._slots(mb) if s in self.by_slot and self.by_slot[s].state == PREFILLING]
        if pre:
            items, ids, info, budget = [], [], [], self.budget
            for r in pre:
                if budget <= 0:
                    break
                n = min(len(r.input_ids) - r.prefilled, budget)
                emit = int(r.prefilled + n == len(r.input_ids))
                items.append((r.slot, r.prefilled, n, emit))
                ids += r.input_ids[r.prefilled:r.prefilled + n]
                info.append(r if emit else None)
                r.prefilled += n
                budget -= n
            self._issue(CMD_PREFILL, mb, items, resets, ids, info)
            return True
        dec = [self.by_slot[s] for s in self._slots(mb) if s in self.by_slot and self.by_slot[s].state == DECODING]
        if dec:
            if self.graph_mode:
                items = [(s, 0, 1, 0) for s in self._slots(mb)]
                info = {r.rid for r in dec}
                ids = None
            else:
                items = [(r.slot, len(r.input_ids) + len(r.output_ids) - 1, 1, 1) for r in dec]
                info = [(r.slot, r.rid) for r in dec]
                ids = [self.cur_tok[r.slot] for r in dec]
            self._issue(CMD_DECODE, mb, items, resets, ids, info)
            return True
        if resets:  # nothing to run, but keep device positions tidy on every rank
            self._issue(CMD_DECODE, mb, [], resets, None, None, run=False)
        return False

    def _issue(self, cmd, mb, items, resets, ids, info, run: bool = True):
        hdr = self.hdr.pack(cmd if run else 0, mb, items, resets)
        self.pending_resets[mb] = []
        self._bcast_header(hdr)
        if not run:
            with self._mb_ctx(mb):
                for s in resets:
                    self._set_pos(s, 0)
            return
        local = self._exec(cmd, mb, items, resets, ids=ids)
        self.outstanding[mb] = (cmd, info, local)

    def _busy(self) -> bool:
        return bool(self.waiting or self.by_slot or any(o is not None for o in self.outstanding)
                    or not self.incoming.empty() or self._replan is not None)

    # ------------------------------------------------------------------ main loops
    def serve(self, stop_when_idle: bool = True, idle_sleep_s: float = 0.0005,
              should_stop: Optional[Callable[[], bool]] = None) -> None:
        """Rank 0: schedule until idle (or ``should_stop()``), then stop every rank.
        Other ranks: execute rank 0's commands until STOP."""
        if not self.first:
            self._follow()
            return
        self.t_start = self.t_start or time.perf_counter()
        while True:
            if self._replan is not None and not self.by_slot and all(o is None for o in self.outstanding):
                self._apply_replan()  # drained: every stage moves to the new split together
            self._intake()
            any_work = False
            for mb in range(self.M):
                self._collect(mb)
                self._intake()
                any_work |= self._schedule(mb)
            if not any_work and not self._busy():
                if stop_when_idle or (should_stop is not None and should_stop()):
                    break
                time.sleep(idle_sleep_s)
        self.stop()

    def stop(self) -> None:
        tracing.export_env(self.tl)
        if self.first:
            self._bcast_header(self.hdr.pack(CMD_STOP, 0))
            for w, _ in self._ctrl_works:
                w.wait()
            self._ctrl_works.clear()
        self._flush_sends()
        if self.gpu:
            torch.cuda.synchronize(self.device)

    def _follow(self) -> None:
        import torch.distributed as dist
        hdr = torch.zeros(self.hdr.size, dtype=torch.int32)
        while True:
            dist.recv(hdr, 0, group=self.ctrl)
            if int(hdr[0]) == CMD_REPLAN:
                b = hdr[4:4 + int(hdr[2])].tolist()
                self._reshard(b[self.rank], b[self.rank + 1])
                continue
            cmd, mb, items, resets = _Header.unpack(hdr)
            if cmd == CMD_STOP:
                break
            if cmd == 0:
                for s in resets:
                    self._set_pos(s, 0)
                continue
            self._exec(cmd, mb, items, resets)
        self._flush_sends()
        if self.gpu:
            torch.cuda.synchronize(self.device)
        tracing.export_env(self.tl)

    # ------------------------------------------------------------------ convenience
    def generate(self, prompts: List[List[int]], max_new_tokens: int = 32, eos_ids=()) -> List[List[int]]:
        """Rank 0: submit ``prompts``, serve until all are done, return their outputs in order.
        (Other ranks must call :meth:`serve` concurrently.)"""
        rids = [self.submit(p, max_new_tokens, eos_ids=eos_ids) for p in prompts]
        self.serve(stop_when_idle=True)
        return [self.requests[r].output_ids for r in rids]

    def stats(self) -> dict:
        done = [r for r in self.finished]
        el = time.perf_counter() - (self.t_start or time.perf_counter())
        return {
            "requests": len(done),
            "tokens": self.tokens_generated,
            "elapsed_s": el,
            "tok_s": self.tokens_generated / el if el > 0 else 0.0,
            "ttft_ms_p50": _percentile([r.ttft_ms for r in done], 0.5),
            "tpot_ms_p50": _percentile([r.tpot_ms for r in done if len(r.output_ids) > 1], 0.5),
            "tpot_ms_p90": _percentile([r.tpot_ms for r in done if len(r.output_ids) > 1], 0.9),
        }


__all__ = ["PipelineServer", "Request"]
