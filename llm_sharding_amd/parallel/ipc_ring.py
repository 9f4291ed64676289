"""Stage-to-stage hand-off through IPC-mapped rings in HBM (csrc/kernels/ipc_ring.hip).

The p2p transport the pipeline plugs in beside :class:`~.pipeline.DistP2P` (RCCL) and
:class:`~.pipeline.LocalP2P`: ``isend(t, dst)`` / ``recv(t, src)`` with the same stream
semantics, but each is ONE kernel on the caller's stream that moves the bytes over xGMI into a
ring slot in the receiver's HBM and signals with device flags - no communicator, no proxy
thread, nothing host-side per message. Every index the kernels use lives in device memory, so a
send / receive can be captured inside a hipGraph with the decode step it feeds (SURVEY.md §5.8,
the graph-captured IPC hand-off; the reference's hop is ZMQ + torch.save through a file:
/root/reference/utils/node_worker.py:44-67).

Per directed edge ``src -> dst`` (default: the pipeline ring r -> r+1 plus the back-edge):
  * dst allocates the inbox (R flag words + R slots of ``slot_bytes``), src the ack box (R words);
  * handles go through one ``all_gather_object`` on a gloo group (a control-plane exchange at
    construction only); each side maps the other's buffer with ``hipIpcOpenMemHandle``.
A message must be a multiple of 4 bytes; one larger than ``slot_bytes`` (a prompt prefill's
hidden states) is carried as consecutive slot-sized chunks, so every message of a run - decode
and prefill - can go through the rings with no communicator at all. Up to R messages per edge
are in flight; a sender that runs R ahead waits in-kernel for the receiver's ack. Every spin is
bounded (``timeout_s``, env ``LSA_IPC_TIMEOUT_S``, per R slots of a message: a chunked prefill
message of C chunks allows ceil(C / R) x timeout_s, since its sender waits for the receiver to drain
the ring, and the receiver may start only after its own stage's compute): a launch that gives up sets a sticky error
word, poisons its receive buffer (0xFF bytes) instead of returning stale data, and every later
launch of the endpoint is poisoned too; :meth:`check` raises once that happened.
An edge whose two ends are the same rank (loopback) works without IPC mapping.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from ..ops import hip

_FLAG_BYTES = 256


def _lib():
    L = hip.lib()
    if not getattr(L, "_ipc_typed", False):
        vp, ll, i = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int
        L.lsa_ipc_alloc.argtypes = [ll, ctypes.POINTER(vp), vp, ctypes.POINTER(i), i]
        L.lsa_ipc_handle_bytes.argtypes = []
        L.lsa_ipc_open.argtypes = [vp, ctypes.POINTER(vp)]
        L.lsa_ipc_close.argtypes = [vp]
        L.lsa_ipc_free.argtypes = [vp]
        L.lsa_ipc_send.argtypes = [vp, ll, vp, ll, vp, vp, i, vp, vp, ll, i, vp]
        L.lsa_ipc_recv.argtypes = [vp, ll, vp, ll, vp, vp, i, vp, vp, ll, i, vp]
        L._ipc_typed = True
    return L


def _device_uuid(dev: torch.device) -> str:
    """Identity of the physical GPU (two processes may share one: the 1-GPU test harness)."""
    try:
        return str(torch.cuda.get_device_properties(dev).uuid)
    except Exception:  # noqa: BLE001 - older torch: fall back to the PCI bus id
        return str(getattr(torch.cuda.get_device_properties(dev), "pci_bus_id", dev.index))


def _ok(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (status {rc})")


class _Work:
    """Send handle: ``wait()`` orders the caller's current stream after the send kernel (the
    source buffer may be rewritten from then on) - RCCL's Work semantics."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        if self.ev is not None:
            torch.cuda.current_stream().wait_event(self.ev)


class IpcRingP2P:
    """``rank``: this process's global rank; ``edges``: directed (src, dst) global-rank pairs
    (default: the ring over ``ranks``); ``ranks``: stage index -> global rank (as DistP2P);
    ``slot_bytes``: largest message; ``slots``: ring depth R per edge. Collective: every rank of
    ``group`` (a gloo group; default: a new one over the world) constructs it at the same point."""

    graph_capturable = True  # sends / receives may be captured in a hipGraph (device-side indices)

    def __init__(self, rank: int, slot_bytes: int, slots: int = 4, ranks: Optional[list] = None,
                 edges: Optional[list] = None, group=None, timeout_s: Optional[float] = None, grid: int = 32):
        import os

        import torch.distributed as dist
        self.rank, self.R, self.grid = rank, int(slots), int(grid)
        hip._req(1 <= self.R <= _FLAG_BYTES // 4, f"ipc ring: 1..{_FLAG_BYTES // 4} slots")
        self.slot_bytes = -(-int(slot_bytes) // 256) * 256
        if timeout_s is None:
            timeout_s = float(os.environ.get("LSA_IPC_TIMEOUT_S", "30"))
        self.timeout_us = int(timeout_s * 1e6)
        self.ranks = ranks
        world = dist.get_world_size() if dist.is_initialized() else 1
        if edges is None:
            ring = ranks if ranks is not None else list(range(world))
            edges = [(ring[i], ring[(i + 1) % len(ring)]) for i in range(len(ring))] if len(ring) > 1 else []
        self.edges = [tuple(e) for e in edges]
        self.dev = torch.device("cuda", torch.cuda.current_device())
        L = _lib()
        hb = L.lsa_ipc_handle_bytes()
        self._own, self._opened = [], []
        mine = {}  # (edge, "inbox" | "acks") -> handle bytes
        self.inbox, self.ackbox = {}, {}
        # what each peer-written buffer was allocated as (csrc/kernels/ipc_ring.hip lsa_ipc_alloc:
        # 2 uncached, 1 fine-grained, 0 coarse-grained); a peer GPU's writes into a coarse-grained
        # buffer are guaranteed visible only at kernel boundaries, so an edge between two
        # different GPUs refuses it (below, once the peers' devices are known)
        # (env LSA_IPC_ALLOC=fine / coarse starts from a weaker kind: cost A/B on one GPU only)
        self.alloc_kinds = {}
        first = {"uncached": 0, "fine": 1, "coarse": 2}[os.environ.get("LSA_IPC_ALLOC", "uncached")]

        def alloc(nbytes: int, key):
            ptr, h, kind = ctypes.c_void_p(), ctypes.create_string_buffer(hb), ctypes.c_int(-1)
            _ok(L.lsa_ipc_alloc(nbytes, ctypes.byref(ptr), h, ctypes.byref(kind), first), "lsa_ipc_alloc")
            self._own.append(ptr.value)
            self.alloc_kinds[key] = kind.value
            mine[key] = h.raw
            mine[(key, "dev")] = _device_uuid(self.dev)
            return ptr.value

        for e in self.edges:
            if e[1] == rank:
                self.inbox[e] = alloc(_FLAG_BYTES + self.R * self.slot_bytes, (e, "inbox"))
            if e[0] == rank:
                self.ackbox[e] = alloc(_FLAG_BYTES, (e, "acks"))
        for key, kind in self.alloc_kinds.items():
            mine[("kind", key)] = kind
        if group is None and dist.is_initialized():
            group = dist.new_group(backend="gloo")
        self.group = group
        allh = [None] * world
        if dist.is_initialized():
            dist.all_gather_object(allh, mine, group=group)
        else:
            allh = [mine]
        theirs = {}
        for d in allh:
            theirs.update(d or {})
        self.peer_inbox, self.peer_acks = {}, {}
        for e in self.edges:
            if e[0] == rank == e[1]:  # loopback edge: both buffers are our own
                self.peer_inbox[e], self.peer_acks[e] = self.inbox[e], self.ackbox[e]
                continue
            if e[0] == rank:  # sender: map the receiver's inbox
                self._check_coherent(e, theirs, "inbox")
                self.peer_inbox[e] = self._open(theirs[(e, "inbox")])
            if e[1] == rank:  # receiver: map the sender's ack box
                self._check_coherent(e, theirs, "acks")
                self.peer_acks[e] = self._open(theirs[(e, "acks")])
        # per edge end: {count, ticket, fail}; one error word for every launch of this endpoint. Each edge
        # end issues on its own stream (ordered against the caller's by events), so sends of one
        # edge made from several compute streams still run one at a time, in issue order
        self.state = {e: torch.zeros((2, 4) if e[0] == e[1] else 4, dtype=torch.int32, device=self.dev)
                      for e in self.edges if rank in e}
        self.streams = {e: torch.cuda.Stream(self.dev) for e in self.state}
        for e in self.state:  # a loopback edge's receive must not queue behind its own send
            if e[0] == e[1]:
                self.streams[(e, "recv")] = torch.cuda.Stream(self.dev)
        self.captured_ops = 0  # sends / receives recorded into hipGraphs (diagnostics)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.dev)
        if dist.is_initialized():
            dist.barrier(group=group)  # every mapping is in place before anyone sends

    def _check_coherent(self, e, theirs: dict, what: str) -> None:
        """An edge between two different GPUs needs its peer-written buffers uncached or
        fine-grained on BOTH ends (ours: ``alloc_kinds``; theirs: the kind they published)."""
        other = (e, "acks") if what == "inbox" else (e, "inbox")
        if theirs.get(((e, what), "dev")) == _device_uuid(self.dev):
            return  # both ends on one GPU: one L2, coarse-grained memory is coherent
        kinds = [theirs.get(("kind", (e, what)), 0)]
        if other in self.alloc_kinds:
            kinds.append(self.alloc_kinds[other])
        hip._req(min(kinds) >= 1, f"ipc ring edge {e}: a cross-GPU ring needs uncached / fine-grained buffers, "
                                  f"got allocation kinds {kinds} (0 = coarse-grained)")

    def _open(self, handle: bytes) -> int:
        ptr = ctypes.c_void_p()
        _ok(_lib().lsa_ipc_open(ctypes.create_string_buffer(handle, len(handle)), ctypes.byref(ptr)), "lsa_ipc_open")
        self._opened.append(ptr.value)
        return ptr.value

    def _global(self, stage: int) -> int:
        return self.ranks[stage] if self.ranks is not None else stage

    def _state(self, e, send: bool) -> int:
        st = self.state[e]
        return (st[0] if send else st[1]).data_ptr() if e[0] == e[1] else st.data_ptr()

    @staticmethod
    def _staged(t: torch.Tensor) -> bool:
        """Tensors the kernels cannot address directly (non-contiguous or not 16-B aligned) go
        through a private contiguous copy; routing never depends on it (only on byte counts)."""
        return not (t.is_contiguous() and t.data_ptr() % 16 == 0)

    def _chunks(self, n: int):
        hip._req(n > 0 and n % 4 == 0, "ipc ring: message bytes must be a positive multiple of 4")
        return [(o, min(self.slot_bytes, n - o)) for o in range(0, n, self.slot_bytes)]

    def _timeout_for(self, n_chunks: int) -> int:
        """Spin bound (us) of each launch of a message of ``n_chunks`` slot-sized chunks: one
        timeout per R chunks (a message longer than the ring waits for its receiver to drain it)."""
        return int(self.timeout_us * max(1, -(-n_chunks // self.R)))

    def isend(self, t: torch.Tensor, dst: int):
        e = (self.rank, self._global(dst))
        hip._req(t.is_cuda, "ipc ring: cuda tensor")
        src = t.contiguous().clone() if self._staged(t) else t
        n = src.numel() * src.element_size()
        base = self.peer_inbox[e]
        cur, cs = torch.cuda.current_stream(self.dev), self.streams[e]
        cs.wait_stream(cur)
        L = _lib()
        chunks = self._chunks(n)
        # a message of more chunks than slots needs its receiver running concurrently; the two
        # streams of a loopback edge (one process) may share a hardware queue, so there the
        # receive could sit behind a send that waits for it
        hip._req(e[0] != e[1] or len(chunks) <= self.R,
                 f"ipc ring: a loopback message may span at most {self.R} slots ({len(chunks)} needed)")
        tmo = self._timeout_for(len(chunks))
        for off, nb in chunks:
            _ok(L.lsa_ipc_send(src.data_ptr() + off, nb, base + _FLAG_BYTES, self.slot_bytes, base, self.ackbox[e],
                               self.R, self._state(e, True), self.err.data_ptr(), tmo, self.grid,
                               cs.cuda_stream), "lsa_ipc_send")
        src.record_stream(cs)
        if torch.cuda.is_current_stream_capturing():
            self.captured_ops += 1
            cur.wait_stream(cs)  # a captured send joins the capturing stream before the capture ends
            return _Work(None)
        ev = torch.cuda.Event()
        ev.record(cs)
        return _Work(ev)

    def recv(self, t: torch.Tensor, src: int) -> None:
        e = (self._global(src), self.rank)
        hip._req(t.is_cuda, "ipc ring: cuda tensor")
        dst = torch.empty(t.shape, dtype=t.dtype, device=t.device) if self._staged(t) else t
        n = dst.numel() * dst.element_size()
        base = self.inbox[e]
        cur, cs = torch.cuda.current_stream(self.dev), self.streams.get((e, "recv"), self.streams[e])
        cs.wait_stream(cur)
        L = _lib()
        chunks = self._chunks(n)
        tmo = self._timeout_for(len(chunks))
        for off, nb in chunks:
            _ok(L.lsa_ipc_recv(dst.data_ptr() + off, nb, base + _FLAG_BYTES, self.slot_bytes, base, self.peer_acks[e],
                               self.R, self._state(e, False), self.err.data_ptr(), tmo, self.grid,
                               cs.cuda_stream), "lsa_ipc_recv")
        dst.record_stream(cs)
        self.captured_ops += int(torch.cuda.is_current_stream_capturing())
        cur.wait_stream(cs)
        if dst is not t:
            t.copy_(dst)

    def fits(self, t: torch.Tensor) -> bool:
        """One ring slot, decided by the byte count only (both ends of an edge agree on it)."""
        n = t.numel() * t.element_size()
        return t.is_cuda and n % 4 == 0 and 0 < n <= self.slot_bytes

    def error_code(self) -> int:
        return int(self.err.item())

    def check(self) -> None:
        """Raise if any send (1: no ack) or receive (2: no message) of this endpoint gave up
        waiting - from then on its receives deliver poison (0xFF bytes), never stale data."""
        code = self.error_code()
        if code:
            raise RuntimeError(f"ipc ring: a {'send' if code == 1 else 'receive'} timed out waiting for its peer "
                               f"(rank {self.rank}); the edge is poisoned")

    def close(self) -> None:
        """Unmap the peers' buffers, then (once every rank has unmapped ours) free our own."""
        import torch.distributed as dist
        torch.cuda.synchronize(self.dev)
        L = _lib()
        for p in self._opened:
            L.lsa_ipc_close(p)
        if dist.is_initialized():
            dist.barrier(group=self.group)
        for p in self._own:
            L.lsa_ipc_free(p)
        self._opened, self._own = [], []
