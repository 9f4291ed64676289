"""Communicator: the stage-to-stage data plane (reference C1, ``utils/node_worker.py:13-67``).

Same constructor and methods as the reference - ``Communicator(src_addr, dst_addr)``,
``transfer_data(data, data_path=..., keep_data=False)``,
``receive_data(no_block=False, data_path=..., keep_data=False)``, ``change_src_addr``,
``change_dst_addr`` - on MI355X-native plumbing:

* ``backend="tcp"`` (default): the native C++ framed transport (PUSH/PULL semantics) with
  in-memory protocol encoding (no disk staging, no pickles). ``data_path``/``keep_data`` are
  honoured only as an optional debug dump of the encoded bytes.
* ``backend="local"``: in-process mailboxes keyed by address (several NodeWorkers in one
  process, like the reference's 4-stage loopback harness ``node_profiler.py:1174-1236``,
  without sockets).
* ``backend="rccl"``: the message envelope still travels over the TCP transport, but every
  tensor in it is replaced by a (shape, dtype) placeholder and its bytes go device-to-device
  with ``torch.distributed`` send/recv to the neighbouring rank - RCCL over xGMI on MI355X
  (gloo on CPU). Ranks default to the ring of a torchrun job in stage order (receive from
  rank-1, send to rank+1); ``rccl_ranks=(src_rank, dst_rank)`` overrides, and
  :meth:`Communicator.change_ranks` re-points a live communicator (hot re-configuration).
  Each DIRECTED edge has its own process group (own RCCL communicator and stream), created
  collectively once per job by :func:`init_edge_groups`: a send queued ahead of a receive on
  one shared communicator can wait forever for a peer whose stream holds the mirror image
  (the cycle :class:`..pipeline.DistP2P` documents), and with several messages in flight both
  ring directions are busy at once. Receives give up after ``recv_timeout_s`` with an error.

``receive_data(no_block=True)`` raises :class:`Again` when nothing is queued, like
``zmq.Again``; ``timeout_ms`` adds a bounded blocking wait (the reference only offers busy
polling).
"""
from __future__ import annotations

import os
import queue
import threading
from typing import Optional

from . import protocol
from .transport import Again, PullSocket, PushSocket, parse_addr

_LOCAL_LOCK = threading.Lock()
_LOCAL_BOXES: dict = {}


def _local_key(addr: str) -> str:
    host, port = parse_addr(addr)
    return str(port)  # "*" / ip / 127.0.0.1 all name the same in-process endpoint


def _local_box(addr: str) -> "queue.Queue":
    with _LOCAL_LOCK:
        return _LOCAL_BOXES.setdefault(_local_key(addr), queue.Queue())


def reset_local_transport() -> None:
    with _LOCAL_LOCK:
        _LOCAL_BOXES.clear()


_TENSOR_KEY = "__rccl_tensor__"
_EDGE_GROUPS: dict = {}


def init_edge_groups(ranks=None) -> dict:
    """Create one process group per ORDERED pair (a, b), a != b, of ``ranks`` (default: every
    rank of the job). Collective: every rank of the default group must call it, in the same
    order, before rccl-backend Communicators are built (start_node.py does right after
    ``init_process_group``). Groups are cheap until first used (RCCL communicators are created
    lazily), so all pairs are registered and any later ring - a re-plan, a failover over the
    survivors - finds its edges."""
    import torch.distributed as dist
    n = dist.get_world_size()
    ranks = list(range(n)) if ranks is None else list(ranks)
    for a in ranks:
        for b in ranks:
            if a != b and (a, b) not in _EDGE_GROUPS:
                _EDGE_GROUPS[(a, b)] = dist.new_group([a, b])
    return _EDGE_GROUPS


def edge_group(src: int, dst: int):
    g = _EDGE_GROUPS.get((src, dst))
    if g is None:
        raise RuntimeError(f"rccl backend: no process group for edge {src} -> {dst}; call "
                           "communicator.init_edge_groups() on every rank after init_process_group")
    return g


def _extract_tensors(obj, out: list):
    """Replace every tensor in a (nested) message by a placeholder; collect the tensors."""
    import torch
    if isinstance(obj, torch.Tensor):
        out.append(obj)
        return {_TENSOR_KEY: len(out) - 1, "shape": list(obj.shape), "dtype": str(obj.dtype).split(".")[-1]}
    if isinstance(obj, dict):
        return {k: _extract_tensors(v, out) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        r = [_extract_tensors(v, out) for v in obj]
        return r if isinstance(obj, list) else tuple(r)
    return obj


def _restore_tensors(obj, fetch):
    if isinstance(obj, dict):
        if _TENSOR_KEY in obj:
            return fetch(obj)
        return {k: _restore_tensors(v, fetch) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_restore_tensors(v, fetch) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_restore_tensors(v, fetch) for v in obj)
    return obj


class Communicator:
    def __init__(self, src_addr: str, dst_addr: str, backend: str = "tcp", device=None,
                 rccl_ranks: Optional[tuple] = None, recv_timeout_s: float = 300.0):
        self.backend = backend
        self.recv_timeout_s = recv_timeout_s
        self.src_addr = src_addr
        self.dst_addr = dst_addr
        self.sent_messages = 0
        self.received_messages = 0
        self._fault_drop = 0
        self.device = device
        self._pending_sends: list = []
        # set once an rccl tensor receive timed out: its irecv stays posted on the edge group (it
        # cannot be cancelled), so a late message would land one receive off - every later
        # send / receive raises instead of silently returning misaligned data
        self.failed: Optional[str] = None
        self._orphans: list = []  # (work, tensor) of timed-out receives: keep the target alive
        if backend == "rccl":
            import torch.distributed as dist
            if not dist.is_initialized():
                raise RuntimeError("rccl backend: torch.distributed is not initialised (launch with torchrun)")
            r, w = dist.get_rank(), dist.get_world_size()
            self.change_ranks(*(rccl_ranks if rccl_ranks is not None else ((r - 1) % w, (r + 1) % w)))
        if backend in ("tcp", "rccl"):
            self.recv_socket = PullSocket(src_addr)
            self.actual_src_addr = self.recv_socket.last_endpoint
            self.send_socket = PushSocket(dst_addr)
        elif backend == "local":
            self.recv_socket = _local_box(src_addr)
            self.actual_src_addr = src_addr
            self.send_socket = None
        else:
            raise ValueError(f"unknown communicator backend {backend!r}")

    # -- address changes (live re-configuration, reference :31-42) -----------------------
    def change_src_addr(self, new_src_addr: str) -> str:
        if self.backend in ("tcp", "rccl"):
            if new_src_addr != self.src_addr:
                self.recv_socket.close()
                self.recv_socket = PullSocket(new_src_addr)
                self.actual_src_addr = self.recv_socket.last_endpoint
        else:
            self.recv_socket = _local_box(new_src_addr)
            self.actual_src_addr = new_src_addr
        self.src_addr = new_src_addr
        return self.src_addr

    def change_ranks(self, src_rank: int, dst_rank: int) -> None:
        """Point the tensor side channel at new neighbours (rccl backend); the directed-edge
        groups come from :func:`init_edge_groups`."""
        import torch.distributed as dist
        me = dist.get_rank()
        self.src_rank, self.dst_rank = int(src_rank), int(dst_rank)
        self._send_group = edge_group(me, self.dst_rank) if self.dst_rank != me else None
        self._recv_group = edge_group(self.src_rank, me) if self.src_rank != me else None

    def change_dst_addr(self, new_dst_addr: str) -> str:
        if self.backend in ("tcp", "rccl") and new_dst_addr != self.dst_addr:
            self.send_socket.close()
            self.send_socket = PushSocket(new_dst_addr)
        self.dst_addr = new_dst_addr
        return self.dst_addr

    # -- data --------------------------------------------------------------------------
    def _check_failed(self) -> None:
        if self.failed:
            raise RuntimeError(f"communicator unusable after an earlier failure: {self.failed}")

    def transfer_data(self, data, data_path: str = "results/send_data.pt", keep_data: bool = False):
        self._check_failed()
        tensors: list = []
        if self.backend == "rccl":
            data = _extract_tensors(data, tensors)
        payload = protocol.encode(data)
        if self.backend in ("tcp", "rccl"):
            self.send_socket.send_bytes(payload)
            if tensors:
                self._send_tensors(tensors)
        else:
            _local_box(self.dst_addr).put(payload)
        self.sent_messages += 1
        if keep_data:
            os.makedirs(os.path.dirname(data_path) or ".", exist_ok=True)
            with open(data_path, "wb") as f:
                f.write(payload)
            return data_path
        return None

    def receive_data(self, no_block: bool = False, data_path: str = "results/recv_data.pt",
                     keep_data: bool = False, timeout_ms: Optional[int] = None):
        self._check_failed()
        tmo = 0 if no_block else (-1 if timeout_ms is None else int(timeout_ms))
        if self.backend in ("tcp", "rccl"):
            payload = self.recv_socket.recv_bytes(tmo)
        else:
            try:
                payload = self.recv_socket.get(block=tmo != 0, timeout=None if tmo < 0 else tmo / 1000)
            except queue.Empty:
                raise Again()
        self.received_messages += 1
        if keep_data:
            os.makedirs(os.path.dirname(data_path) or ".", exist_ok=True)
            with open(data_path, "wb") as f:
                f.write(payload)
        msg = protocol.decode(payload)
        if self.backend == "rccl":
            msg = _restore_tensors(msg, self._recv_tensor)
        return msg

    # -- rccl tensor side channel --------------------------------------------------------
    def _send_tensors(self, tensors: list) -> None:
        import torch.distributed as dist
        for t in tensors:
            t = t.contiguous()
            if self.device is not None and t.device != self.device and str(self.device) != "cpu":
                t = t.to(self.device)
            self._pending_sends.append((dist.isend(t, self.dst_rank, group=self._send_group), t))
        # bound the outstanding sends (their tensors must stay alive until complete)
        while len(self._pending_sends) > 16:
            w, _ = self._pending_sends.pop(0)
            w.wait()

    def _recv_tensor(self, ph: dict):
        import torch
        import torch.distributed as dist
        dev = self.device if self.device is not None else "cpu"
        import datetime
        t = torch.empty(ph["shape"], dtype=getattr(torch, ph["dtype"]), device=dev)
        work = dist.irecv(t, self.src_rank, group=self._recv_group)
        try:
            ok = work.wait(timeout=datetime.timedelta(seconds=self.recv_timeout_s))
        except RuntimeError as e:  # backend-specific timeout error
            self._fail(work, t, f"rccl recv from rank {self.src_rank} failed or timed out "
                                f"({self.recv_timeout_s:.0f} s): {e}")
            raise RuntimeError(self.failed) from e
        if ok is False:
            self._fail(work, t, f"rccl recv from rank {self.src_rank} timed out ({self.recv_timeout_s:.0f} s)")
            raise RuntimeError(self.failed)
        return t

    def _fail(self, work, t, why: str) -> None:
        self.failed = why
        self._orphans.append((work, t))

    def flush(self, timeout_ms: int = 5000) -> bool:
        for w, _ in self._pending_sends:
            w.wait()
        self._pending_sends.clear()
        return self.send_socket.flush(timeout_ms) if self.backend in ("tcp", "rccl") else True

    def inject_faults(self, drop_every: int = 0, delay_ms: int = 0) -> None:
        """Test hook: drop every Nth outgoing message / delay each one (tcp backend; rccl:
        delays only - a dropped envelope would leave its tensors unmatched on the side channel
        and desynchronise every later message instead of simulating one lost message)."""
        if self.backend == "rccl" and drop_every > 0:
            raise ValueError("inject_faults: message drops are not supported on the rccl backend")
        if self.backend in ("tcp", "rccl"):
            self.send_socket.inject_faults(drop_every, delay_ms)

    def close(self) -> None:
        if self.backend in ("tcp", "rccl"):
            for w, _ in self._pending_sends:
                w.wait()
            self._pending_sends.clear()
            self.send_socket.close(linger_ms=1000)
            self.recv_socket.close()


__all__ = ["Communicator", "Again", "reset_local_transport", "init_edge_groups", "edge_group"]
