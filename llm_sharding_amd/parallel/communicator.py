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


class Communicator:
    def __init__(self, src_addr: str, dst_addr: str, backend: str = "tcp"):
        self.backend = backend
        self.src_addr = src_addr
        self.dst_addr = dst_addr
        self.sent_messages = 0
        self.received_messages = 0
        self._fault_drop = 0
        if backend == "tcp":
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
        if self.backend == "tcp":
            if new_src_addr != self.src_addr:
                self.recv_socket.close()
                self.recv_socket = PullSocket(new_src_addr)
                self.actual_src_addr = self.recv_socket.last_endpoint
        else:
            self.recv_socket = _local_box(new_src_addr)
            self.actual_src_addr = new_src_addr
        self.src_addr = new_src_addr
        return self.src_addr

    def change_dst_addr(self, new_dst_addr: str) -> str:
        if self.backend == "tcp" and new_dst_addr != self.dst_addr:
            self.send_socket.close()
            self.send_socket = PushSocket(new_dst_addr)
        self.dst_addr = new_dst_addr
        return self.dst_addr

    # -- data --------------------------------------------------------------------------
    def transfer_data(self, data, data_path: str = "results/send_data.pt", keep_data: bool = False):
        payload = protocol.encode(data)
        if self.backend == "tcp":
            self.send_socket.send_bytes(payload)
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
        tmo = 0 if no_block else (-1 if timeout_ms is None else int(timeout_ms))
        if self.backend == "tcp":
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
        return protocol.decode(payload)

    def flush(self, timeout_ms: int = 5000) -> bool:
        return self.send_socket.flush(timeout_ms) if self.backend == "tcp" else True

    def inject_faults(self, drop_every: int = 0, delay_ms: int = 0) -> None:
        """Test hook: drop every Nth outgoing message / delay each one (tcp backend)."""
        if self.backend == "tcp":
            self.send_socket.inject_faults(drop_every, delay_ms)

    def close(self) -> None:
        if self.backend == "tcp":
            self.send_socket.close(linger_ms=1000)
            self.recv_socket.close()


__all__ = ["Communicator", "Again", "reset_local_transport"]
