"""Python binding of the native framed TCP transport (csrc/comm/tcp_transport.cpp).

``PullSocket`` / ``PushSocket`` provide ZeroMQ PUSH/PULL semantics (the reference's
``zmq.PULL.bind`` / ``zmq.PUSH.connect``, ``/root/reference/utils/node_worker.py:14-42``)
without pyzmq: in-memory framing, a blocking ``recv`` with timeout instead of the
reference's busy ``NOBLOCK`` poll, queued sends with lazy (re)connect, and ``flush``.

Addresses use the same ``tcp://host:port`` strings as the reference (``tcp://*:40800`` to
bind all interfaces).
"""
from __future__ import annotations

import ctypes
import os
import socket
from typing import Optional

NATIVE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native")
COMM_SO = os.path.join(NATIVE_DIR, "liblsa_comm.so")

_lib = None


class Again(Exception):
    """No message available (the reference's ``zmq.Again``)."""


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(COMM_SO):
        raise RuntimeError(f"native transport not built: {COMM_SO} missing; run `python csrc/build.py`")
    L = ctypes.CDLL(COMM_SO)
    vp, i, ll = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
    L.lsa_pull_bind.argtypes = [ctypes.c_char_p, i, ctypes.POINTER(i)]
    L.lsa_pull_bind.restype = vp
    L.lsa_pull_wait.argtypes = [vp, i]
    L.lsa_pull_wait.restype = ll
    L.lsa_pull_take.argtypes = [vp, vp, ll]
    L.lsa_pull_take.restype = ll
    L.lsa_pull_port.argtypes = [vp]
    L.lsa_pull_port.restype = i
    L.lsa_pull_received.argtypes = [vp]
    L.lsa_pull_received.restype = ll
    L.lsa_pull_close.argtypes = [vp]
    L.lsa_pull_close.restype = None
    L.lsa_push_connect.argtypes = [ctypes.c_char_p, i]
    L.lsa_push_connect.restype = vp
    L.lsa_push_send.argtypes = [vp, vp, ll]
    L.lsa_push_send.restype = i
    L.lsa_push_flush.argtypes = [vp, i]
    L.lsa_push_flush.restype = i
    L.lsa_push_pending.argtypes = [vp]
    L.lsa_push_pending.restype = ll
    L.lsa_push_connected.argtypes = [vp]
    L.lsa_push_connected.restype = i
    L.lsa_push_fault.argtypes = [vp, i, i]
    L.lsa_push_fault.restype = None
    L.lsa_push_close.argtypes = [vp]
    L.lsa_push_close.restype = None
    _lib = L
    return L


def parse_addr(addr: str) -> tuple:
    """``tcp://host:port`` -> (host, port). ``*`` means all interfaces."""
    if not addr.startswith("tcp://"):
        raise ValueError(f"unsupported address {addr!r} (expected tcp://host:port)")
    hp = addr[len("tcp://"):]
    host, _, port = hp.rpartition(":")
    if not host or not port:
        raise ValueError(f"bad address {addr!r}")
    return host, int(port)


def local_ip() -> str:
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        try:
            s.connect(("10.255.255.255", 1))
            return s.getsockname()[0]
        finally:
            s.close()
    except OSError:
        return "127.0.0.1"


class PullSocket:
    def __init__(self, addr: str):
        host, port = parse_addr(addr)
        out = ctypes.c_int(0)
        self._h = lib().lsa_pull_bind(host.encode(), port, ctypes.byref(out))
        if not self._h:
            raise OSError(f"cannot bind {addr} (address in use?)")
        self.port = out.value
        self.addr = addr
        bind_host = "0.0.0.0" if host in ("*", "0.0.0.0") else host
        # resolved endpoint, like zmq.LAST_ENDPOINT (reference node_worker.py:24)
        self.last_endpoint = f"tcp://{bind_host}:{self.port}"

    def recv_bytes(self, timeout_ms: int = -1) -> bytes:
        if self._h is None:
            raise OSError("socket closed")
        n = lib().lsa_pull_wait(self._h, int(timeout_ms))
        if n == -1:
            raise Again()
        if n < 0:
            raise OSError("socket closed")
        buf = ctypes.create_string_buffer(max(1, n))
        got = lib().lsa_pull_take(self._h, buf, n)
        if got != n:
            raise OSError("transport race: message vanished")
        return buf.raw[:n]

    @property
    def received(self) -> int:
        return int(lib().lsa_pull_received(self._h))

    def close(self) -> None:
        if self._h:
            lib().lsa_pull_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PushSocket:
    def __init__(self, addr: str):
        host, port = parse_addr(addr)
        if host in ("*", "0.0.0.0"):
            host = "127.0.0.1"
        self.addr = addr
        self._h = lib().lsa_push_connect(host.encode(), port)

    def send_bytes(self, data: bytes) -> None:
        rc = lib().lsa_push_send(self._h, data, len(data))
        if rc != 0:
            raise OSError("send on closed socket")

    def flush(self, timeout_ms: int = -1) -> bool:
        return lib().lsa_push_flush(self._h, int(timeout_ms)) == 0

    @property
    def pending(self) -> int:
        return int(lib().lsa_push_pending(self._h))

    @property
    def connected(self) -> bool:
        return bool(lib().lsa_push_connected(self._h))

    def inject_faults(self, drop_every: int = 0, delay_ms: int = 0) -> None:
        lib().lsa_push_fault(self._h, int(drop_every), int(delay_ms))

    def close(self, linger_ms: Optional[int] = 2000) -> None:
        if self._h:
            if linger_ms:
                self.flush(linger_ms)
            lib().lsa_push_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close(linger_ms=0)
        except Exception:
            pass
