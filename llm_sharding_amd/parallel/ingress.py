"""Request ingress of a PipelineServer (rank 0): the reference's ``user_request`` control
messages (``utils/node_worker.send_user_request``; the reference itself never reads requests in
serve mode) turned into ``PipelineServer.submit`` calls, and finished requests
pushed back to the client's ``reply_to`` address.

Used by ``serve.py`` (its own ingress port) and by :class:`..utils.node_worker.NodeController`
in pipeline mode (the controller's config port, when the master deploys the RCCL pipeline)."""
from __future__ import annotations

import json
import threading
from typing import Callable, Optional

from . import protocol
from .transport import Again, PullSocket, PushSocket


class Replies:
    """on_token callback: prints each finished request and pushes ``{"request_id",
    "output_ids", "text", "ttft_ms", "tpot_ms"}`` to its ``reply_to`` address."""

    def __init__(self, tokenizer=None, verbose: bool = True, on_done: Optional[Callable] = None):
        self.tok = tokenizer
        self.verbose = verbose
        self.on_done = on_done
        self.socks: dict = {}
        # __call__ runs on the serve thread, error() on the listener thread: one lock guards the
        # socket table and the sends (one PushSocket per reply_to, never two racing creations)
        self._lock = threading.Lock()

    def _send(self, reply_to: str, payload: bytes) -> None:
        with self._lock:
            sock = self.socks.get(reply_to)
            if sock is None:
                sock = self.socks[reply_to] = PushSocket(reply_to)
            sock.send_bytes(payload)

    def __call__(self, r, t) -> None:
        if not (t in r.eos_ids or len(r.output_ids) >= r.max_new_tokens):
            return
        text = self.tok.decode(r.output_ids) if self.tok is not None else ""
        if self.verbose:
            print(f"[INFO] request {r.rid} done: {len(r.output_ids)} tokens  ttft {r.ttft_ms:.1f} ms  "
                  f"output: {text!r}", flush=True)
        if self.on_done is not None:
            self.on_done(r, text)
        if r.reply_to:
            self._send(r.reply_to, protocol.encode({
                "request_id": r.rid, "output_ids": list(r.output_ids), "text": text,
                "ttft_ms": r.ttft_ms, "tpot_ms": r.tpot_ms}))

    def error(self, reply_to: Optional[str], reason: str, request_id=None) -> None:
        """Tell a client its request will not be served (``{"request_id", "error"}``)."""
        if self.verbose:
            print(f"[ERROR] request {request_id} not served: {reason}", flush=True)
        if not reply_to:
            return
        try:
            self._send(reply_to, protocol.encode({"request_id": request_id, "error": reason,
                                                  "output_ids": [], "text": ""}))
        except OSError as e:
            print(f"[WARNING] error reply to {reply_to} failed: {e}", flush=True)

    def close(self) -> None:
        with self._lock:
            for s in self.socks.values():
                s.close(linger_ms=2000)
            self.socks.clear()


def decode_message(raw: bytes) -> dict:
    return json.loads(raw) if protocol.is_json_message(raw) else protocol.decode(raw)


def submit_message(srv, msg: dict, tokenizer, default_new: int, replies: Replies) -> int:
    """Submit every prompt of a ``user_request`` message (``input_ids``: one list or a batch of
    lists, else ``text`` through the tokenizer). Returns the number of requests queued."""
    n_new = int(msg.get("max_new_tokens") or default_new)
    rows = msg.get("input_ids")
    if rows is None:
        if tokenizer is None:
            print("[ERROR] text request but no tokenizer", flush=True)
            return 0
        rows = [tokenizer.encode(msg.get("text", ""))]
    elif rows and not isinstance(rows[0], (list, tuple)):
        rows = [rows]
    n = 0
    for ids in rows:
        try:
            srv.submit(ids, n_new, on_token=replies, reply_to=msg.get("reply_to"))
            n += 1
        except ValueError as e:
            replies.error(msg.get("reply_to"), f"request rejected: {e}")
    return n


def run_ingress(srv, sock: PullSocket, tokenizer, stop_evt: threading.Event, default_new: int,
                replies: Replies, on_other: Optional[Callable[[dict], None]] = None,
                accepting: Optional[Callable[[], Optional[str]]] = None) -> None:
    """Read control messages from ``sock`` until ``shutdown`` (or ``stop_evt``): queue
    ``user_request`` prompts on the server; other commands go to ``on_other`` (e.g. ping).
    ``accepting()`` returning a reason string refuses new requests with an error reply (a
    pipeline being dropped after a lost rank must not swallow them)."""
    while not stop_evt.is_set():
        try:
            raw = sock.recv_bytes(timeout_ms=200)
        except Again:
            continue
        msg = decode_message(raw)
        cmd = msg.get("command") if isinstance(msg, dict) else None
        if cmd == "shutdown":
            stop_evt.set()
            break
        if cmd == "user_request":
            why = accepting() if accepting is not None else None
            if why:
                replies.error(msg.get("reply_to"), why)
                continue
            submit_message(srv, msg, tokenizer, default_new, replies)
        elif on_other is not None:
            on_other(msg)
        else:
            print(f"[WARNING] ingress: unknown message {cmd!r}", flush=True)


__all__ = ["Replies", "run_ingress", "submit_message", "decode_message"]
