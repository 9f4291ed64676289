"""Master-side configuration client (reference C7, ``utils/config_sender.py:4-47``).

``ConfigSender(node_port=40700)``, ``build_config(shards_start, shards_end,
can_receive_user_request, src_addr, dst_addr, first_node_addr="")`` and
``send_config(node_ip)`` with the same 6-key JSON schema. The native PUSH socket queues the
message and ``send_config`` flushes it before returning, so the sender no longer has to be
kept alive (``while True: pass``) for delivery. Optional extra keys
(e.g. ``backend``, ``rank``, ``world_size``) ride along for the RCCL pipeline mode.
"""
from __future__ import annotations

import json
from typing import Optional

from ..parallel.transport import PushSocket


class ConfigSender:
    def __init__(self, node_port: int = 40700):
        self.node_port = node_port
        self.node_addr = ""
        self.config: dict = {}
        self.send_socket: Optional[PushSocket] = None

    def build_config(self, shards_start: int, shards_end: int, can_receive_user_request: bool,
                     src_addr: str, dst_addr: str, first_node_addr: str = "", **extra) -> dict:
        if can_receive_user_request and first_node_addr == "":
            raise ValueError("first_node_addr cannot be empty when can_receive_user_request = True")
        if not (0 <= shards_start < shards_end):
            raise ValueError("invalid shard range")
        self.config = {
            "src_addr": src_addr,
            "dst_addr": dst_addr,
            "can_receive_user_request": can_receive_user_request,
            "first_node_addr": first_node_addr,
            "shards_start": shards_start,
            "shards_end": shards_end,
        }
        self.config.update(extra)
        return self.config

    def send_config(self, node_ip: str, timeout_ms: int = 10000) -> bool:
        addr = "tcp://" + node_ip + ":" + str(self.node_port)
        if addr != self.node_addr:
            if self.send_socket is not None:
                self.send_socket.close()
            self.send_socket = PushSocket(addr)
            self.node_addr = addr
        self.send_socket.send_bytes(json.dumps(self.config).encode())
        return self.send_socket.flush(timeout_ms)

    def close(self) -> None:
        if self.send_socket is not None:
            self.send_socket.close()
            self.send_socket = None


if __name__ == "__main__":
    sender = ConfigSender()
    sender.build_config(shards_start=0, shards_end=10, can_receive_user_request=True,
                        src_addr="tcp://*:40800", dst_addr="tcp://127.0.0.1:40800",
                        first_node_addr="tcp://127.0.0.1:40800")
    print("delivered:", sender.send_config(node_ip="127.0.0.1"))
