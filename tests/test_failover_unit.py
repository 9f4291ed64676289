"""Pipeline -> chain failover, one controller in-process (the reference's elastic
path is the live re-config of ``/root/reference/utils/node_worker.py:445-474``).

A NodeController runs in pipeline mode around a stand-in stage server whose ``serve()`` blocks
until the test makes it fail (a lost peer). These tests pin the message-ordering contract of
``NodeController._run_pipeline``: a chain config that reaches the config port while the pipeline
listener thread is still alive is applied, never dropped; the controller only reports
``awaiting_redeploy`` once that listener is gone; requests that arrive while the pipeline is being
dropped, or that were in flight on it, get an error reply instead of silence."""
import json
import threading
import time

import torch

from llm_sharding_amd.parallel import protocol
from llm_sharding_amd.parallel.transport import PullSocket, PushSocket
from llm_sharding_amd.utils.node_worker import NodeController, ping_node


class _Req:
    def __init__(self, rid, reply_to):
        self.rid, self.reply_to = rid, reply_to


class _FakeStage:
    """What _run_pipeline needs of a PipelineServer: ``first``, ``serve()``, ``unfinished()``."""

    def __init__(self, first=False, inflight=()):
        self.first = first
        self.fail = threading.Event()
        self.serving = threading.Event()
        self.p2p = None
        self.ctrl = None
        self.start, self.end, self.replans = 0, 1, 0
        self._inflight = list(inflight)
        self.submitted = []

    def serve(self, stop_when_idle=True, should_stop=None):
        self.serving.set()
        while not self.fail.wait(0.01):
            if should_stop is not None and should_stop():
                return
        raise RuntimeError("Connection closed by peer [127.0.0.1]:12345")

    def unfinished(self):
        return list(self._inflight)

    def submit(self, ids, n, on_token=None, reply_to=None):
        self.submitted.append(ids)
        return len(self.submitted) - 1


def _send(port, msg):
    s = PushSocket(f"tcp://127.0.0.1:{port}")
    s.send_bytes(json.dumps(msg).encode())
    s.close(linger_ms=2000)


def _chain_cfg(first, ingress_port, data_port, layers):
    return {"src_addr": f"tcp://127.0.0.1:{data_port}", "dst_addr": f"tcp://127.0.0.1:{data_port}",
            "can_receive_user_request": first, "first_node_addr": f"tcp://127.0.0.1:{ingress_port}" if first else "",
            "shards_start": 0, "shards_end": layers}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _controller(tiny_shards, stage):
    ctrl = NodeController(tiny_shards, device="cpu", dtype=torch.float32, listen_port=0, wait_config=False,
                          verbose=False)
    ctrl.server = stage
    ctrl.tokenizer = None
    return ctrl


def test_chain_config_during_live_listener_is_applied(tiny_shards):
    from llm_sharding_amd.config import LlamaConfig
    L = LlamaConfig.from_pretrained(tiny_shards).num_hidden_layers
    stage = _FakeStage(first=False)
    ctrl = _controller(tiny_shards, stage)
    port = ctrl.listen_port
    th = threading.Thread(target=ctrl.run_worker_loop, kwargs={"max_new_tokens": 4, "max_idle_s": 30}, daemon=True)
    th.start()
    try:
        assert stage.serving.wait(10)
        # the master's chain config arrives while the pipeline listener still owns the socket
        _send(port, _chain_cfg(False, port, _free_port(), L))
        t0 = time.time()
        while not ctrl._early_configs:
            assert time.time() - t0 < 10, "chain config not queued by the live listener"
            time.sleep(0.01)
        st = ping_node("127.0.0.1", port, 2000)
        assert st is not None and st["mode"] == "pipeline" and st["phase"] == "serving"
        stage.fail.set()  # the peer dies: serve() raises, the stage is dropped
        t0 = time.time()
        while True:
            st = ping_node("127.0.0.1", port, 2000)
            if st is not None and st["configured"] and st["shards"] == [0, L]:
                break
            assert time.time() - t0 < 20, st
            time.sleep(0.05)
        assert st["phase"] == "chain" and st["pipeline_lost"]
    finally:
        _send(port, {"command": "shutdown"})
        th.join(timeout=20)
        ctrl.close()


def test_requests_during_drop_and_inflight_get_error_replies(tiny_shards):
    reply = PullSocket("tcp://127.0.0.1:0")
    to = f"tcp://127.0.0.1:{reply.port}"
    stage = _FakeStage(first=True, inflight=[_Req(7, to)])
    ctrl = _controller(tiny_shards, stage)
    port = ctrl.listen_port
    th = threading.Thread(target=ctrl.run_worker_loop, kwargs={"max_new_tokens": 4, "max_idle_s": 30}, daemon=True)
    th.start()
    try:
        assert stage.serving.wait(10)
        # abort_pipeline from the master: acknowledged, rank 0 stops scheduling
        st = ping_node("127.0.0.1", port, 5000, command="abort_pipeline")
        assert st is not None
        # the in-flight request is answered with an error, not dropped
        m = protocol.decode(reply.recv_bytes(timeout_ms=20000))
        assert m["request_id"] == 7 and "error" in m
        t0 = time.time()
        while (ping_node("127.0.0.1", port, 2000) or {}).get("phase") != "awaiting_redeploy":
            assert time.time() - t0 < 20
            time.sleep(0.05)
        assert ctrl._abort_timer is not None and not ctrl._abort_timer.is_alive()  # cancelled
        # a request after the drop is kept for the new ingress; a non-ingress chain role rejects it
        _send(port, {"command": "user_request", "input_ids": [[1, 2, 3]], "reply_to": to})
        from llm_sharding_amd.config import LlamaConfig
        L = LlamaConfig.from_pretrained(tiny_shards).num_hidden_layers
        _send(port, _chain_cfg(False, port, _free_port(), L))
        m = protocol.decode(reply.recv_bytes(timeout_ms=20000))
        assert m["request_id"] is None and "not the chain's ingress" in m["error"]
        assert stage.submitted == []  # nothing reached the dropped stage
    finally:
        _send(port, {"command": "shutdown"})
        th.join(timeout=20)
        ctrl.close()
        reply.close()
