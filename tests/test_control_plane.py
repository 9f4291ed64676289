"""CPU tests of the data/control plane: protocol, native TCP transport, NodeWorker chains,
NodeController + ConfigSender deployments (BASELINE.json config 1: shards on CPU with socket
hand-off on localhost), clear-KV ring, hot re-configuration, fault injection."""
import json
import socket
import threading
import time

import pytest
import torch

from llm_sharding_amd.models import weights as W
from llm_sharding_amd.models.reference import ReferenceLlama
from llm_sharding_amd.parallel import protocol
from llm_sharding_amd.parallel.communicator import reset_local_transport
from llm_sharding_amd.parallel.transport import Again, PullSocket, PushSocket
from llm_sharding_amd.utils.config_sender import ConfigSender
from llm_sharding_amd.utils.node_worker import NodeController, NodeWorker, send_shutdown, send_user_request


def free_ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


# ----------------------------------------------------------------------------- protocol
def test_protocol_roundtrip_all_kinds():
    msgs = [
        {"hidden_states": torch.randn(2, 3, 8).to(torch.bfloat16), "batch_size": 2, "seq_len": 3},
        {"hidden_states": torch.randn(1, 1, 8, dtype=torch.float16), "cos": torch.randn(1, 1, 4), "sin": torch.randn(1, 1, 4)},
        torch.tensor([17, 3], dtype=torch.long),
        {"command": "clear_KV_cache", "origin_node": {"src_addr": "tcp://*:1", "dst_addr": "tcp://h:2",
                                                      "shards_start": 0, "shards_end": 4}},
        {"profile_command": "prefill_ack"},
        {"a": (1, 2.5, None, True), "b": [torch.zeros(0, 3), "x"]},
    ]
    for m in msgs:
        d = protocol.decode(protocol.encode(m))
        if isinstance(m, torch.Tensor):
            assert torch.equal(d, m) and d.dtype == m.dtype
            continue
        for k, v in m.items():
            if isinstance(v, torch.Tensor):
                assert d[k].dtype == v.dtype and torch.equal(d[k], v)
            elif k == "b":
                assert d[k][0].shape == (0, 3) and d[k][1] == "x"
            else:
                assert d[k] == v


def test_protocol_rejects_garbage():
    with pytest.raises(ValueError):
        protocol.decode(b"not a message at all")
    with pytest.raises(TypeError):
        protocol.encode({1: 2})


# ----------------------------------------------------------------------------- transport
def test_transport_basic_and_again():
    (port,) = free_ports(1)
    pull = PullSocket(f"tcp://*:{port}")
    with pytest.raises(Again):
        pull.recv_bytes(0)
    push = PushSocket(f"tcp://127.0.0.1:{port}")
    for i in range(50):
        push.send_bytes(bytes([i]) * (i * 1000 + 1))
    assert push.flush(5000)
    got = [pull.recv_bytes(2000) for _ in range(50)]
    assert [len(g) for g in got] == [i * 1000 + 1 for i in range(50)]
    assert got[7][0] == 7
    push.close()
    pull.close()


def test_transport_send_before_bind_is_queued():
    (port,) = free_ports(1)
    push = PushSocket(f"tcp://127.0.0.1:{port}")
    push.send_bytes(b"early bird")
    time.sleep(0.2)
    pull = PullSocket(f"tcp://*:{port}")  # peer appears later (ZMQ semantics)
    assert pull.recv_bytes(5000) == b"early bird"
    push.close()
    pull.close()


def test_transport_large_and_many_pushers():
    (port,) = free_ports(1)
    pull = PullSocket(f"tcp://*:{port}")
    pushers = [PushSocket(f"tcp://127.0.0.1:{port}") for _ in range(4)]
    big = bytes(range(256)) * (64 * 1024)  # 16 MiB
    for p in pushers:
        p.send_bytes(big)
    got = [pull.recv_bytes(10000) for _ in pushers]
    assert all(g == big for g in got)
    for p in pushers:
        p.close()
    pull.close()


def test_transport_fault_injection_drop():
    (port,) = free_ports(1)
    pull = PullSocket(f"tcp://*:{port}")
    push = PushSocket(f"tcp://127.0.0.1:{port}")
    push.inject_faults(drop_every=2)
    for i in range(6):
        push.send_bytes(str(i).encode())
    push.flush(5000)
    got = []
    while True:
        try:
            got.append(pull.recv_bytes(300).decode())
        except Again:
            break
    assert got == ["0", "2", "4"]
    push.close()
    pull.close()


# ----------------------------------------------------------------------------- chains
def golden(tiny_shards, prompt, n):
    cfg, emb, layers, fn, lm = W.load_full_model(tiny_shards)
    return ReferenceLlama(cfg, emb, layers, fn, lm).generate(prompt, n)[0].tolist()


@pytest.mark.parametrize("backend", ["tcp", "local"])
def test_four_stage_ring_manual(tiny_shards, backend):
    """Reference go_through_every_shards harness (node_profiler.py:1174-1236): 4 NodeWorkers
    in one process, stepping the ring by hand."""
    reset_local_transport()
    ports = free_ports(4)
    ranges = [(0, 1), (1, 2), (2, 3), (3, 4)]
    nodes = []
    for i, (a, b) in enumerate(ranges):
        w = NodeWorker(f"tcp://*:{ports[i]}", f"tcp://127.0.0.1:{ports[(i + 1) % 4]}", i == 0, tiny_shards,
                       device="cpu", dtype=torch.float32, backend=backend, verbose=False)
        w.load_shards(a, b)
        nodes.append(w)
    prompt = torch.tensor([[1, 40, 41, 42, 43]])
    data0 = nodes[0].receive_user_request(input_ids=prompt)
    for _ in range(8):
        d = nodes[0].pass_through_shard(data0)
        nodes[0].communicator.transfer_data(d)
        for k in (1, 2, 3):
            d = nodes[k].communicator.receive_data(timeout_ms=5000)
            assert NodeWorker.is_next_state_info(d)
            out = nodes[k].pass_through_shard(d)
            nodes[k].communicator.transfer_data(out)
        tok = nodes[0].communicator.receive_data(timeout_ms=5000)
        assert isinstance(tok, torch.Tensor)
        reached_end, data0 = nodes[0].receive_next_token(tok, max_new_tokens=8)
        if reached_end:
            break
    got = nodes[0].output_ids()[0, 5:].tolist()
    assert got == golden(tiny_shards, prompt, len(got))
    for n in nodes:
        n.close()


def _start_controllers(tiny_shards, n, cfg_ports):
    ctrls, threads = [], []
    for i in range(n):
        c = NodeController(tiny_shards, device="cpu", dtype=torch.float32, listen_port=cfg_ports[i],
                           wait_config=False, verbose=False)
        ctrls.append(c)
    return ctrls


def _configure(ctrls, cfg_ports, data_ports, ranges, ingress=0):
    n = len(ranges)
    for i, (a, b) in enumerate(ranges):
        s = ConfigSender(node_port=cfg_ports[i])
        s.build_config(a, b, i == ingress, f"tcp://*:{data_ports[i]}", f"tcp://127.0.0.1:{data_ports[(i + 1) % n]}",
                       first_node_addr=f"tcp://127.0.0.1:{data_ports[0]}" if i == ingress else "")
        assert s.send_config("127.0.0.1")
        s.close()
    for c in ctrls:  # each controller picks its config up (blocking) like the reference __init__
        c.received_config = c._receive_config()
        c._apply_new_role(c.received_config)


def test_controllers_end_to_end_request_clear_and_reconfig(tiny_shards):
    cfg_ports = free_ports(3)
    data_ports = free_ports(3)
    ctrls = _start_controllers(tiny_shards, 3, cfg_ports)
    _configure(ctrls, cfg_ports, data_ports, [(0, 2), (2, 3), (3, 4)])
    threads = [threading.Thread(target=c.run_worker_loop, kwargs={"max_new_tokens": 6}, daemon=True) for c in ctrls]
    for t in threads:
        t.start()
    prompt = [[1, 70, 71, 72]]
    send_user_request("127.0.0.1", cfg_ports[0], input_ids=prompt)
    t0 = time.time()
    while not ctrls[0].finished_outputs and time.time() - t0 < 60:
        time.sleep(0.05)
    assert ctrls[0].finished_outputs, "no output produced"
    out = ctrls[0].finished_outputs[0][0, 4:].tolist()
    assert out == golden(tiny_shards, torch.tensor(prompt), 6)
    # the clear-KV ring reached every stage (all KV lengths back to 0)
    time.sleep(0.5)
    assert all(c.node_worker.engine.seq_len[0] == 0 for c in ctrls)
    # hot re-configuration: new layer split, same roles; second request
    for i, (a, b) in enumerate([(0, 1), (1, 3), (3, 4)]):
        s = ConfigSender(node_port=cfg_ports[i])
        s.build_config(a, b, i == 0, f"tcp://*:{data_ports[i]}", f"tcp://127.0.0.1:{data_ports[(i + 1) % 3]}",
                       first_node_addr=f"tcp://127.0.0.1:{data_ports[0]}" if i == 0 else "")
        assert s.send_config("127.0.0.1")
        s.close()
    t0 = time.time()
    while time.time() - t0 < 30 and [(c.node_worker.start, c.node_worker.end) for c in ctrls] != [(0, 1), (1, 3), (3, 4)]:
        time.sleep(0.05)
    assert [(c.node_worker.start, c.node_worker.end) for c in ctrls] == [(0, 1), (1, 3), (3, 4)]
    prompt2 = [[1, 9, 99, 199, 29]]
    send_user_request("127.0.0.1", cfg_ports[0], input_ids=prompt2)
    t0 = time.time()
    while len(ctrls[0].finished_outputs) < 2 and time.time() - t0 < 60:
        time.sleep(0.05)
    out2 = ctrls[0].finished_outputs[1][0, 5:].tolist()
    assert out2 == golden(tiny_shards, torch.tensor(prompt2), 6)
    for p in cfg_ports:
        send_shutdown("127.0.0.1", p)
    for t in threads:
        t.join(timeout=10)
    for c in ctrls:
        c.close()


def test_noncausal_prefill_compat(tiny_shards):
    """Q1: the reference's unmasked prefill is reproducible with noncausal_prefill=True."""
    cfg, emb, layers, fn, lm = W.load_full_model(tiny_shards)
    ref = ReferenceLlama(cfg, emb, layers, fn, lm, causal=False)
    prompt = torch.tensor([[1, 5, 6, 7, 8, 9]])
    want, _ = ref.step(prompt)
    (p,) = free_ports(1)
    w = NodeWorker(f"tcp://*:{p}", f"tcp://127.0.0.1:{p}", True, tiny_shards, dtype=torch.float32,
                   noncausal_prefill=True, verbose=False)
    w.load_shards(0, cfg.num_hidden_layers)
    tok = w.pass_through_shard(w.receive_user_request(input_ids=prompt))
    assert int(tok[0]) == int(want[0])
    w.close()


def test_worker_role_errors(tiny_shards):
    (p,) = free_ports(1)
    w = NodeWorker(f"tcp://*:{p}", f"tcp://127.0.0.1:{p}", False, tiny_shards, dtype=torch.float32, verbose=False)
    with pytest.raises(RuntimeError):
        w.receive_user_request("hi")
    with pytest.raises(ValueError):
        w.load_shards(3, 2)
    w.load_shards(1, 2)
    with pytest.raises(RuntimeError):
        w.pass_through_shard({"hidden_states": torch.zeros(1, 1, 256), "batch_size": 1, "seq_len": 1})
    with pytest.raises(RuntimeError):
        w.pass_through_shard({"weird": 1})
    cmd = w.build_clear_KV_cache_command()
    assert NodeWorker.is_clear_KV_cache_command(cmd) and w.is_clear_KV_cache_command_origin(cmd)
    w.close()


def test_foreign_command_is_not_a_config(tiny_shards):
    """A command of another mode (the master's abort_pipeline sent during a failover, a replan)
    reaching an unconfigured controller is acknowledged and ignored; the next real config is
    the one applied."""
    from llm_sharding_amd.utils.node_worker import ping_node
    cport, dport = free_ports(2)
    ctrl = NodeController(tiny_shards, device="cpu", dtype=torch.float32, listen_port=cport, wait_config=False,
                          verbose=False)
    box = {}
    th = threading.Thread(target=lambda: box.update(cfg=ctrl._receive_config()), daemon=True)
    th.start()
    try:
        assert ping_node("127.0.0.1", cport, 5000, command="abort_pipeline") is not None
        s = PushSocket(f"tcp://127.0.0.1:{cport}")
        s.send_bytes(json.dumps({"command": "replan", "stages": [[0, 2]]}).encode())
        s.close(linger_ms=2000)
        cs = ConfigSender(node_port=cport)
        cs.build_config(0, 2, True, f"tcp://*:{dport}", f"tcp://127.0.0.1:{dport}",
                        first_node_addr=f"tcp://127.0.0.1:{cport}")
        assert cs.send_config("127.0.0.1", 5000)
        th.join(timeout=30)
        assert box["cfg"]["shards_start"] == 0 and box["cfg"]["shards_end"] == 2 and "command" not in box["cfg"]
    finally:
        ctrl.close()


def _rccl_chain_worker(rank, port, ports, shards, n_new, q):
    import torch.distributed as dist
    from llm_sharding_amd.utils.node_worker import NodeWorker
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    from llm_sharding_amd.parallel.communicator import init_edge_groups
    init_edge_groups()
    try:
        w = NodeWorker(f"tcp://*:{ports[rank]}", f"tcp://127.0.0.1:{ports[1 - rank]}", rank == 0, shards,
                       device="cpu", dtype=torch.float32, backend="rccl", verbose=False)
        w.load_shards(0, 2) if rank == 0 else w.load_shards(2, 4)
        if rank == 0:
            d = w.receive_user_request(input_ids=torch.tensor([[1, 33, 44, 55, 66]]))
            while True:
                w.communicator.transfer_data(w.pass_through_shard(d))
                tok = w.communicator.receive_data(timeout_ms=60000)
                end, d = w.receive_next_token(tok, max_new_tokens=n_new)
                if end:
                    break
            w.communicator.transfer_data({"command": "stop"})
            q.put(w.output_ids()[0].tolist())
        else:
            while True:
                x = w.communicator.receive_data(timeout_ms=60000)
                if isinstance(x, dict) and x.get("command") == "stop":
                    break
                w.communicator.transfer_data(w.pass_through_shard(x))
        w.communicator.flush()
        w.close()
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_communicator_rccl_backend_two_processes(tiny_shards):
    """Reference-API NodeWorkers in two processes with backend="rccl": envelopes over TCP,
    hidden states / token ids via torch.distributed send/recv (gloo here, RCCL on GPUs)."""
    import multiprocessing as mp
    import socket as _s
    socks = [_s.socket() for _ in range(3)]
    for s in socks:
        s.bind(("127.0.0.1", 0))
    ports = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    n_new = 5
    ps = [ctx.Process(target=_rccl_chain_worker, args=(r, ports[2], ports[:2], tiny_shards, n_new, q))
          for r in range(2)]
    for p in ps:
        p.start()
    try:
        got = q.get(timeout=240)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    cfg, emb, layers, fn, lm = W.load_full_model(tiny_shards)
    prompt = torch.tensor([[1, 33, 44, 55, 66]])
    want = ReferenceLlama(cfg, emb, layers, fn, lm).generate(prompt, n_new)[0].tolist()
    eos = set(cfg.eos_ids)
    if any(t in eos for t in want):
        want = want[:next(i for i, t in enumerate(want) if t in eos) + 1]
    assert got == prompt[0].tolist() + want
