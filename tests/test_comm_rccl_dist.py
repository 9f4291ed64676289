"""The rccl-backend Communicator (envelopes over the native TCP transport, tensors over
torch.distributed point-to-point) on gloo with 3 processes: one process group per DIRECTED ring
edge, several messages in flight in both ring directions at once, a re-ordered ring after a
hot re-configuration (change_ranks), receive timeouts surfacing as errors, and the rejected
drop-fault hook. RCCL runs the same code on GPUs (start_node.py --backend rccl)."""
import multiprocessing as mp
import socket

import pytest
import torch


def _ports(n):
    socks = [socket.socket() for _ in range(n)]
    for s in socks:
        s.bind(("127.0.0.1", 0))
    ports = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    return ports


def _worker(rank, world, port, fwd_ports, bwd_ports, new_ports, q):
    import torch.distributed as dist
    from llm_sharding_amd.parallel.communicator import Communicator, init_edge_groups
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        groups = init_edge_groups()
        assert len(groups) == world * (world - 1)
        nxt, prv = (rank + 1) % world, (rank - 1) % world
        # forward ring r -> r+1 and backward ring r -> r-1, both live at once
        fwd = Communicator(f"tcp://*:{fwd_ports[rank]}", f"tcp://127.0.0.1:{fwd_ports[nxt]}", backend="rccl",
                           device=torch.device("cpu"), recv_timeout_s=60)
        bwd = Communicator(f"tcp://*:{bwd_ports[rank]}", f"tcp://127.0.0.1:{bwd_ports[prv]}", backend="rccl",
                           device=torch.device("cpu"), rccl_ranks=(nxt, prv), recv_timeout_s=60)
        n_msg = 3
        for i in range(n_msg):  # several messages queued in each direction before any receive
            fwd.transfer_data({"i": i, "x": torch.full((64, 1024), rank * 100.0 + i), "src": rank})
            bwd.transfer_data({"i": i, "x": torch.full((1024,), -rank * 100.0 - i), "src": rank})
        got_f = [fwd.receive_data(timeout_ms=60000) for _ in range(n_msg)]
        got_b = [bwd.receive_data(timeout_ms=60000) for _ in range(n_msg)]
        for i in range(n_msg):
            assert got_f[i]["i"] == i and got_f[i]["src"] == prv
            assert torch.all(got_f[i]["x"] == prv * 100.0 + i)
            assert got_b[i]["i"] == i and got_b[i]["src"] == nxt
            assert torch.all(got_b[i]["x"] == -nxt * 100.0 - i)
        fwd.flush()
        bwd.flush()
        bwd.close()
        with pytest.raises(ValueError):
            fwd.inject_faults(drop_every=2)
        # hot re-configuration: the ring order becomes 0 -> 2 -> 1 -> 0
        order = [0, 2, 1]
        pos = order.index(rank)
        src, dst = order[(pos - 1) % world], order[(pos + 1) % world]
        fwd.change_src_addr(f"tcp://*:{new_ports[rank]}")
        fwd.change_dst_addr(f"tcp://127.0.0.1:{new_ports[dst]}")
        fwd.change_ranks(src, dst)
        fwd.transfer_data({"hello_from": rank, "t": torch.arange(10.0) + rank})
        m = fwd.receive_data(timeout_ms=60000)
        assert m["hello_from"] == src and torch.equal(m["t"], torch.arange(10.0) + src)
        fwd.flush()
        dist.barrier()
        fwd.close()
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_rccl_communicator_edges_both_directions_and_reorder():
    world = 3
    port = _ports(1)[0]
    fwd, bwd, new = _ports(world), _ports(world), _ports(world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fwd, bwd, new, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, v = q.get(timeout=240)
            res[r] = v
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert res == {r: "ok" for r in range(world)}, res
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]


def _timeout_worker(rank, port, ports, q):
    import torch.distributed as dist
    from llm_sharding_amd.parallel import protocol
    from llm_sharding_amd.parallel.communicator import Communicator, init_edge_groups
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        init_edge_groups()
        c = Communicator(f"tcp://*:{ports[rank]}", f"tcp://127.0.0.1:{ports[1 - rank]}", backend="rccl",
                         device=torch.device("cpu"), recv_timeout_s=3)
        if rank == 0:
            # an envelope that announces a tensor, whose bytes never follow
            ph = {"x": {"__rccl_tensor__": 0, "shape": [4], "dtype": "float32"}}
            c.send_socket.send_bytes(protocol.encode(ph))
            c.send_socket.flush(5000)
            q.put((rank, "sent"))
        else:
            try:
                c.receive_data(timeout_ms=30000)
                q.put((rank, "no error"))
            except RuntimeError as e:
                verdict = "timeout" if "timed out" in str(e) or "failed" in str(e) else repr(e)
                # the timed-out irecv stays posted: the communicator refuses further traffic
                for op in (lambda: c.receive_data(no_block=True), lambda: c.transfer_data({"a": 1})):
                    try:
                        op()
                        verdict = "usable after failure"
                    except RuntimeError as e2:
                        if "unusable" not in str(e2):
                            verdict = repr(e2)
                q.put((rank, verdict))
        dist.barrier()
        c.close()
    finally:
        dist.destroy_process_group()


def test_rccl_communicator_recv_timeout_is_an_error():
    port = _ports(1)[0]
    ports = _ports(2)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_timeout_worker, args=(r, port, ports, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(2):
            r, v = q.get(timeout=120)
            res[r] = v
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert res == {0: "sent", 1: "timeout"}, res
