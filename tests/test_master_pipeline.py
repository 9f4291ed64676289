"""Master -> ConfigSender -> NodeControllers -> micro-batched pipeline, end to end (SURVEY.md
C16 + §2.5; BASELINE north star: "the master_node scheduler places shards on the GPUs of one
node and the hand-off becomes a pipeline-parallel RCCL send/recv chain").

Four controller processes form one torch.distributed job (gloo here; start_node.py --backend
rccl uses RCCL on GPUs) and wait on their config ports like the reference's run_this.sh nodes.
The master plans the layer ranges, sends every controller the reference config extended with
``mode="pipeline"`` + rank/world, submits requests to rank 0's config port with a ``reply_to``
address and receives the finished outputs, which must equal the fp32 golden model's greedy
generation token for token."""
import multiprocessing as mp
import socket
import time

import pytest
import torch

from llm_sharding_amd.models import weights as W
from llm_sharding_amd.models.reference import ReferenceLlama
from llm_sharding_amd.utils.node_worker import ping_node


def _ports(n):
    socks = [socket.socket() for _ in range(n)]
    for s in socks:
        s.bind(("127.0.0.1", 0))
    ports = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    return ports


def _static_ports(n):
    """Free ports below the kernel's ephemeral range (32768-60999 here): the controllers bind their
    config / data ports after the gloo job exists, and an ephemeral pick could meanwhile be taken
    by one of gloo's (or a ZMQ ping's) own sockets - a static pick cannot."""
    import random
    out = []
    while len(out) < n:
        p = random.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("0.0.0.0", p))
        except OSError:
            continue
        finally:
            s.close()
        if p not in out:
            out.append(p)
    return out


def _node(rank, world, port, cfg_port, shards, q):
    import torch.distributed as dist
    from llm_sharding_amd.parallel.communicator import init_edge_groups
    from llm_sharding_amd.utils.node_worker import NodeController
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        init_edge_groups()  # what start_node.py --backend rccl does after init_process_group
        ctrl = NodeController(shards, device="cpu", dtype=torch.float32, listen_port=cfg_port, backend="rccl",
                              verbose=False)
        assert ctrl.server is not None and ctrl.status()["mode"] == "pipeline"
        ctrl.run_worker_loop(max_new_tokens=8)
        outs = [o.reshape(-1).tolist() if torch.is_tensor(o) else o for o in ctrl.finished_outputs]  # chain: tensors
        q.put((rank, outs if rank == 0 or outs else "ok"))  # (a chain ingress after a failover: its outputs)
        ctrl.close()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
        raise
    finally:
        if dist.is_initialized():  # (a pipeline that lost a rank has destroyed it already)
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [4])
def test_master_deploys_rccl_pipeline_token_exact(tiny_shards, world):
    from llm_sharding_amd.parallel import protocol
    from llm_sharding_amd.parallel.scheduler import DeviceSpec
    from llm_sharding_amd.parallel.transport import PullSocket
    from llm_sharding_amd.utils.master_node import MasterNode
    port = _ports(1)[0]
    cfg_ports, data_ports = _static_ports(world), _static_ports(world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_node, args=(r, world, port, cfg_ports[r], tiny_shards, q)) for r in range(world)]
    for p in ps:
        p.start()
    reply = PullSocket("tcp://127.0.0.1:0")
    try:
        devs = [DeviceSpec(host="127.0.0.1", config_port=cfg_ports[i], data_port=data_ports[i]) for i in range(world)]
        master = MasterNode.from_shards(tiny_shards, devs)
        cfgs = master.deploy_pipeline(batch=2, microbatches=world, max_seq=64, prefill_budget=64)
        assert [c["rank"] for c in cfgs] == list(range(world)) and all(c["mode"] == "pipeline" for c in cfgs)
        ranges = [(c["shards_start"], c["shards_end"]) for c in cfgs]
        assert ranges[0][0] == 0 and all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
        prompts = [[1, 33, 44, 55, 66], [7, 8, 9], [100, 5, 17, 200, 3, 41, 12], [2, 2, 2, 2]]
        n_new = 6
        for pr in prompts:
            master.submit(input_ids=[pr], max_new_tokens=n_new, reply_to=f"tcp://127.0.0.1:{reply.port}")
        got = {}
        for _ in prompts:
            m = protocol.decode(reply.recv_bytes(timeout_ms=120000))
            got[m["request_id"]] = m["output_ids"]
        st = master.health()
        assert all(s is not None and s["mode"] == "pipeline" for _, s in st)
        master.shutdown()
        res = {}
        for _ in range(world):
            r, v = q.get(timeout=120)
            res[r] = v
    finally:
        reply.close()
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(res[r] == "ok" for r in range(1, world)), res
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    cfg, emb, layers, fn, lm = W.load_full_model(tiny_shards)
    ref = ReferenceLlama(cfg, emb, layers, fn, lm)
    eos = set(cfg.eos_ids)
    for rid, pr in enumerate(prompts):
        want = ref.generate(torch.tensor([pr]), n_new)[0].tolist()
        if any(t in eos for t in want):
            want = want[:next(i for i, t in enumerate(want) if t in eos) + 1]
        assert got[rid] == want, (rid, got[rid], want)
    assert sorted(map(tuple, res[0])) == sorted(tuple(got[r]) for r in range(len(prompts)))


@pytest.fixture(scope="module")
def tiny8_shards(tmp_path_factory):
    from llm_sharding_amd.config import tiny
    from llm_sharding_amd.models.weights import write_random_shards
    d = tmp_path_factory.mktemp("shards8")
    return write_random_shards(tiny(layers=8), str(d / "tiny8-llama"), dtype=torch.float32, seed=11)


def _golden(shards, prompts, n_new):
    cfg, emb, layers, fn, lm = W.load_full_model(shards)
    ref = ReferenceLlama(cfg, emb, layers, fn, lm)
    eos = set(cfg.eos_ids)
    out = []
    for pr in prompts:
        want = ref.generate(torch.tensor([pr]), n_new)[0].tolist()
        if any(t in eos for t in want):
            want = want[:next(i for i, t in enumerate(want) if t in eos) + 1]
        out.append(want)
    return out


def test_master_replans_live_pipeline_token_exact(tiny8_shards):
    """Live re-shard of the DEPLOYED pipeline (reference hot re-config, node_worker.py:445-474):
    deploy 4 ranks, serve, re-plan inside the same world (explicit ranges moving two
    boundaries while a request is in flight, then a speed-driven re-plan through the planner),
    serve again - every output equals the fp32 golden model's greedy tokens."""
    from llm_sharding_amd.parallel import protocol
    from llm_sharding_amd.parallel.scheduler import DeviceSpec
    from llm_sharding_amd.parallel.transport import PullSocket
    from llm_sharding_amd.utils.master_node import MasterNode
    world = 4
    port = _ports(1)[0]
    cfg_ports, data_ports = _static_ports(world), _static_ports(world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_node, args=(r, world, port, cfg_ports[r], tiny8_shards, q)) for r in range(world)]
    for p in ps:
        p.start()
    reply = PullSocket("tcp://127.0.0.1:0")
    to = f"tcp://127.0.0.1:{reply.port}"
    rounds = [[[1, 33, 44, 55, 66], [7, 8, 9]], [[100, 5, 17, 200, 3, 41, 12], [2, 2, 2, 2]], [[9, 19, 29], [4, 40, 4]]]
    n_new = 6
    got, rid = [], 0

    def serve(prompts):
        nonlocal rid
        for pr in prompts:
            master.submit(input_ids=[pr], max_new_tokens=n_new, reply_to=to)
        out = {}
        for _ in prompts:
            m = protocol.decode(reply.recv_bytes(timeout_ms=120000))
            out[m["request_id"]] = m["output_ids"]
        got.append([out[rid + i] for i in range(len(prompts))])
        rid += len(prompts)

    try:
        devs = [DeviceSpec(host="127.0.0.1", config_port=cfg_ports[i], data_port=data_ports[i]) for i in range(world)]
        master = MasterNode.from_shards(tiny8_shards, devs)
        cfgs = master.deploy_pipeline(batch=2, microbatches=world, max_seq=64, prefill_budget=64)
        before = [[c["shards_start"], c["shards_end"]] for c in cfgs]
        assert before == [[0, 2], [2, 4], [4, 6], [6, 8]], before
        serve(rounds[0])
        # a request in flight while the re-plan arrives: it finishes on the old split
        master.submit(input_ids=[[5, 6, 7, 8]], max_new_tokens=n_new, reply_to=to)
        new = master.replan(stages=[[0, 3], [3, 4], [4, 7], [7, 8]])
        m = protocol.decode(reply.recv_bytes(timeout_ms=120000))
        inflight = m["output_ids"]
        rid += 1
        st = master.health()
        assert [s["shards"] for _, s in st] == new and all(s["replans"] == 1 for _, s in st), st
        serve(rounds[1])
        # planner-driven: rank 1 is 3x slower -> it gets the fewest layers
        new2 = master.replan(speeds=[1.0, 3.0, 1.0, 1.0])
        assert new2 != new and new2[1][1] - new2[1][0] == min(b - a for a, b in new2), new2
        serve(rounds[2])
        master.shutdown()
        res = {}
        for _ in range(world):
            r, v = q.get(timeout=120)
            res[r] = v
    finally:
        reply.close()
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(res[r] == "ok" for r in range(1, world)), res
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    for prompts, outs in zip(rounds, got):
        assert outs == _golden(tiny8_shards, prompts, n_new), (prompts, outs)
    assert inflight == _golden(tiny8_shards, [[5, 6, 7, 8]], n_new)[0]


@pytest.mark.parametrize("dead", [2, 0])
def test_pipeline_failover_to_chain_token_exact(tiny8_shards, dead):
    """Failure of a DEPLOYED pipeline rank (reference failure handling is a
    restart): 4 ranks serve, rank 2's process is killed, MasterNode.failover() notices it (no
    pong), the survivors drop the torchrun world (abort_pipeline -> each releases its stage and
    process groups) and are re-deployed as a 3-stage ZMQ chain over the same layers; requests
    before and after the failure produce the fp32 golden model's greedy tokens. dead = 0: the
    ingress itself is lost (the survivors fail on its closed connections; rank 1 becomes the
    chain's ingress)."""
    from llm_sharding_amd.parallel import protocol
    from llm_sharding_amd.parallel.scheduler import DeviceSpec
    from llm_sharding_amd.parallel.transport import PullSocket
    from llm_sharding_amd.utils.master_node import MasterNode
    world, n_new = 4, 6
    port = _ports(1)[0]
    cfg_ports, data_ports = _static_ports(world), _static_ports(world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_node, args=(r, world, port, cfg_ports[r], tiny8_shards, q)) for r in range(world)]
    for p in ps:
        p.start()
    reply = PullSocket("tcp://127.0.0.1:0")
    before = [[1, 33, 44, 55, 66], [7, 8, 9]]
    after = [1, 40, 41, 42]
    res = {}
    try:
        devs = [DeviceSpec(host="127.0.0.1", config_port=cfg_ports[i], data_port=data_ports[i]) for i in range(world)]
        master = MasterNode.from_shards(tiny8_shards, devs)
        master.deploy_pipeline(batch=2, microbatches=world, max_seq=64, prefill_budget=64)
        for pr in before:
            master.submit(input_ids=[pr], max_new_tokens=n_new, reply_to=f"tcp://127.0.0.1:{reply.port}")
        got = {}
        for _ in before:
            m = protocol.decode(reply.recv_bytes(timeout_ms=120000))
            got[m["request_id"]] = m["output_ids"]
        assert master.failover(1000) == []
        ps[dead].kill()
        ps[dead].join(timeout=30)
        dropped = master.failover(1000)
        assert [d.config_port for d in dropped] == [cfg_ports[dead]]
        assert master.mode == "chain" and len(master.plan.stages) == 3
        assert master.plan.stages[0].start == 0 and master.plan.stages[-1].end == 8
        t0 = time.time()
        while True:  # every survivor re-configured with its chain range
            st = dict((d.config_port, x) for d, x in master.health(1000))
            if all(x and x["configured"] and x["shards"] == [sg.start, sg.end] and x["pipeline_lost"]
                   for sg, x in ((sg, st[sg.device.config_port]) for sg in master.plan.stages)):
                break
            assert time.time() - t0 < 120, st
        master.submit(input_ids=[after])
        ing = master.plan.stages[0].device
        assert ing.config_port == cfg_ports[1 if dead == 0 else 0]
        done0 = len(before) if dead else 0  # the old ingress's pipeline outputs count there too
        t0 = time.time()
        while (ping_node(ing.host, ing.config_port, 1000) or {}).get("finished_requests", 0) < done0 + 1:
            assert time.time() - t0 < 120
            time.sleep(0.2)
        master.shutdown()
        for _ in range(world - 1):
            r, v = q.get(timeout=120)
            res[r] = v
    finally:
        reply.close()
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    alive = [r for r in range(world) if r != dead]
    chain_ing = alive[0]
    assert sorted(res) == alive and all(res[r] == "ok" for r in alive if r != chain_ing), res
    assert all(ps[r].exitcode == 0 for r in alive), [p.exitcode for p in ps]
    assert [got[i] for i in range(len(before))] == _golden(tiny8_shards, before, n_new)
    # the chain stage generates the controller's max_new_tokens (8) after the prompt
    chain_out = res[chain_ing][-1]
    assert chain_out == after + _golden(tiny8_shards, [after], 8)[0], chain_out
