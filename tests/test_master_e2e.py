"""Multi-process end-to-end (BASELINE.json config 1, plumbing): NodeControllers started as
separate processes with start_node.py, the master (send_config.py -> MasterNode: scheduler
plan + ConfigSender) deploys a 2-stage chain on localhost and submits a request; the ingress
node's output must equal the golden model's greedy tokens."""
import os
import re
import socket
import subprocess
import sys
import time

import pytest
import torch

from llm_sharding_amd.models import weights as W
from llm_sharding_amd.models.reference import ReferenceLlama
from llm_sharding_amd.parallel.scheduler import DeviceSpec, plan_stages
from llm_sharding_amd.utils.master_node import MasterNode
from llm_sharding_amd.utils.node_worker import send_shutdown

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_ports(n):
    socks = [socket.socket() for _ in range(n)]
    for s in socks:
        s.bind(("127.0.0.1", 0))
    ps = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    return ps


def test_master_plan_configs(tiny_shards):
    devs = [DeviceSpec(config_port=1000 + i, data_port=2000 + i) for i in range(3)]
    m = MasterNode.from_shards(tiny_shards, devs)
    cfgs = m.configs()
    assert [c["shards_start"] for c in cfgs] == [0, 1, 3] or cfgs[0]["shards_start"] == 0
    assert cfgs[-1]["shards_end"] == 4 and cfgs[0]["can_receive_user_request"]
    assert cfgs[-1]["dst_addr"].endswith(":2000") and cfgs[0]["first_node_addr"].endswith(":2000")
    # a slower device gets fewer layers
    devs[1].speed = 4.0
    p = plan_stages(m.cfg, devs)
    assert p.stages[1].n_layers == 1
    assert MasterNode.speed_from_profiles([{"prefill_c_k": 2.0}, {"decode_c_k": 1.0}]) == [2.0, 1.0]


@pytest.mark.slow
def test_two_node_processes_end_to_end(tiny_shards, tmp_path):
    cports = free_ports(2)
    dports = free_ports(2)
    env = dict(os.environ, PYTHONUNBUFFERED="1", PYTHONPATH=ROOT)
    logs = [open(tmp_path / f"node{i}.log", "w") for i in range(2)]
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "start_node.py"), "--port", str(cports[i]),
                               "--shards", tiny_shards, "--device", "cpu", "--dtype", "float32",
                               "--max-new-tokens", "6"], stdout=logs[i], stderr=subprocess.STDOUT, env=env)
             for i in range(2)]
    try:
        nodes = ",".join(f"127.0.0.1:{cports[i]}:{dports[i]}" for i in range(2))
        r = subprocess.run([sys.executable, os.path.join(ROOT, "send_config.py"), "--shards", tiny_shards,
                            "--nodes", nodes, "--request", "Why the sky blue"], env=env, capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert "plan:" in r.stdout
        log0 = tmp_path / "node0.log"
        t0 = time.time()
        while time.time() - t0 < 120 and "output token number" not in log0.read_text():
            time.sleep(0.2)
        text = log0.read_text()
        assert "output token number: 6" in text, text[-2000:]
    finally:
        for p in cports:
            send_shutdown("127.0.0.1", p)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        for f in logs:
            f.close()
    # compare with the golden model on the same prompt
    from llm_sharding_amd.models.tokenizer import load_tokenizer
    tok = load_tokenizer(tiny_shards)
    ids = tok("Why the sky blue", return_tensors="pt")["input_ids"]
    cfg, emb, layers, fn, lm = W.load_full_model(tiny_shards)
    want = ReferenceLlama(cfg, emb, layers, fn, lm).generate(ids, 6)[0].tolist()
    m = re.search(r"output:  ?(.*)", text)
    assert m and tok.decode(ids[0].tolist() + want) == m.group(1).rstrip("\n")


@pytest.mark.slow
def test_failure_detection_and_elastic_failover(tiny_shards, tmp_path):
    """3 controllers deployed by the master; one process dies; health() notices (no pong),
    failover() re-plans over the 2 survivors and hot re-configures them; a request then
    produces the golden tokens."""
    from llm_sharding_amd.utils.node_worker import ping_node
    cports, dports = free_ports(3), free_ports(3)
    env = dict(os.environ, PYTHONUNBUFFERED="1", PYTHONPATH=ROOT)
    logs = [open(tmp_path / f"node{i}.log", "w") for i in range(3)]
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "start_node.py"), "--port", str(cports[i]),
                               "--shards", tiny_shards, "--device", "cpu", "--dtype", "float32",
                               "--max-new-tokens", "5"], stdout=logs[i], stderr=subprocess.STDOUT, env=env)
             for i in range(3)]
    try:
        # liveness before configuration
        t0 = time.time()
        while any(ping_node("127.0.0.1", p, 500) is None for p in cports):
            assert time.time() - t0 < 120
        devs = [DeviceSpec(host="127.0.0.1", config_port=cports[i], data_port=dports[i]) for i in range(3)]
        m = MasterNode.from_shards(tiny_shards, devs)
        m.deploy()
        t0 = time.time()
        while not all((st or {}).get("configured") for _, st in m.health(1000)):
            assert time.time() - t0 < 120
        assert m.failover(1000) == []
        procs[1].kill()
        procs[1].wait(timeout=30)
        dropped = m.failover(1000)
        assert [d.config_port for d in dropped] == [cports[1]]
        assert len(m.plan.stages) == 2
        t0 = time.time()
        while True:
            st = dict((d.config_port, s) for d, s in m.health(1000))
            if all(s and s["configured"] and s["shards"] == [p.start, p.end]
                   for p, s in ((p, st[p.device.config_port]) for p in m.plan.stages)):
                break
            assert time.time() - t0 < 120
        m.submit(input_ids=[[1, 40, 41, 42]])
        log0 = tmp_path / "node0.log"
        t0 = time.time()
        while time.time() - t0 < 120 and "output token number" not in log0.read_text():
            time.sleep(0.2)
        text = log0.read_text()
        assert "output token number: 5" in text, text[-2000:]
    finally:
        for i, p in enumerate(cports):
            if procs[i].poll() is None:
                send_shutdown("127.0.0.1", p)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        for f in logs:
            f.close()
    cfg, emb, layers, fn, lm = W.load_full_model(tiny_shards)
    want = ReferenceLlama(cfg, emb, layers, fn, lm).generate(torch.tensor([[1, 40, 41, 42]]), 5)[0].tolist()
    from llm_sharding_amd.models.tokenizer import load_tokenizer
    tok = load_tokenizer(tiny_shards)
    m2 = re.search(r"output:  ?(.*)", text)
    assert m2 and tok.decode([1, 40, 41, 42] + want) == m2.group(1).rstrip("\n")
