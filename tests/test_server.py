"""Continuous-batching PipelineServer on CPU: single process and multi-process gloo pipelines
(the same code that runs over RCCL on GPUs) must produce the golden model's greedy tokens for
every request, with more requests than KV slots (slot reuse), prompts longer than the prefill
budget (chunked prefill) and EOS stops."""
import multiprocessing as mp
import socket

import pytest
import torch

from llm_sharding_amd.config import tiny
from llm_sharding_amd.models import weights as W
from llm_sharding_amd.models.reference import ReferenceLlama
from llm_sharding_amd.parallel.scheduler import plan_stages
from llm_sharding_amd.parallel.server import PipelineServer
from llm_sharding_amd.runtime.engine import RandomSource

SEED, NEW, B, M = 11, 6, 2, 2


def _cfg():
    return tiny(layers=4)


def _prompts(cfg):
    g = torch.Generator().manual_seed(5)
    lens = [3, 9, 40, 1, 17, 6, 25]
    return [torch.randint(3, cfg.vocab_size, (n,), generator=g).tolist() for n in lens]


def _golden(cfg, prompts, n):
    dt = torch.float32
    ref = ReferenceLlama(cfg, W.random_embedding(cfg, dt, seed=SEED),
                         [W.random_layer(cfg, i, dt, seed=SEED) for i in range(cfg.num_hidden_layers)],
                         W.random_final_norm(cfg, dt, seed=SEED), W.random_lm_head(cfg, dt, seed=SEED), max_pos=128)
    return [ref.generate(torch.tensor([p]), n)[0].tolist() for p in prompts]


@pytest.fixture(scope="module")
def golden():
    cfg = _cfg()
    return _golden(cfg, _prompts(cfg), NEW)


def _server(cfg, rank=0, world=1, ctrl=None):
    plan = plan_stages(cfg, world)
    st = plan.stages[rank]
    return PipelineServer(cfg, RandomSource(cfg, SEED), rank, world, st.start, st.end, device="cpu",
                          batch=B, microbatches=M, max_seq=128, prefill_budget=16, dtype=torch.float32,
                          ctrl_group=ctrl)


def test_single_process_matches_golden(golden):
    cfg = _cfg()
    srv = _server(cfg)
    outs = srv.generate(_prompts(cfg), NEW, eos_ids=())
    assert outs == golden
    st = srv.stats()
    assert st["requests"] == len(golden) and st["tokens"] == len(golden) * NEW


def test_eos_stops_and_frees_slot(golden):
    cfg = _cfg()
    srv = _server(cfg)
    prompts = _prompts(cfg)
    eos = golden[2][2]  # the 3rd token of request 2
    outs = srv.generate(prompts, NEW, eos_ids=(eos,))
    for o, g in zip(outs, golden):
        want = g[:g.index(eos) + 1] if eos in g else g
        assert o == want


def test_streaming_callback_and_incremental_submit(golden):
    cfg = _cfg()
    srv = _server(cfg)
    prompts = _prompts(cfg)
    seen = {}
    rids = [srv.submit(p, NEW, eos_ids=(), on_token=lambda r, t: seen.setdefault(r.rid, []).append(t))
            for p in prompts[:3]]
    srv.serve(stop_when_idle=True)
    assert [seen[r] for r in rids] == golden[:3]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ctrl = dist.new_group(backend="gloo")
        cfg = _cfg()
        srv = _server(cfg, rank, world, ctrl)
        if rank == 0:
            q.put(srv.generate(_prompts(cfg), NEW, eos_ids=()))
        else:
            srv.serve()
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_multiprocess_server_matches_golden(world, golden):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = q.get(timeout=240)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    assert res == golden


@pytest.mark.slow
def test_serve_cli_tcp_ingress(tmp_path):
    """serve.py (world 1, CPU): a reference-style user_request with reply_to over the native
    TCP transport comes back with the golden tokens; shutdown stops the server."""
    import json
    import os
    import subprocess
    import sys
    import time
    from llm_sharding_amd.config import get_preset
    from llm_sharding_amd.parallel import protocol
    from llm_sharding_amd.parallel.transport import PullSocket, PushSocket
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = _free_port()
    log = open(tmp_path / "serve.log", "w")
    env = dict(os.environ, PYTHONUNBUFFERED="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    p = subprocess.Popen([sys.executable, os.path.join(root, "serve.py"), "--random", "tiny", "--port", str(port),
                          "--batch", "2", "--max-seq", "128", "--max-new-tokens", "5"],
                         stdout=log, stderr=subprocess.STDOUT, env=env)
    reply = PullSocket("tcp://127.0.0.1:0")
    try:
        t0 = time.time()
        while "ingress listening" not in (tmp_path / "serve.log").read_text():
            assert p.poll() is None and time.time() - t0 < 120, (tmp_path / "serve.log").read_text()
            time.sleep(0.2)
        prompt = [1, 50, 60, 70, 80]
        s = PushSocket(f"tcp://127.0.0.1:{port}")
        s.send_bytes(json.dumps({"command": "user_request", "input_ids": [prompt], "max_new_tokens": 5,
                                 "reply_to": f"tcp://127.0.0.1:{reply.port}"}).encode())
        s.flush(5000)
        msg = protocol.decode(reply.recv_bytes(timeout_ms=120000))
        cfg = get_preset("tiny")
        dt = torch.float32
        ref = ReferenceLlama(cfg, W.random_embedding(cfg, dt, seed=0),
                             [W.random_layer(cfg, i, dt, seed=0) for i in range(cfg.num_hidden_layers)],
                             W.random_final_norm(cfg, dt, seed=0), W.random_lm_head(cfg, dt, seed=0), max_pos=128)
        want = ref.generate(torch.tensor([prompt]), 5)[0].tolist()
        eos = set(cfg.eos_ids)
        if any(t in eos for t in want):
            want = want[:next(i for i, t in enumerate(want) if t in eos) + 1]
        assert msg["output_ids"] == want
        s.send_bytes(json.dumps({"command": "shutdown"}).encode())
        s.close()
        assert p.wait(timeout=60) == 0
    finally:
        reply.close()
        if p.poll() is None:
            p.kill()
        log.close()
