#!/usr/bin/env python3
"""Continuous-batching server over the layer-sharded pipeline, one process per GPU.

    # 8 MI355X, Llama-2-7B shards (or --random for random-init weights of that architecture)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29500 \\
        serve.py --shards shards/Llama-2-7b-chat-hf_bfloat16 --port 40700
    # client (any host): reference-style user_request message on the ingress port
    python -c "from llm_sharding_amd.utils.node_worker import send_user_request; \\
               send_user_request('127.0.0.1', 40700, text='Write a poem about the blue sky.')"

    # self-contained load test: N synthetic requests, prints a JSON stats line and exits
    python serve.py --model llama2-7b --requests 256 --prompt-len 128 --max-new-tokens 128

All runtime knobs are RuntimeConfig fields (``--batch --microbatches --max-seq --prefill-budget
--no-use-graph --no-causal --trace-dir --log-level ...``).

Rank 0 (embedding stage) is the ingress: it accepts ``{"command": "user_request", "text" |
"input_ids", "max_new_tokens", "reply_to"}`` messages (the reference's control-port JSON /
our LSAM framing, see ``utils/node_worker.send_user_request``) on ``--port``, streams every
finished request to stdout and, if ``reply_to`` is given, pushes ``{"request_id",
"output_ids", "text", "ttft_ms", "tpot_ms"}`` back to that address. ``{"command":
"shutdown"}`` drains the queue and stops every rank.
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from llm_sharding_amd.parallel.scheduler import plan_stages  # noqa: E402
from llm_sharding_amd.parallel.server import PipelineServer  # noqa: E402
from llm_sharding_amd.utils.log import get_logger  # noqa: E402
from llm_sharding_amd.utils.runtime_config import RuntimeConfig  # noqa: E402


def _ingress(srv, port, tok, stop_evt, default_new):
    from llm_sharding_amd.parallel.ingress import Replies, run_ingress
    from llm_sharding_amd.parallel.transport import PullSocket
    sock = PullSocket(f"tcp://*:{port}")
    print(f"[INFO] ingress listening on tcp://*:{sock.port}", flush=True)
    replies = Replies(tok)
    try:
        run_ingress(srv, sock, tok, stop_evt, default_new, replies)
    finally:
        sock.close()
        replies.close()


def main():
    ap = argparse.ArgumentParser(description="continuous-batching pipeline server (one process per GPU)")
    RuntimeConfig.add_arguments(ap)
    ap.add_argument("--random", default="", help="alias of --model: random-init weights of a preset")
    ap.add_argument("--requests", type=int, default=0, help="synthetic load test: N requests, then exit")
    ap.add_argument("--prompt-len", type=int, default=128)
    a = ap.parse_args()
    if a.random:
        a.model = a.random
    rc = RuntimeConfig.from_args(a)
    if rc.trace_dir:
        os.environ["LSA_TRACE"] = rc.trace_dir
    os.environ.setdefault("LSA_LOG_LEVEL", rc.log_level)
    log = get_logger("serve")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = rc.torch_device(local)
    gpu = dev.type == "cuda"
    if gpu:
        torch.cuda.set_device(dev)
    ctrl = None
    if world > 1:
        import torch.distributed as dist
        if gpu:
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        ctrl = dist.new_group(backend="gloo")
    cfg, source = rc.model_and_source()
    M = rc.microbatches or max(2, world)
    if rc.batch == 0:  # size the KV cache from this GPU's HBM
        from llm_sharding_amd.parallel.scheduler import kv_slots_for_memory, scratch_bytes
        mem = torch.cuda.get_device_properties(dev).total_memory if gpu else 64e9
        # activations / workspaces of every concurrently replayed scratch set, plus 8 GB slack
        reserve = 8e9 + scratch_bytes(cfg, rc.prefill_budget, sets=max(1, rc.streams))
        plan = plan_stages(cfg, world)
        for _ in range(8):  # the KV budget moves layer boundaries: iterate to a fixed point
            rc.batch = min(kv_slots_for_memory(cfg, s.n_layers, rc.max_seq, mem, s.weight_bytes, reserve_bytes=reserve,
                                               microbatches=M) for s in plan.stages)
            nxt = plan_stages(cfg, world, kv_tokens=rc.max_seq * rc.batch * M)
            if nxt.ranges() == plan.ranges():
                break
            plan = nxt
        log.info(f"KV cache sized from {mem / 1e9:.0f} GB HBM: {rc.batch} slots x {M} micro-batches")
    plan = plan_stages(cfg, world, kv_tokens=rc.max_seq * rc.batch * M)
    st = plan.stages[rank]
    if rank == 0:
        log.info(f"{cfg.name}: {world} stage(s) {plan.ranges()}, {M} x {rc.batch} slots")
    srv = PipelineServer(cfg, source, rank, world, st.start, st.end, dev, batch=rc.batch, microbatches=M,
                         max_seq=rc.max_seq, prefill_budget=rc.prefill_budget, use_graph=rc.use_graph,
                         dtype=rc.torch_dtype(dev) if gpu else torch.float32, ctrl_group=ctrl, causal=rc.causal,
                         streams=rc.streams)
    if rank != 0:
        srv.serve()
    elif a.requests:
        g = torch.Generator().manual_seed(rc.seed + 1)
        for _ in range(a.requests):
            ids = torch.randint(3, cfg.vocab_size, (a.prompt_len,), generator=g).tolist()
            srv.submit(ids, rc.max_new_tokens, eos_ids=())
        t0 = time.perf_counter()
        srv.t_start = t0
        srv.serve(stop_when_idle=True)
        s = srv.stats()
        s.update({"metric": "serving_output_tokens_per_sec", "n_gpus": world, "model": cfg.name,
                  "requests": a.requests, "prompt_len": a.prompt_len, "max_new_tokens": rc.max_new_tokens,
                  "slots": rc.batch * M, "microbatches": M})
        print(json.dumps(s), flush=True)
    else:
        tok = None
        try:
            from llm_sharding_amd.models.tokenizer import load_tokenizer
            tok = load_tokenizer(rc.shards) if rc.shards else None
        except Exception as e:  # noqa: BLE001
            log.warning(f"no tokenizer: {e}")
        stop_evt = threading.Event()
        th = threading.Thread(target=_ingress, args=(srv, rc.port, tok, stop_evt, rc.max_new_tokens), daemon=True)
        th.start()
        srv.serve(stop_when_idle=False, should_stop=stop_evt.is_set)
        th.join(timeout=5)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
