#!/usr/bin/env python3
"""Reference-API chain path (NodeWorker, the reference's node_worker.py:227-309 loop) on one GPU:
per-token decode time of a whole-model stage with the hipGraph decode replay against eager
kernel launches. Random-init weights of the named model (no checkpoint), batch 1, one ingress +
head node, no network hop (pass_through_shard -> receive_next_token in-process).

usage: chain_graph_bench.py [--model llama2-7b] [--tokens 64] [--prompt 32]
One JSON line per mode on stdout."""
import argparse
import json
import os
import socket
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llm_sharding_amd.config import get_preset  # noqa: E402
from llm_sharding_amd.runtime.engine import RandomSource  # noqa: E402
from llm_sharding_amd.utils.node_worker import NodeWorker  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--tokens", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=32)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    cfg = get_preset(a.model)
    d = tempfile.mkdtemp()
    cfg.save_pretrained(d)
    socks = [socket.socket() for _ in range(2)]
    for s in socks:
        s.bind(("127.0.0.1", 0))
    ports = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    w = NodeWorker(f"tcp://*:{ports[0]}", f"tcp://127.0.0.1:{ports[1]}", True, d, device=a.device, dtype=torch.bfloat16,
                   max_batch=1, max_seq=a.prompt + a.tokens + 8, source=RandomSource(cfg), verbose=False)
    w.load_shards(0, cfg.num_hidden_layers)
    prompt = torch.randint(0, cfg.vocab_size, (1, a.prompt))
    res = {}
    for mode in ("graph", "eager", "graph"):
        w.use_graph = mode == "graph"
        w.clear_KV_cache()
        st = w.receive_user_request(input_ids=prompt)
        times = []
        for i in range(a.tokens):
            if a.device == "cuda":
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            tok = w.pass_through_shard(st)  # host sync: the token goes back over the wire
            end, st = w.receive_next_token(tok, max_new_tokens=a.tokens + 1)
            times.append(time.perf_counter() - t0)
        toks = w.output_ids()[0, a.prompt:].tolist()
        dec = sorted(times[1:])  # [0] is the prefill
        res[mode] = toks
        print(json.dumps({"model": a.model, "mode": mode, "tokens": a.tokens, "prefill_ms": round(times[0] * 1e3, 2),
                          "p50_tpot_ms": round(dec[len(dec) // 2] * 1e3, 3),
                          "p90_tpot_ms": round(dec[int(len(dec) * 0.9)] * 1e3, 3),
                          "tokens_sha": hash(tuple(toks)) & 0xffffffff}), flush=True)
    print(json.dumps({"graph_tokens_equal_eager": res["graph"] == res["eager"]}))
    w.close()


if __name__ == "__main__":
    main()
