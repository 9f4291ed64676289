#!/usr/bin/env python3
"""The micro-batched pipeline with the IPC ring as its stage hand-off (parallel/ipc_ring.py):
two ranks (processes) of a tiny Llama, here both on one GPU, prefill + hipGraph decode (one
stream: the hand-offs captured inside the decode graphs; several: micro-batches on concurrent
streams with the ring kernels launched between replays); rank 0 checks the generated ids token-exact against the
same model run as a single stage in-process.

    python scripts/ipc_pipeline_check.py --rank R --port P [--streams S]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=20.0)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank, world_size=2)
    torch.cuda.set_device(a.device)
    dev = torch.device("cuda", a.device)
    from llm_sharding_amd.config import tiny
    from llm_sharding_amd.parallel.ipc_ring import IpcRingP2P
    from llm_sharding_amd.parallel.pipeline import LocalP2P, run_pipeline_generate
    from llm_sharding_amd.runtime.engine import RandomSource
    cfg = tiny(layers=8)
    src = RandomSource(cfg, seed=21)
    prompts = torch.randint(3, cfg.vocab_size, (3, 4, 9), generator=torch.Generator().manual_seed(5))
    p2p = IpcRingP2P(a.rank, slot_bytes=4 * 9 * cfg.hidden_size * 2, slots=4, timeout_s=a.timeout)
    print(f"[rank {a.rank}] ipc ring up", flush=True)
    kw = dict(device=dev, batch=4, microbatches=3, max_seq=64, dtype=torch.bfloat16)
    out = run_pipeline_generate(cfg, src, prompts if a.rank == 0 else None, 10, a.rank, 2, streams=a.streams, p2p=p2p,
                                **kw)
    torch.cuda.synchronize()
    print(f"[rank {a.rank}] pipeline done", flush=True)
    p2p.check()
    res = {"rank": a.rank, "ok": True, "captured_ops": p2p.captured_ops}
    if a.rank == 0:
        # (a single stage sends nothing; LocalP2P keeps DistP2P's collective group setup out of it)
        single = run_pipeline_generate(cfg, src, prompts, 10, 0, 1, p2p=LocalP2P().bind(0), **kw)
        res["ok"] = out.tolist() == single.tolist()
        res["tokens"] = out[:3, 0].tolist()
    p2p.close()
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()
    sys.exit(0 if res["ok"] else 1)


if __name__ == "__main__":
    main()
