#!/usr/bin/env python3
"""Start one NodeController (reference start_node.py): wait for a config from the master on
tcp://*:<port>, load the assigned layer range, serve the chain until shut down.

    python start_node.py [--port 40700 | 40700] [--shards DIR] [--device cuda:0] [--dtype bfloat16]

    # one node, one controller per GPU, stage hand-off over RCCL (xGMI) instead of TCP:
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29500 \
        start_node.py --backend rccl --port 40700 --shards DIR      # rank r listens on 40700 + r
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from llm_sharding_amd.utils.node_worker import NodeController  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("port_pos", nargs="?", type=int, default=None)
    ap.add_argument("--port", type=int, default=40700)
    ap.add_argument("--shards", default="shards/Llama-2-7b-chat-hf_bfloat16")
    ap.add_argument("--device", default="cuda:0" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--max-new-tokens", type=int, default=512)
    ap.add_argument("--noncausal-prefill", action="store_true", help="reference-compatible unmasked prefill")
    ap.add_argument("--backend", default="tcp", choices=("tcp", "rccl"),
                    help="stage hand-off: tcp (reference-compatible) or rccl (torchrun, one rank per GPU)")
    a = ap.parse_args()
    port = a.port_pos if a.port_pos is not None else a.port
    device = a.device
    if a.backend == "rccl":
        import torch.distributed as dist
        rank, local = int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
        if torch.cuda.is_available():
            device = f"cuda:{local}"
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device(device))
        else:
            dist.init_process_group("gloo")
        from llm_sharding_amd.parallel.communicator import init_edge_groups
        init_edge_groups()  # collective: one RCCL communicator per directed stage edge
        port += rank
    ctrl = NodeController(a.shards, device=device, dtype=getattr(torch, a.dtype), listen_port=port,
                          backend=a.backend, worker_kwargs={"noncausal_prefill": a.noncausal_prefill})
    ctrl.run_worker_loop(max_new_tokens=a.max_new_tokens)
    ctrl.close()


if __name__ == "__main__":
    main()
