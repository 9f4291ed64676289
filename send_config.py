#!/usr/bin/env python3
"""Master side (reference send_config.py): plan the layer placement with the scheduler and
push the configs to the NodeControllers started by run_this.sh, then optionally submit a
request. The reference hard-codes a 3-host chain; here hosts/ports are arguments.

    python send_config.py --shards DIR --nodes 127.0.0.1:40700:40800,127.0.0.1:40701:40801 \
        [--request "Write a poem about the blue sky."]

    # RCCL deployment on one 8-GPU node: controllers are the ranks of one torchrun job
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29500 \
        start_node.py --backend rccl --port 40700 --shards DIR          # rank r on port 40700 + r
    python send_config.py --shards DIR --pipeline --gpus 8 --batch 64 --request "..." --wait
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from llm_sharding_amd.parallel.scheduler import DeviceSpec  # noqa: E402
from llm_sharding_amd.utils.master_node import MasterNode  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", default="shards/Llama-2-7b-chat-hf_bfloat16")
    ap.add_argument("--nodes", default="127.0.0.1:40700:40800,127.0.0.1:40701:40801,"
                                       "127.0.0.1:40702:40802,127.0.0.1:40703:40803",
                    help="host:config_port:data_port[:mem_GB[:speed]] comma-separated, chain order")
    ap.add_argument("--request", default="")
    ap.add_argument("--kv-tokens", type=int, default=4096)
    ap.add_argument("--pipeline", action="store_true",
                    help="deploy the micro-batched RCCL pipeline on the ranks of a torchrun job of "
                         "start_node.py --backend rccl (node i = rank i)")
    ap.add_argument("--gpus", type=int, default=0, help="--pipeline: ranks on 127.0.0.1:<base port + i> "
                                                       "(instead of --nodes)")
    ap.add_argument("--base-port", type=int, default=40700)
    ap.add_argument("--batch", type=int, default=8, help="--pipeline: KV slots per micro-batch")
    ap.add_argument("--microbatches", type=int, default=0)
    ap.add_argument("--max-seq", type=int, default=2048)
    ap.add_argument("--max-new-tokens", type=int, default=128)
    ap.add_argument("--wait", action="store_true", help="wait for the request's output, then shut down")
    a = ap.parse_args()
    if a.pipeline and a.gpus:
        a.nodes = ",".join(f"127.0.0.1:{a.base_port + i}:{a.base_port + 100 + i}" for i in range(a.gpus))
    devs = []
    for n in a.nodes.split(","):
        parts = n.split(":")
        d = DeviceSpec(host=parts[0], config_port=int(parts[1]), data_port=int(parts[2]))
        if len(parts) > 3:
            d.mem_bytes = float(parts[3]) * 1e9
        if len(parts) > 4:
            d.speed = float(parts[4])
        devs.append(d)
    master = MasterNode.from_shards(a.shards, devs, kv_tokens=a.kv_tokens)
    if a.pipeline:
        for c in master.deploy_pipeline(batch=a.batch, microbatches=a.microbatches, max_seq=a.max_seq):
            print("[MASTER] sent", c)
        print("[MASTER] plan:", master.plan.summary())
    else:
        plan = master.make_plan()
        print("[MASTER] plan:", plan.summary())
        for c in master.deploy():
            print("[MASTER] sent", c)
    if a.request:
        reply = None
        if a.wait:
            from llm_sharding_amd.parallel.transport import PullSocket
            reply = PullSocket("tcp://127.0.0.1:0")
        master.submit(a.request, max_new_tokens=a.max_new_tokens,
                      reply_to=f"tcp://127.0.0.1:{reply.port}" if reply is not None else None)
        print("[MASTER] request submitted to the ingress node")
        if reply is not None:
            from llm_sharding_amd.parallel import protocol
            out = protocol.decode(reply.recv_bytes(timeout_ms=600000))
            print("[MASTER] output:", out.get("text") or out.get("output_ids"))
            reply.close()
            master.shutdown()


if __name__ == "__main__":
    main()
