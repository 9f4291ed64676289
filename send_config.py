#!/usr/bin/env python3
"""Master side (reference send_config.py): plan the layer placement with the scheduler and
push the configs to the NodeControllers started by run_this.sh, then optionally submit a
request. The reference hard-codes a 3-host chain; here hosts/ports are arguments.

    python send_config.py --shards DIR --nodes 127.0.0.1:40700:40800,127.0.0.1:40701:40801 \
        [--request "Write a poem about the blue sky."]
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
    a = ap.parse_args()
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
    plan = master.make_plan()
    print("[MASTER] plan:", plan.summary())
    for c in master.deploy():
        print("[MASTER] sent", c)
    if a.request:
        master.submit(a.request)
        print("[MASTER] request submitted to the ingress node")


if __name__ == "__main__":
    main()
