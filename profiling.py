#!/usr/bin/env python3
"""Profile this device's compute capability (reference profiling.py). Assisted mode pairs
with assist_profiling.py on a second device for targets that cannot hold the whole model."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from llm_sharding_amd.utils.node_profiler import NodeProfiler  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", default="shards/Llama-2-7b-chat-hf_bfloat16")
    ap.add_argument("--device", default="cuda:0" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--max-layer-num", type=int, default=-1)
    ap.add_argument("--assisted", action="store_true")
    ap.add_argument("--src-addr", default="tcp://*:40800")
    ap.add_argument("--dst-addr", default="tcp://172.16.0.1:40800")
    ap.add_argument("--cold-start", action="store_true")
    ap.add_argument("--json-out", default="results/profiling/profile.json")
    a = ap.parse_args()
    p = NodeProfiler(a.shards, device=a.device, dtype=torch.bfloat16)
    res = p.profile_compute_capability(max_layer_num=a.max_layer_num, assisted=a.assisted,
                                       src_addr=a.src_addr, dst_addr=a.dst_addr)
    if a.cold_start:
        res["cold_start"] = p.profile_cold_start_latency(max_layer_num=a.max_layer_num)
    os.makedirs(os.path.dirname(a.json_out), exist_ok=True)
    with open(a.json_out, "w") as f:
        json.dump({k: v for k, v in res.items() if not k.endswith("_fit")}, f, indent=1, default=str)


if __name__ == "__main__":
    main()
