#!/usr/bin/env python3
"""Assistor side of the two-device profile (reference assist_profiling.py)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from llm_sharding_amd.utils.node_profiler import NodeProfiler  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", default="shards/Llama-2-7b-chat-hf_bfloat16")
    ap.add_argument("--device", default="cuda:0" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--target-max-layer-num", type=int, default=7)
    ap.add_argument("--src-addr", default="tcp://*:40800")
    ap.add_argument("--dst-addr", default="tcp://172.16.0.2:40800")
    a = ap.parse_args()
    NodeProfiler(a.shards, device=a.device, dtype=torch.bfloat16).assist_profile_compute_capability(
        target_max_layer_num=a.target_max_layer_num, src_addr=a.src_addr, dst_addr=a.dst_addr)


if __name__ == "__main__":
    main()
