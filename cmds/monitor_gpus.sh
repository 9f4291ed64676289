#!/bin/bash
# Watch the node's MI355X GPUs while shards run (the reference installs jtop for its Jetson
# devices: /root/reference/cmds/install-jetson_stats.sh). Usage: cmds/monitor_gpus.sh [interval_s] [out.jsonl]
cd "$(dirname "$0")/.."
python3 -m llm_sharding_amd.utils.device_monitor --interval "${1:-1}" ${2:+--out "$2"}
