#!/bin/bash
# Start NUM_NODES NodeControllers (reference run_this.sh): config ports 40700+i, one process
# per node, node i on GPU (i mod NUM_GPUS). Logs: node_<port>.log
# Usage: ./run_this.sh [NUM_NODES] [SHARDS_DIR]
export PYTHONUNBUFFERED=1
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
NUM_NODES=${1:-4}
SHARDS=${2:-shards/Llama-2-7b-chat-hf_bfloat16}
BASE_PORT=40700
NUM_GPUS=$(python3 -c "import torch; print(max(torch.cuda.device_count(), 1))" 2>/dev/null || echo 1)
for ((i=0; i<NUM_NODES; i++)); do
    PORT=$((BASE_PORT + i))
    DEV="cuda:$((i % NUM_GPUS))"
    python3 -c "import torch; exit(0 if torch.cuda.is_available() else 1)" 2>/dev/null || DEV=cpu
    echo "Starting node $i on port $PORT ($DEV)..."
    python3 start_node.py --port "$PORT" --shards "$SHARDS" --device "$DEV" > "node_${PORT}.log" 2>&1 &
    echo $! >> .node_pids
    sleep 1
done
echo "All $NUM_NODES nodes started (ports $BASE_PORT to $((BASE_PORT + NUM_NODES - 1)))."
echo 'Logs: node_<port>.log. Stop: python3 -c "from llm_sharding_amd.utils.node_worker import send_shutdown; [send_shutdown(\"127.0.0.1\", 40700+i) for i in range(N)]"'
