"""IPC ring transport (csrc/kernels/ipc_ring.hip, parallel/ipc_ring.py): two processes exchange
messages through rings mapped with HIP IPC - bursts filling every slot, byte-exact echoes,
hipGraph-captured send / receive replayed with fresh contents, and 8 KiB ping-pong - here both
ranks on one MI355X (the same kernels carry xGMI peer stores between GPUs)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_two(script, *extra):
    port = _port()
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "scripts", script), "--rank", str(r),
                               "--port", str(port), *extra], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True, env=env, cwd=ROOT) for r in range(2)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out))
    for rc, out in outs:
        assert rc == 0, out[-3000:]
    return [json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1]) for _, out in outs]


def test_ipc_ring_two_processes():
    res = _run_two("ipc_ring_check.py", "--world", "2")
    assert all(r["stream_ok"] and r["graph_ok"] and r["pingpong_ok"] for r in res), res
    # (both ranks time-share one GPU here, so this is not the xGMI latency between two GPUs)
    print("ipc ring one-way latency (us):", [r["one_way_us"] for r in res])


@pytest.mark.parametrize("streams", [1, 2])
def test_pipeline_over_ipc_ring(streams):
    """Two pipeline ranks handing hidden states / argmax keys over the IPC ring generate exactly
    the single-stage tokens (prefill, hipGraph decode with the hand-offs captured in the graphs,
    or concurrent micro-batch streams)."""
    res = _run_two("ipc_pipeline_check.py", "--streams", str(streams))
    assert all(r["ok"] for r in res), res
    if streams == 1:  # one compute stream: the hand-offs are captured inside the decode graphs
        assert all(r["captured_ops"] > 0 for r in res), res
