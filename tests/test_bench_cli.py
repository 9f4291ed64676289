"""bench.py as the driver runs it: ``python bench.py --gpus N ...`` with NO external launcher
(the script starts its N rank processes itself, like the reference's run_this.sh starts its
stage processes), here on gloo + the CPU path (``--device cpu``). The JSON line must carry the
whole-job metric, the batch-1 latency keys, and the 8-rank run must generate the same tokens as
one process."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(*args, timeout=300):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", *args], cwd=ROOT, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


COMMON = ["--steps", "3", "--warmup", "2", "--batch", "2", "--prompt-len", "4", "--latency-steps", "2"]


def test_bench_cli_single_rank():
    line = _run_bench("--gpus", "1", "--model", "tiny", *COMMON)
    assert line["n_gpus"] == 1 and line["steps"] == 3 and line["warmup"] == 2
    assert line["metric"] == "output_tokens_per_sec_whole_node" and line["value"] > 0
    assert line["config"]["parallelism"] == "pp1"
    assert line["b1_p50_tpot_ms"] > 0 and line["b1_tok_s"] > 0


@pytest.mark.parametrize("n", [2, 8])
def test_bench_cli_spawns_ranks(n):
    model = "tiny8" if n == 8 else "tiny"
    line = _run_bench("--gpus", str(n), "--model", model, *COMMON)
    assert line["n_gpus"] == n and line["config"]["parallelism"] == f"pp{n}"
    assert line["value"] > 0 and line["b1_p50_tpot_ms"] > 0
    assert line["config"]["microbatches"] == n  # bench default: one stream -> M = stages


def test_bench_cli_rank_failure_is_reported():
    """A failing rank must make the launcher exit non-zero (the driver must not see a number)."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2",
                        "--model", "no-such-model", *COMMON], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode != 0
    assert not any(l.startswith("{") for l in r.stdout.splitlines())
