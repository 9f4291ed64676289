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


def test_bench_cli_two_ranks_match_one_and_prove_placement():
    """The CPU rehearsal of tests/test_multigpu_gpu.py: the same placement checks and the same
    token comparison, over gloo (every rank its own process, so its own "device")."""
    from bench_checks import check_placement
    one = _run_bench("--gpus", "1", "--model", "tiny", *COMMON)
    two = _run_bench("--gpus", "2", "--model", "tiny", *COMMON)
    check_placement(two, 2, "gloo")
    assert two["tokens_mb0_sha16"] == one["tokens_mb0_sha16"]


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


def _bench_env(**extra):
    env = dict(os.environ, OMP_NUM_THREADS="1", **extra)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    return env


def test_bench_preflight_reports_edges():
    """The ring-edge preflight (one small message per directed edge before the weights load)
    runs on every multi-rank run and its per-edge latencies reach the JSON line."""
    line = _run_bench("--gpus", "3", "--model", "tiny", *COMMON)
    assert line["transport"] == "rccl" and line["fallback"] is False
    assert sorted(line["preflight_us"]) == ["0->1", "1->2", "2->0"], line["preflight_us"]
    assert all(v > 0 for v in line["preflight_us"].values())


def test_bench_dead_edge_fails_fast_and_falls_back_once():
    """An injected dead edge (rank 1 never sends on 1 -> 2): rank 2's preflight names the edge
    and exits 75 within LSA_PREFLIGHT_TIMEOUT_S; the per-rank supervisors (which never touched a
    device) stop the other workers and start every rank ONCE more in a fresh process with
    --transport ipc; that run produces the number, marked ``"fallback": true``."""
    import time
    env = _bench_env(LSA_PREFLIGHT_FAULT="1->2", LSA_PREFLIGHT_TIMEOUT_S="5")
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "3",
                        "--model", "tiny", *COMMON], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "PREFLIGHT FAILED on rank 2: edge 1->2 (receive)" in r.stderr, r.stderr[-3000:]
    assert "restarting every rank once with --transport ipc" in r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["fallback"] is True and line["transport"] == "ipc" and line["value"] > 0
    assert time.time() - t0 < 200


def test_bench_dead_edge_without_fallback_exits_nonzero():
    env = _bench_env(LSA_PREFLIGHT_FAULT="0->1", LSA_PREFLIGHT_TIMEOUT_S="5")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2",
                        "--model", "tiny", "--no-fallback", *COMMON], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 75, (r.returncode, r.stderr[-3000:])
    assert "PREFLIGHT FAILED on rank 1: edge 0->1 (receive)" in r.stderr
    assert not any(l.startswith("{") for l in r.stdout.splitlines())


def test_bench_under_torchrun_supervised():
    """The driver's launch form: torch.distributed.run starts the ranks (its agent hosts the
    rendezvous store); the supervisors' workers rendezvous on their own port."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--device", "cpu",
                        "--gpus", "2", "--model", "tiny", *COMMON], cwd=ROOT, env=_bench_env(),
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["fallback"] is False and sorted(line["preflight_us"]) == ["0->1", "1->0"]


@pytest.mark.parametrize("how", ["sigterm-launcher", "sigkill-supervisor"])
def test_bench_workers_do_not_outlive_their_supervisor(how):
    """Killing the launcher (SIGTERM, as a driver timeout or a launcher's killpg would) or a
    per-rank supervisor outright (SIGKILL: no handler runs) leaves no worker behind: the
    supervisors forward termination to their workers' process groups, and every child dies with
    its parent (PR_SET_PDEATHSIG) - the workers run in their own sessions, so nothing else would
    reach them (advisor round 4)."""
    import signal
    import time

    import psutil
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2",
                          "--model", "tiny", "--steps", "100000", "--warmup", "1", "--batch", "2",
                          "--prompt-len", "4", "--latency-steps", "2"], cwd=ROOT, env=_bench_env(),
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        deadline = time.time() + 120
        workers = []
        while time.time() < deadline:
            kids = psutil.Process(p.pid).children(recursive=True)
            workers = [k for k in kids if _is_worker(k)]
            if len(workers) == 2:
                break
            time.sleep(0.5)
        assert len(workers) == 2, "the two bench workers did not start"
        if how == "sigterm-launcher":
            p.send_signal(signal.SIGTERM)
        else:
            workers[0].parent().kill()  # rank's supervisor, SIGKILL
        gone, alive = psutil.wait_procs(workers, timeout=60)
        assert not alive, f"workers outlived their supervisor: {[w.pid for w in alive]}"
    finally:
        for k in psutil.Process(p.pid).children(recursive=True) if p.poll() is None else []:
            k.kill()
        p.kill()
        p.wait()


def _is_worker(proc) -> bool:
    try:
        return proc.environ().get("LSA_BENCH_ROLE") == "worker"
    except Exception:  # noqa: BLE001 - exited meanwhile
        return False
