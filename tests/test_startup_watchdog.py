"""The RCCL startup watchdog of the bench (parallel/pipeline._startup_watchdog): a rank stuck in
the process-group setup exits with PREFLIGHT_EXIT and says why; a cancelled watchdog does nothing."""
import subprocess
import sys
import textwrap

from llm_sharding_amd.parallel.pipeline import PREFLIGHT_EXIT


def _run(code: str):
    return subprocess.run([sys.executable, "-c", textwrap.dedent(code)], capture_output=True, text=True, timeout=60)


def test_startup_watchdog_fires_with_preflight_exit():
    r = _run("""
        import time
        from llm_sharding_amd.parallel.pipeline import _startup_watchdog
        _startup_watchdog(3, timeout_s=0.3)
        time.sleep(30)  # a setup that never returns
    """)
    assert r.returncode == PREFLIGHT_EXIT, (r.returncode, r.stderr)
    assert "PREFLIGHT FAILED on rank 3" in r.stderr and "process-group setup" in r.stderr


def test_startup_watchdog_cancelled_is_silent():
    r = _run("""
        import time
        from llm_sharding_amd.parallel.pipeline import _startup_watchdog
        wd = _startup_watchdog(0, timeout_s=0.3)
        wd.cancel()
        time.sleep(0.6)
    """)
    assert r.returncode == 0 and "PREFLIGHT" not in r.stderr


def test_preflight_edge_that_raises_exits_with_preflight_code():
    """An RCCL edge that FAILS fast (isend / irecv / wait raises) is treated like one that hangs:
    the rank names the edge and exits PREFLIGHT_EXIT (so the supervisor can fall back), the
    watchdog is cancelled (advisor round 4)."""
    r = _run("""
        import torch
        from llm_sharding_amd.parallel.pipeline import preflight_edges

        class Work:
            def wait(self):
                raise RuntimeError("NCCL error: remote process exited")

        class FakeP2P:
            def _global(self, s):
                return s
            def isend(self, t, dst):
                return Work()
            def irecv(self, t, src):
                return Work()

        preflight_edges(FakeP2P(), 1, 3, torch.device("cpu"), timeout_s=30)
        print("returned")
    """)
    assert r.returncode == PREFLIGHT_EXIT, (r.returncode, r.stderr)
    assert "PREFLIGHT FAILED on rank 1: edge 0->1 (receive) and 1->2 (send) raised RuntimeError" in r.stderr, r.stderr
    assert "returned" not in r.stdout
