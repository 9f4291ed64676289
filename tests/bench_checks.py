"""Checks on bench.py's JSON line shared by the CPU rehearsal (tests/test_bench_cli.py, gloo) and
the real multi-GPU runs (tests/test_multigpu_gpu.py, RCCL / IPC)."""


def check_placement(line: dict, n: int, kind: str, distinct: bool = True) -> None:
    """N ranks, N distinct devices (unless a one-GPU rehearsal), one ``kind`` edge per ring hop."""
    d = line["dist"]
    assert d["world_size"] == n and len(d["ranks"]) == n, d
    if distinct:
        assert d["distinct_devices"] is True and not d["shared_gpu_rehearsal"], d
        assert len({(r["host"], r["pci_bus_id"], r["uuid"]) for r in d["ranks"]}) == n, d["ranks"]
    ring = {f"{i}->{(i + 1) % n}" for i in range(n)}
    assert {k for k in d["edges"] if "->" in k} == ring, d["edges"]
    assert all(d["edges"][e] == kind for e in ring), d["edges"]
