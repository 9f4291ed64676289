"""bench.py on one MI355X: the JSON line's placement block ("dist") names the device the rank
really ran on - its PCI address / UUID from the HIP runtime - so the same keys on an 8-GPU run
prove 8 distinct GPUs. A short run of a 2-layer cut of the 7B (stage profile)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_line_names_the_device():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--batch", "16",
                        "--prompt-len", "8", "--stage-layers", "2", "--latency-steps", "0", "--mid-batch", "0",
                        "--ttft-lens", "", "--extras", ""], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    d = line["dist"]
    assert d["world_size"] == 1 and len(d["ranks"]) == 1 and d["edges"] == {}
    rk = d["ranks"][0]
    import torch
    p = torch.cuda.get_device_properties(0)
    print(f"[bench-gpu] rank 0 on {rk}, torch reports uuid={p.uuid} pci={p.pci_domain_id}:{p.pci_bus_id}:{p.pci_device_id}")
    assert rk["device_index"] == 0
    assert rk["pci_bus_id"] and rk["pci_bus_id"] != "0000:00:00" or str(rk["uuid"]).strip("0-"), rk
    assert d["distinct_devices"] is True
