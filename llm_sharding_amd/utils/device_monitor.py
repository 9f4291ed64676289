"""Device monitoring for MI355X nodes - the counterpart of the reference's Jetson tooling
(``/root/reference/cmds/install-jetson_stats.sh:1-3`` installs ``jtop`` to watch the edge
devices that run the shards).

``sample()`` returns one record per visible GPU (busy %, VRAM %, power, temperature) from
``rocm-smi --json`` (shipped with ROCm), plus the HIP runtime's own free/total memory when
torch can see the device; ``monitor()`` appends such records as JSON lines, e.g. next to a
running node:  ``python -m llm_sharding_amd.utils.device_monitor --interval 1 --out gpus.jsonl``.
"""
from __future__ import annotations

import argparse
import json
import shutil
import subprocess
import sys
import time
from typing import Optional

ROCM_SMI_ARGS = ["--showuse", "--showmemuse", "--showpower", "--showtemp", "--json"]


def _num(v) -> Optional[float]:
    try:
        return float(str(v).strip().rstrip("%").split()[0])
    except (ValueError, IndexError):
        return None


def parse_rocm_smi(text: str) -> list:
    """rocm-smi --json -> [{"card": i, "busy_pct", "vram_pct", "power_w", "temp_c"}]. Keys are
    matched loosely (their exact wording differs between ROCm releases)."""
    data = json.loads(text) if text.strip() else {}
    out = []
    for card, fields in sorted(data.items()):
        if not card.startswith("card") or not isinstance(fields, dict):
            continue
        rec = {"card": int(card[4:]) if card[4:].isdigit() else card}
        for k, v in fields.items():
            kl = k.lower()
            if "gpu use" in kl and "%" in kl:
                rec["busy_pct"] = _num(v)
            elif "vram" in kl and "%" in kl:
                rec["vram_pct"] = _num(v)
            elif "power" in kl and "(w)" in kl:
                rec.setdefault("power_w", _num(v))
            elif "temperature" in kl and ("edge" in kl or "junction" in kl or "hotspot" in kl):
                rec.setdefault("temp_c", _num(v))
        out.append(rec)
    return out


def sample() -> dict:
    """One snapshot of every visible GPU."""
    rec: dict = {"ts": time.time(), "gpus": []}
    smi = shutil.which("rocm-smi") or "/opt/rocm/bin/rocm-smi"
    try:
        r = subprocess.run([smi, *ROCM_SMI_ARGS], capture_output=True, text=True, timeout=20)
        if r.returncode == 0:
            rec["gpus"] = parse_rocm_smi(r.stdout)
        else:
            rec["error"] = r.stderr.strip()[-200:]
    except (OSError, subprocess.TimeoutExpired, json.JSONDecodeError) as e:
        rec["error"] = str(e)
    try:
        import torch
        if torch.cuda.is_available():
            rec["hip_mem"] = []
            for i in range(torch.cuda.device_count()):
                free, total = torch.cuda.mem_get_info(i)
                rec["hip_mem"].append({"device": i, "free_gb": round(free / 1e9, 2),
                                       "total_gb": round(total / 1e9, 2)})
    except Exception as e:  # noqa: BLE001 - monitoring must never take the node down
        rec["hip_mem_error"] = str(e)
    return rec


def monitor(interval: float = 1.0, count: int = 0, out: Optional[str] = None) -> None:
    f = open(out, "a") if out else sys.stdout
    try:
        n = 0
        while count <= 0 or n < count:
            f.write(json.dumps(sample()) + "\n")
            f.flush()
            n += 1
            if count <= 0 or n < count:
                time.sleep(interval)
    finally:
        if out:
            f.close()


def main() -> None:
    ap = argparse.ArgumentParser(description="sample MI355X busy / VRAM / power / temperature")
    ap.add_argument("--interval", type=float, default=1.0)
    ap.add_argument("--count", type=int, default=0, help="0 = until interrupted")
    ap.add_argument("--out", default="", help="append JSON lines here (default stdout)")
    a = ap.parse_args()
    monitor(a.interval, a.count, a.out or None)


if __name__ == "__main__":
    main()
