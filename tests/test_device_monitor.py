"""Device monitor parsing (rocm-smi JSON) and a CPU-side sample that never raises."""
import json

from llm_sharding_amd.utils.device_monitor import parse_rocm_smi, sample

SMI = {
    "card0": {"GPU use (%)": "87", "GPU Memory Allocated (VRAM%)": "41",
              "Current Socket Graphics Package Power (W)": "905.0", "Temperature (Sensor edge) (C)": "61.0"},
    "card1": {"GPU use (%)": "0", "GPU Memory Allocated (VRAM%)": "0"},
    "system": {"Driver version": "x"},
}


def test_parse_rocm_smi():
    recs = parse_rocm_smi(json.dumps(SMI))
    assert [r["card"] for r in recs] == [0, 1]
    assert recs[0] == {"card": 0, "busy_pct": 87.0, "vram_pct": 41.0, "power_w": 905.0, "temp_c": 61.0}
    assert recs[1]["busy_pct"] == 0.0 and "power_w" not in recs[1]


def test_sample_without_gpu_does_not_raise():
    rec = sample()
    assert "ts" in rec and isinstance(rec["gpus"], list)
