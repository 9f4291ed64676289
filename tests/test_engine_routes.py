"""Model-shape routes of the decode path (CPU: the rule only, no weights loaded)."""
import torch

from llm_sharding_amd.config import get_preset
from llm_sharding_amd.runtime.engine import StageEngine


def test_mid_batch_gemm_route_by_model_shape(monkeypatch):
    """65-128-row decode steps go to the MFMA GEMMs only for the shapes measured faster there
    (Llama-2-13B: profiles/r5_gemv_max_rows_ab.md); LSA_GEMV_MAX_ROWS overrides the table."""
    monkeypatch.delenv("LSA_GEMV_MAX_ROWS", raising=False)
    for name, want in (("llama2-13b", 64), ("llama2-7b", StageEngine.GEMV_MAX_ROWS),
                       ("llama3.2-3b", StageEngine.GEMV_MAX_ROWS), ("llama2-70b", StageEngine.GEMV_MAX_ROWS)):
        eng = StageEngine(get_preset(name), 0, 1, "cpu", torch.float32, load=False)
        assert eng.GEMV_MAX_ROWS == want, name
    monkeypatch.setenv("LSA_GEMV_MAX_ROWS", "128")
    eng = StageEngine(get_preset("llama2-13b"), 0, 1, "cpu", torch.float32, load=False)
    assert eng.GEMV_MAX_ROWS == StageEngine.GEMV_MAX_ROWS
