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


def test_route_table_and_fallback():
    """ops/routes.py: one table keyed by (N, K, row range); anything unlisted falls back to the
    GEMV family up to 128 rows and to gemm_sk above."""
    from llm_sharding_amd.ops import routes
    assert routes.route(512, 12288, 4096, routes.EPI_QKV).kernel == "gemm_wr"
    assert routes.route(512, 12288, 4096, routes.EPI_QKV).params == {"bn": 192}
    assert routes.route(512, 12288, 4096, routes.EPI_RESID).kernel == "gemm_sk"  # epilogue not on gemm_wr
    assert routes.route(100, 5120, 13824).kernel == "gemm_sk"                       # 13B mid batch
    # an unknown model shape: the fallback rule
    assert routes.route(1, 7168, 2048).kernel == "gemv"
    assert routes.route(128, 7168, 2048).kernel == "gemv"
    assert routes.route(129, 7168, 2048).kernel == "gemm_sk"
    assert routes.route(4096, 12288, 4096, routes.EPI_QKV).kernel == "gemm_sk"
    for r in routes.ROUTES:
        assert r.kernel in ("gemm_wr", "gemm_sk", "gemv") and 1 <= r.lo <= r.hi and r.evidence, r
        if r.kernel == "gemm_wr":
            assert r.params["bn"] in (128, 192, 256) and r.N % r.params["bn"] == 0, r
    # no two entries of one shape overlap in rows
    by = {}
    for r in routes.ROUTES:
        for q in by.get((r.N, r.K), []):
            assert r.hi < q.lo or q.hi < r.lo or set(r.epis).isdisjoint(q.epis or (0, 1, 2, 3)), (r, q)
        by.setdefault((r.N, r.K), []).append(r)
    # the layer decision: one family per layer
    shapes13 = StageEngine.proj_shapes(get_preset("llama2-13b"))
    assert routes.layer_family(64, shapes13) == "gemv" and routes.layer_family(65, shapes13) == "gemm"
    assert routes.gemv_max_rows(StageEngine.proj_shapes(get_preset("llama2-7b"))) == 128
