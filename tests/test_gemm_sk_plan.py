"""gemm_sk's work-decomposition planner (ops/hip.py gemm_sk_plan): measured winners from
ops/gemm_sk_tuning.json (scripts/tune_gemm_sk.py) for tuned shapes, the cost model elsewhere;
every plan is one the kernel accepts (N tiles by bn, one workgroup per CU)."""
from llm_sharding_amd.ops import hip


def test_tuned_shapes_use_the_table():
    tab = hip._sk_tuned()
    assert tab, "ops/gemm_sk_tuning.json missing or empty"
    for (N, K), rows in tab.items():
        for M, cfg in rows:
            assert hip.gemm_sk_plan(M, N, K) == (cfg[0], hip.N_CU, cfg[2], cfg[3], cfg[4] if len(cfg) > 4 else 256)


def test_nearest_measured_m_with_same_row_tiles():
    tab = hip._sk_tuned()
    rows = dict(tab[(4096, 4096)])
    # 500 rows -> four 128-row tiles: the M=512 entry, never the M=384 or M=640 one
    got = hip.gemm_sk_plan(500, 4096, 4096)
    want = rows[512]
    assert got == (want[0], hip.N_CU, want[2], want[3], want[4] if len(want) > 4 else 256)


def test_cost_model_for_untuned_shapes():
    for M, N, K in [(65536, 12288, 4096), (300, 5120, 3072), (4096, 128, 64)]:
        bn, grid, dp, split, bm = hip.gemm_sk_plan(M, N, K)
        assert bn in (128, 192, 256) and N % (16 if bn == 192 else bn) == 0 and grid == hip.N_CU and split >= 0
        assert bm in (128, 256)
        assert hip.gemm_sk_plan(M, N, K, tuned=False) == (bn, grid, dp, split, bm) or (N, K) in hip._sk_tuned()


def test_gemm_wr_route(monkeypatch):
    """hip.gemm sends a projection to gemm_wr.hip only where it measured faster than gemm_sk in the
    engine: one round of 192-256 whole 128 x 192 tiles with a store / QKV epilogue, for the measured
    (N, K) pairs only (the 7B qkv projection at 320-512 rows); everything else, and LSA_GEMM_WR=0,
    stays on gemm_sk."""
    monkeypatch.delenv("LSA_GEMM_WR", raising=False)
    ep = hip.EpiArgs()
    assert hip.gemm_wr_plan(512, 12288, 4096, hip.EPI_QKV, ep) == 192
    assert hip.gemm_wr_plan(448, 12288, 4096, hip.EPI_STORE, ep) == 192
    assert hip.gemm_wr_plan(384, 12288, 4096, hip.EPI_QKV, ep) == 192  # 3 row tiles: 192 tiles
    assert hip.gemm_wr_plan(447, 12288, 4096, hip.EPI_STORE, ep) is None  # last row tile < half full
    assert hip.gemm_wr_plan(319, 12288, 4096, hip.EPI_STORE, ep) is None  # last row tile < half full
    for M, N, K, epi in [(256, 12288, 4096, hip.EPI_QKV),   # 2 row tiles: 128 tiles
                         (513, 12288, 4096, hip.EPI_QKV),   # 5 row tiles: 320 tiles
                         (512, 12288, 4096, hip.EPI_SWIGLU),
                         (512, 4096, 4096, hip.EPI_RESID),
                         (384, 15360, 5120, hip.EPI_QKV),   # 13B qkv: tiles by 192, never measured
                         (1024, 6144, 4096, hip.EPI_QKV),   # 224 tiles, never measured
                         (512, 22016, 4096, hip.EPI_SWIGLU),
                         (512, 12288, 4160, hip.EPI_QKV)]:  # K % 256 != 0
        assert hip.gemm_wr_plan(M, N, K, epi, ep) is None, (M, N, K, epi)
    monkeypatch.setenv("LSA_GEMM_WR", "0")
    assert hip.gemm_wr_plan(512, 12288, 4096, hip.EPI_QKV, ep) is None
