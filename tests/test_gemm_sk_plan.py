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
    """hip.gemm sends a qkv projection to gemm_wr.hip only inside its measured row ranges
    (hip.WR_ROUTES); everything else, and LSA_GEMM_WR=0, stays on gemm_sk."""
    monkeypatch.delenv("LSA_GEMM_WR", raising=False)
    ep = hip.EpiArgs()
    assert hip.gemm_wr_plan(512, 12288, 4096, hip.EPI_QKV, ep) == 192
    assert hip.gemm_wr_plan(448, 12288, 4096, hip.EPI_STORE, ep) == 192
    assert hip.gemm_wr_plan(384, 12288, 4096, hip.EPI_QKV, ep) == 192
    assert hip.gemm_wr_plan(384, 15360, 5120, hip.EPI_QKV, ep) == 192   # 13B
    assert hip.gemm_wr_plan(512, 15360, 5120, hip.EPI_QKV, ep) == 256
    assert hip.gemm_wr_plan(512, 5120, 3072, hip.EPI_QKV, ep) == 128    # 3B
    assert hip.gemm_wr_plan(512, 16384, 3072, hip.EPI_SWIGLU, ep) == 256  # 3B gate_up
    assert hip.gemm_wr_plan(447, 12288, 4096, hip.EPI_STORE, ep) is None  # last row tile < half full
    assert hip.gemm_wr_plan(319, 12288, 4096, hip.EPI_STORE, ep) is None
    assert hip.gemm_wr_plan(256, 12288, 4096, hip.EPI_QKV, ep) == 128   # 2 row tiles
    assert hip.gemm_wr_plan(256, 16384, 3072, hip.EPI_SWIGLU, ep) == 128
    for M, N, K, epi in [(192, 12288, 4096, hip.EPI_QKV),   # below the measured range
                         (513, 12288, 4096, hip.EPI_QKV),   # above it
                         (512, 12288, 4096, hip.EPI_SWIGLU),
                         (512, 4096, 4096, hip.EPI_RESID),
                         (384, 10240, 8192, hip.EPI_QKV),   # 70B qkv: measured a tie, not routed
                         (1024, 6144, 4096, hip.EPI_QKV),   # never measured
                         (512, 22016, 4096, hip.EPI_SWIGLU),
                         (128, 5120, 3072, hip.EPI_QKV),    # 3B below its range
                         (512, 12288, 4160, hip.EPI_QKV)]:  # another K
        assert hip.gemm_wr_plan(M, N, K, epi, ep) is None, (M, N, K, epi)
    monkeypatch.setenv("LSA_GEMM_WR", "0")
    assert hip.gemm_wr_plan(512, 12288, 4096, hip.EPI_QKV, ep) is None
