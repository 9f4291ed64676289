"""The shared error metric of every GPU kernel test (llm_sharding_amd/utils/numerics.py), with the
negative controls that a single global Frobenius error misses (no GPU needed)."""
import torch

from llm_sharding_amd.utils.numerics import LOCAL_FACTOR, assert_close, rel_err


def _gemm_like(M=512, N=12288, seed=0):
    """An fp32 'reference' and its bf16-rounded copy: what a correct bf16-output GEMM returns."""
    g = torch.Generator().manual_seed(seed)
    ref = torch.randn(M, N, generator=g) * 3.0
    out = ref.to(torch.bfloat16).float()
    return out, ref


def test_correct_output_passes_with_margin():
    out, ref = _gemm_like()
    e = rel_err(out, ref)
    assert e < 8e-3
    # the local gate has room: the worst of 24,576 tiles / 512 rows of a correctly rounded output
    # sits well inside LOCAL_FACTOR x the global error
    assert e.tile < 2.0 * e.global_ and e.row < 1.5 * e.global_, e
    assert e.local < LOCAL_FACTOR * 8e-3


def test_zeroed_tile_is_caught():
    out, ref = _gemm_like()
    bad = out.clone()
    bad[256:272, 4096:4112] = 0.0  # one 16 x 16 output tile never written (stream-K fix-up bug)
    e = rel_err(bad, ref)
    # the old metric alone would have passed it ...
    assert e.global_ < 8e-3, e
    # ... the shared one does not, and it names the tile
    assert not (e < 8e-3)
    assert e.tile_at == (256 // 16, 4096 // 16) and e.tile > 0.9, e


def test_misaligned_zero_tile_is_caught():
    out, ref = _gemm_like(seed=1)
    bad = out.clone()
    bad[100:116, 1000:1016] = 0.0  # straddles four 16 x 16 tiles of the check grid
    assert not (rel_err(bad, ref) < 8e-3)


def test_wrong_row_is_caught():
    out, ref = _gemm_like(M=1024, N=4096, seed=2)
    bad = out.clone()
    bad[777] *= 1.05  # one row 5 % off (a GEMV split-K hand-off reading a stale partial)
    e = rel_err(bad, ref)
    assert e.global_ < 8e-3, e
    assert not (e < 8e-3)
    assert e.row_at == 777, e


def test_zero_reference_regions_do_not_blow_up():
    out, ref = _gemm_like(M=64, N=256)
    ref[:16] = 0.0
    out[:16] = 0.0
    e = rel_err(out, ref)
    assert e < 8e-3, e


def test_nan_fails():
    out, ref = _gemm_like(M=32, N=64)
    out[3, 5] = float("nan")
    assert not (rel_err(out, ref) < 1.0)


def test_assert_close_message_names_location():
    out, ref = _gemm_like(M=64, N=256)
    out[16:32, 32:48] = 0.0
    try:
        assert_close(out, ref, 8e-3, "gemm")
    except AssertionError as ex:
        assert "tile (1, 2)" in str(ex), str(ex)
    else:
        raise AssertionError("assert_close missed a zeroed tile")


def test_vectors_and_3d():
    g = torch.Generator().manual_seed(4)
    ref = torch.randn(8, 4, 128, generator=g)
    out = ref.to(torch.bfloat16).float()
    assert rel_err(out, ref) < 8e-3
    out[5, 2] = 0.0  # one (row, head) vector lost
    assert not (rel_err(out, ref) < 8e-3)
    v = torch.randn(1000, generator=g)
    assert rel_err(v.to(torch.bfloat16).float(), v) < 8e-3
