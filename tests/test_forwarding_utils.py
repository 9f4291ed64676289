"""C5 ``build_position_ids`` against the reference contract (/root/reference/utils/forwarding_utils.py:4-26):
positions continue after the cached length, for every ``past_key_value`` form the reference takes."""
import pytest
import torch

from llm_sharding_amd.utils.forwarding_utils import build_position_ids


def test_no_cache_starts_at_zero():
    p = build_position_ids(None, 5, "cpu")
    assert p.dtype == torch.long and p.shape == (1, 5)
    assert p.tolist() == [[0, 1, 2, 3, 4]]


def test_kv_tuple_uses_the_key_length():
    k = torch.zeros(2, 4, 7, 16)  # [B, n_kv, past, Hd]
    p = build_position_ids((k, k.clone()), 3, "cpu", batch_size=2)
    assert p.tolist() == [[7, 8, 9], [7, 8, 9]]
    assert p.is_contiguous()  # expanded rows are materialised, as in the reference


def test_object_with_get_seq_length():
    class Handle:
        def get_seq_length(self):
            return 11

    assert build_position_ids(Handle(), 1, "cpu").tolist() == [[11]]


def test_hf_dynamic_cache():
    transformers = pytest.importorskip("transformers")
    cache = transformers.DynamicCache()
    k = torch.zeros(1, 2, 9, 8)
    cache.update(k, k.clone(), 0)
    assert build_position_ids(cache, 2, "cpu").tolist() == [[9, 10]]


@pytest.mark.parametrize("bad", [[1, 2], (torch.zeros(1),), "cache"])
def test_unsupported_structure_raises(bad):
    with pytest.raises(ValueError, match=r"\[ERROR\] Unsupported past_key_value structure"):
        build_position_ids(bad, 1, "cpu")
