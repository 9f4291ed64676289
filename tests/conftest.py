import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "multigpu: needs >= 2 GPUs (skipped on a 1-GPU box); run after the rest")


def _has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    # multi-GPU cases last: under -x a failure there cannot hide the single-GPU results
    items.sort(key=lambda it: "multigpu" in it.keywords)  # stable: the rest keep their order
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def tiny_shards(tmp_path_factory):
    """A random-init tiny model written in the reference shard format."""
    from llm_sharding_amd.config import tiny
    from llm_sharding_amd.models.weights import write_random_shards
    import torch
    d = tmp_path_factory.mktemp("shards")
    return write_random_shards(tiny(), str(d / "tiny-llama"), dtype=torch.float32, seed=3)


@pytest.fixture(scope="session")
def tiny_shards_bf16(tmp_path_factory):
    from llm_sharding_amd.config import tiny
    from llm_sharding_amd.models.weights import write_random_shards
    import torch
    d = tmp_path_factory.mktemp("shards_bf16")
    return write_random_shards(tiny(), str(d / "tiny-llama"), dtype=torch.bfloat16, seed=5)
