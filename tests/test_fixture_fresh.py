"""The full-depth tripwire's recording (tests/fixtures/full_depth_7b.json, read by
tests/test_full_depth_gpu.py) must belong to this tree: a change of any kernel, tuning table or
routing code needs a new recording on the GPU box (LSA_RECORD_FULL_DEPTH=1), so a stale fixture
fails here, on the CPU, before it can fail - or mask a regression - on the GPU."""
import json
import os

from fixture_hash import tree_hash

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "full_depth_7b.json")


def test_full_depth_fixture_matches_tree():
    with open(FIXTURE) as fh:
        fx = json.load(fh)
    assert {"small_batch", "big_batch"} <= set(fx), sorted(fx)
    assert fx["kernel_hash"] == tree_hash(ROOT), (
        f"tests/fixtures/full_depth_7b.json was recorded at {fx.get('commit')} for kernel hash {fx['kernel_hash']}, "
        f"the tree is {tree_hash(ROOT)}: re-record with LSA_RECORD_FULL_DEPTH=1 python -m pytest "
        f"tests/test_full_depth_gpu.py on the GPU box")
    for k in ("small_batch", "big_batch"):
        r = fx[k]
        assert len(r["steps"]) + 1 == len(r["fingerprint"]) and r["tokens"] > 0
