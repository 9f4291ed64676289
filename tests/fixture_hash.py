"""Hash of everything that decides the numerics of the HIP decode path: the kernel sources, the
measured tuning / route tables and the Python code that routes shapes to kernels. Recorded with
tests/fixtures/full_depth_7b.json; tests/test_fixture_fresh.py compares it with the tree."""
import glob
import hashlib
import os
import re

NUMERICS_FILES = ("csrc/kernels/*.hip", "csrc/kernels/*.h", "llm_sharding_amd/ops/*.json", "llm_sharding_amd/ops/hip.py",
                  "llm_sharding_amd/ops/packing.py", "llm_sharding_amd/runtime/engine.py")
FLAGS_RE = re.compile(r"hip_flags = \[[^\]]*\]", re.S)  # csrc/build.py's compile flags (not its comments)


def tree_hash(root: str) -> str:
    h = hashlib.sha256()
    for pat in NUMERICS_FILES:
        for p in sorted(glob.glob(os.path.join(root, pat))):
            h.update(os.path.relpath(p, root).encode())
            with open(p, "rb") as fh:
                h.update(fh.read())
    with open(os.path.join(root, "csrc", "build.py")) as fh:
        h.update(FLAGS_RE.search(fh.read()).group(0).encode())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    # After a change that the GPU run of tests/test_full_depth_gpu.py confirmed numerically neutral
    # (fingerprint unchanged vs the recording), re-stamp the fixture with the tree's hash:
    #   python tests/fixture_hash.py --update
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fx_path = os.path.join(root, "tests", "fixtures", "full_depth_7b.json")
    with open(fx_path) as fh:
        fx = json.load(fh)
    print(f"fixture {fx['kernel_hash']}  tree {tree_hash(root)}")
    if "--update" in sys.argv:
        fx["kernel_hash"] = tree_hash(root)
        with open(fx_path, "w") as fh:
            json.dump(fx, fh, indent=1)
