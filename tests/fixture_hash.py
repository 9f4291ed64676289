"""Hash of everything that decides the numerics of the HIP decode path: the kernel sources, the
measured tuning / route tables and the Python code that routes shapes to kernels. Recorded with
tests/fixtures/full_depth_7b.json; tests/test_fixture_fresh.py compares it with the tree."""
import glob
import hashlib
import os

NUMERICS_FILES = ("csrc/kernels/*.hip", "csrc/kernels/*.h", "llm_sharding_amd/ops/*.json", "llm_sharding_amd/ops/hip.py",
                  "llm_sharding_amd/ops/packing.py", "llm_sharding_amd/runtime/engine.py", "csrc/build.py")


def tree_hash(root: str) -> str:
    h = hashlib.sha256()
    for pat in NUMERICS_FILES:
        for p in sorted(glob.glob(os.path.join(root, pat))):
            h.update(os.path.relpath(p, root).encode())
            with open(p, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]
