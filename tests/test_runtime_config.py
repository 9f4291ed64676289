"""RuntimeConfig CLI/JSON round trip and the prefixed / JSON logger."""
import argparse
import json

import pytest

from llm_sharding_amd.utils.log import get_logger
from llm_sharding_amd.utils.runtime_config import RuntimeConfig


def test_cli_roundtrip():
    ap = RuntimeConfig.add_arguments(argparse.ArgumentParser())
    rc = RuntimeConfig.from_args(ap.parse_args(["--batch", "8", "--no-use-graph", "--no-causal", "--model", "tiny",
                                                "--backend", "tcp", "--max-seq", "64"]))
    assert (rc.batch, rc.use_graph, rc.causal, rc.backend, rc.max_seq) == (8, False, False, "tcp", 64)
    assert RuntimeConfig.from_json(rc.to_json()) == rc
    cfg, src = rc.model_and_source()
    assert cfg.num_hidden_layers == 4 and src.layer(0, "cpu", __import__("torch").float32)
    with pytest.raises(ValueError):
        RuntimeConfig(backend="zmq")


def test_logger_prefix_and_json(capsys, monkeypatch):
    log = get_logger("t")
    log.info("hello", stage=1)
    log.debug("hidden")
    assert capsys.readouterr().out.strip() == "[INFO] hello stage=1"
    monkeypatch.setenv("LSA_LOG_JSON", "1")
    monkeypatch.setenv("LSA_LOG_LEVEL", "DEBUG")
    log.debug("x", k=2)
    rec = json.loads(capsys.readouterr().out)
    assert rec["level"] == "DEBUG" and rec["msg"] == "x" and rec["k"] == 2 and rec["logger"] == "t"


def test_every_lsa_knob_is_listed():
    """utils/runtime_config.KNOBS names every LSA_* environment variable the code reads and every
    LSA_* compile define the kernels test (one list, product vs diagnostic)."""
    import glob
    import os
    import re
    from llm_sharding_amd.utils.runtime_config import KNOBS
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env, defines = set(), set()
    pys = glob.glob(os.path.join(root, "llm_sharding_amd", "**", "*.py"), recursive=True) + \
        [os.path.join(root, f) for f in ("bench.py", "serve.py", "start_node.py", "__graft_entry__.py")] + \
        glob.glob(os.path.join(root, "tests", "*.py"))
    for p in pys:
        env |= set(re.findall(r"environ(?:\.get)?[\(\[]\s*[\"'](LSA_[A-Z0-9_]+)", open(p).read()))
        env |= set(re.findall(r"(LSA_[A-Z0-9_]+)=str\(", open(p).read()))
    for p in glob.glob(os.path.join(root, "csrc", "kernels", "*")):
        defines |= set(re.findall(r"#\s*if(?:n?def)?\s+(LSA_[A-Z0-9_]+)", open(p).read()))
    for sh in glob.glob(os.path.join(root, "scripts", "probes", "*.sh")):
        env |= set(re.findall(r"\$\{(LSA_[A-Z0-9_]+)", open(sh).read()))
    missing = sorted((env | defines) - set(KNOBS))
    assert not missing, f"LSA_* knobs not listed in runtime_config.KNOBS: {missing}"
    for k in defines:
        assert KNOBS[k][0] == "define", k
    assert all(v[1] in ("product", "diagnostic", "test") for v in KNOBS.values())
