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
