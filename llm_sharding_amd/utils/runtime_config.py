"""``RuntimeConfig``: one dataclass for every runtime knob (SURVEY.md §5.6 - the reference
hard-codes constructor arguments in scripts, ``start_node.py:13-20``, ``profiling.py:4-19``,
and takes only a port on the command line). Used by serve.py / the CLIs; serialisable to
JSON so a master can ship it to nodes next to the 6-key stage config."""
from __future__ import annotations

import argparse
import dataclasses
import json
from dataclasses import dataclass, fields
from typing import Optional

import torch

BACKENDS = ("tcp", "rccl", "local")


@dataclass
class RuntimeConfig:
    model: str = "llama2-7b"      # preset for random-init weights (when no shards are given)
    shards: str = ""              # shard folder (reference .pth layout / safetensors)
    device: str = ""              # "" = cuda:<LOCAL_RANK> if a GPU is visible, else cpu
    dtype: str = "bfloat16"
    backend: str = "rccl"         # stage hand-off: rccl (torch.distributed/RCCL), tcp, local
    batch: int = 32               # KV slots per micro-batch (0 = as many as HBM holds, <= 128)
    microbatches: int = 0         # 0 = max(2, pipeline stages)
    streams: int = 1              # one GPU: micro-batches on this many concurrent HIP streams
    max_seq: int = 2048
    prefill_budget: int = 2048    # prompt tokens per prefill command (longer prompts are chunked)
    max_new_tokens: int = 128
    use_graph: bool = True        # hipGraph-captured decode
    causal: bool = True           # False = the reference's unmasked prefill
    port: int = 40700             # ingress / config port
    seed: int = 0
    trace_dir: str = ""           # per-rank Chrome-trace timelines (LSA_TRACE)
    log_level: str = "INFO"

    def __post_init__(self):
        if self.backend not in BACKENDS:
            raise ValueError(f"backend must be one of {BACKENDS}, got {self.backend!r}")
        if self.batch < 0 or self.max_seq < 2 or self.prefill_budget < 1:
            raise ValueError("batch must be >= 0 (0 = auto), max_seq and prefill_budget positive")

    # ------------------------------------------------------------------ CLI
    @classmethod
    def add_arguments(cls, ap: argparse.ArgumentParser) -> argparse.ArgumentParser:
        for f in fields(cls):
            flag = "--" + f.name.replace("_", "-")
            if f.type in (bool, "bool"):
                if f.default:
                    ap.add_argument("--no-" + f.name.replace("_", "-"), dest=f.name, action="store_false",
                                    help=f"disable {f.name}")
                else:
                    ap.add_argument(flag, dest=f.name, action="store_true")
            else:
                typ = int if f.type in (int, "int") else str
                ap.add_argument(flag, dest=f.name, type=typ, default=f.default)
        return ap

    @classmethod
    def from_args(cls, ns: argparse.Namespace) -> "RuntimeConfig":
        return cls(**{f.name: getattr(ns, f.name) for f in fields(cls) if hasattr(ns, f.name)})

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self))

    @classmethod
    def from_json(cls, s: str) -> "RuntimeConfig":
        d = json.loads(s)
        return cls(**{k: v for k, v in d.items() if k in {f.name for f in fields(cls)}})

    # ------------------------------------------------------------------ resolution
    def torch_device(self, local_rank: int = 0) -> torch.device:
        if self.device:
            return torch.device(self.device)
        return torch.device("cuda", local_rank) if torch.cuda.is_available() else torch.device("cpu")

    def torch_dtype(self, device: Optional[torch.device] = None) -> torch.dtype:
        if device is not None and device.type == "cuda":
            return torch.bfloat16  # the HIP path computes in bf16
        return getattr(torch, self.dtype)

    def model_and_source(self):
        """(LlamaConfig, WeightSource) for the shards folder or the random-init preset."""
        from ..config import LlamaConfig, get_preset
        from ..runtime.engine import RandomSource, ShardFolderSource
        if self.shards:
            cfg = LlamaConfig.from_pretrained(self.shards)
            return cfg, ShardFolderSource(self.shards, cfg)
        cfg = get_preset(self.model)
        return cfg, RandomSource(cfg, self.seed)


__all__ = ["RuntimeConfig", "BACKENDS"]
