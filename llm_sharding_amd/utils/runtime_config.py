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


# Every LSA_* switch in the package, kernels and entry points, in one place.
# kind: "env" (read at run time) or "define" (a -D compile flag of csrc/kernels, never set by
# csrc/build.py: only probe builds under probe_bin/ use them). role: "product" (changes what a
# deployment runs or how it reports), "diagnostic" (A/B and ablation switches; the default is the
# shipped behaviour, measured in the profile named), "test" (test harness only).
# tests/test_runtime_config.py::test_every_lsa_knob_is_listed keeps this table complete.
KNOBS = {
    # ---- product
    "LSA_LOG_LEVEL": ("env", "product", "INFO", "log level of utils/log.py"),
    "LSA_LOG_JSON": ("env", "product", "", "1 = JSON log lines"),
    "LSA_TRACE": ("env", "product", "", "directory for per-rank Chrome-trace timelines (bench --trace, serve)"),
    "LSA_DIST_TIMEOUT_S": ("env", "product", "300", "torch.distributed collective timeout of the pipeline"),
    "LSA_STARTUP_TIMEOUT_S": ("env", "product", "180", "RCCL bring-up watchdog (exit PREFLIGHT_EXIT when exceeded)"),
    "LSA_PREFLIGHT_TIMEOUT_S": ("env", "product", "30", "per-edge receive timeout of the ring preflight"),
    "LSA_IPC_TIMEOUT_S": ("env", "product", "30", "bounded spin of an IPC-ring hand-off before it poisons"),
    "LSA_IPC_ALLOC": ("env", "product", "uncached", "IPC ring buffer kind: uncached | fine (coarse is refused across GPUs)"),
    "LSA_PP_STREAMS": ("env", "product", "1", "pipeline: concurrent micro-batch streams per stage"),
    "LSA_GRAPH_COMM": ("env", "product", "1", "capture IPC-ring hand-offs inside the decode hipGraph"),
    "LSA_BENCH_ROLE": ("env", "product", "", "set by bench.py's supervisor for its worker process"),
    "LSA_BENCH_FALLBACK": ("env", "product", "", "set by bench.py when it restarted on --transport ipc"),
    "LSA_PARENT_PID": ("env", "product", "", "set by bench.py for its children (PR_SET_PDEATHSIG check)"),
    # ---- diagnostic (A/B switches; defaults = the shipped routes)
    "LSA_KERNELS_SO": ("env", "diagnostic", "_native/liblsa_kernels.so", "load another build of the kernel library"),
    "LSA_GEMV_MAX_ROWS": ("env", "diagnostic", "128 (64 for MID_GEMM_SHAPES)",
                          "rows up to which decode projections stay on the GEMVs (profiles/r5_gemv_max_rows_ab.md)"),
    "LSA_GEMM_WR": ("env", "diagnostic", "1", "0 = no gemm_wr routes (profiles/r4_gemm_wr_engine_ab.txt)"),
    "LSA_ATTN_MIN_CHUNK": ("env", "diagnostic", "256", "shortest split-KV chunk in keys"),
    "LSA_ATTN_MFMA": ("env", "diagnostic", "1", "0 = no MFMA GQA decode kernel"),
    "LSA_ATTN_MFMA_MIN_ITEMS": ("env", "diagnostic", "512", "rows x kv-heads from which GQA decode uses MFMA"),
    "LSA_ATTN_GQA_NW": ("env", "diagnostic", "0", "waves of the GQA decode kernel (0 = planner)"),
    "LSA_ATTN_SMALL_MAX_WGS": ("env", "diagnostic", "", "grid size limit of the small-grid decode attention"),
    "LSA_ATTN_OPROJ": ("env", "diagnostic", "0", "1 = batch-1 attention + o projection in one launch (profiles/r6_attn_oproj.md)"),
    "LSA_AO_ABLATE": ("define", "diagnostic", "0", "attn_oproj ablation builds (scripts/probes/build_attn_oproj_ab.sh)"),
    "LSA_PREFLIGHT_FAULT": ("env", "diagnostic", "", "fault injection: 'a->b' drops the preflight message of edge a->b"),
    "LSA_SK_ABLATE": ("define", "diagnostic", "0", "gemm_sk ablation builds (scripts/sk_ablate.py)"),
    "LSA_COOP_ABLATE": ("define", "diagnostic", "0", "coop GEMV ablation builds"),
    "LSA_GEMM_SK_TUNING": ("env", "diagnostic", "", "path of a gemm_sk tuning table to use instead of ops/gemm_sk_tuning.json (A/B runs)"),
    "LSA_GEMV_TUNING": ("env", "diagnostic", "", "path of a decode-GEMV tuning table to use instead of ops/gemv_tuning.json (A/B runs)"),
    "LSA_STREAM_ABLATE": ("define", "diagnostic", "0", "gemv_stream probe ablation builds (scripts/probes/build_gemv_stream.sh)"),
    "LSA_GEMM_STAMPS": ("define", "diagnostic", "", "gemm_sk per-phase s_memrealtime stamps"),
    "LSA_COOP_STAMPS": ("define", "diagnostic", "", "coop GEMV per-phase stamps"),
    # ---- tests
    "LSA_RECORD_FULL_DEPTH": ("env", "test", "", "1 = record tests/fixtures/full_depth_7b.json instead of checking it"),
    "LSA_FULL_DEPTH_FIXTURE": ("env", "test", "tests/fixtures/full_depth_7b.json", "where the full-depth fixture lives"),
    "LSA_VARIANT_SLP": ("env", "diagnostic", "", "scripts/probes/build_kernels_variant.sh: build with SLP on"),
}


def knobs_in_effect() -> dict:
    """The run-time knobs set in this process's environment (for logs / bench lines)."""
    import os
    return {k: os.environ[k] for k, v in KNOBS.items() if v[0] == "env" and k in os.environ}


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
