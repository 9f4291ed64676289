"""llm_sharding_amd - an MI355X-native (gfx950 / CDNA4, ROCm) layer-sharded LLM inference engine.

Same capabilities and public API as seanbonjean/llm-sharding (master ``ConfigSender`` ->
``NodeController`` -> ``NodeWorker``; ``ModelSharder`` on-disk shard format; ``NodeProfiler``),
re-designed for MI355X: hand-written HIP kernels for the stage forward, a static KV cache,
hipGraph-captured decode steps and an RCCL (xGMI) pipeline between one process per GPU.

Package layout:
  models/    config-driven Llama decoder: golden fp32 reference, RoPE tables, shard IO, tokenizer
  ops/       HIP kernel bindings (ctypes -> _native/liblsa_kernels.so) and weight packing
  runtime/   StageEngine (per-stage weights/KV/forward) and DecodeGraph (hipGraph step)
  parallel/  transports (native TCP, in-process, RCCL), wire protocol, pipeline engine, scheduler
  utils/     reference-compatible API: node_worker, config_sender, model_sharder, node_profiler ...
"""
__version__ = "0.1.0"

from .config import LlamaConfig, get_preset  # noqa: F401
