"""Latency profiling and model fitting (reference C8, ``utils/node_profiler.py``).

Same class, constants and public methods:

* ``profile_max_layer_num()`` - layers (with the embedding) that fit before OOM (C8a). On a
  288 GB MI355X every supported model fits; ``memory_limit_bytes`` emulates a smaller device.
* ``_fit_latency_models(...)`` - least-squares ``T = aS + b`` and ``T = aS^2 + bS + c`` in
  fp64, RMSE / R^2, PNG plot under ``results/profiling/`` (C8b).
* ``_report_prefill_decode_similarity(...)`` - average c_k, linear slope and quadratic
  marginal cost comparison against a 30 % threshold (C8c).
* ``profile_compute_capability(max_layer_num, assisted, src_addr, dst_addr)`` - prefill at
  prompt lengths 8..512 x 3 repeats, cumulative decode latency up to 512 tokens, fits and
  similarity report (C8f); ``assisted=True`` + ``assist_profile_compute_capability`` on a
  second device for targets that cannot hold the whole model (C8g), with the reference's
  ``prefill_ack`` / ``decode_done`` commands over the Communicator.
* ``profile_cold_start_latency(max_layer_num)`` (C8h), ``go_through_every_shards`` (4-stage
  loopback chain, C8i), ``go_through_every_shards_only_by_profiler`` (no networking, C8j).

Every timing is host wall time bracketed by ``torch.cuda.synchronize`` (reference
``:300-308``). Results are also *returned* as dicts (the reference only prints), so the master
scheduler (``plan_stages`` layer costs / device speed factors) can consume them directly.

The scheduler's inputs should come from the path that is DEPLOYED, not from the reference-API
worker: :func:`profile_stage_costs` (``NodeProfiler.profile_pipeline_costs``) times the
pipeline's own hipGraph decode replays (hipEvents; ``DecodeGraph`` modes mid / first / full on
1 and n layers -> per-layer, embedding, head and per-stage fixed costs at a given batch and
context) plus the engine's prefill forward, and :func:`costs_for_planner` /
``MasterNode.deploy_pipeline(profiles=...)`` turn that into the planner's cost model
(reference: ``c_k`` feeds the master scheduler, ``/root/reference/README.md:7-8``,
``/root/reference/utils/node_profiler.py:822-979``).
Fixes: Q11 (``_resolve_assisted_target_loaded_layer_num(None)`` no longer computes ``None - 1``).
"""
from __future__ import annotations

import os
import time
from typing import Optional

import torch

from ..config import LlamaConfig
from ..models.tokenizer import load_tokenizer
from .node_worker import NodeWorker


def _timed_replays(step, n: int, gpu: bool) -> float:
    """Median-free mean ms per call of ``step`` over ``n`` back-to-back calls (device events on
    a GPU, so the host launch cost of a graph replay is not counted)."""
    if gpu:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            step()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        step()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def profile_stage_costs(cfg: LlamaConfig, source, device, batch: int = 1, context: int = 128,
                        n_layers: int = 4, prefill_len: int = 128, replays: int = 20,
                        dtype=torch.bfloat16) -> dict:
    """Cost model of the DEPLOYED stage engine (runtime/engine.py StageEngine + DecodeGraph):
    one engine with ``n_layers`` layers (+ embedding + lm_head) and ``batch`` sequences whose
    KV caches hold ``context`` tokens; decode steps are timed as the pipeline runs them
    (hipGraph replays, hipEvents; the eager step on CPU) in the modes a stage can have:

        mid(j)  = overhead + j * layer          (hidden in -> j layers -> hidden out)
        first(n) = mid(n) + embed               (token ids -> embedding -> layers)
        full(n)  = first(n) + head              (... -> final norm + lm_head + argmax)

    from j = 1 and j = n; prefill per layer from the engine's forward over ``prefill_len``
    tokens at 1 and n layers. Returns ms: ``layer_decode_ms``, ``embed_decode_ms``,
    ``head_decode_ms``, ``stage_overhead_ms``, ``layer_prefill_ms``, ``prefill_overhead_ms``
    plus the geometry."""
    from ..runtime.engine import DecodeGraph, EagerDecode, StageEngine
    dev = torch.device(device)
    gpu = dev.type == "cuda"
    n = max(2, min(int(n_layers), cfg.num_hidden_layers))
    max_seq = -(-(context + 4 * (replays + 4) + prefill_len + 8) // 64) * 64
    eng = StageEngine(cfg, 0, n, dev, dtype if gpu else torch.float32, has_embed=True, has_head=True,
                      source=source, max_slots=batch, max_seq=max_seq,
                      max_prefill_rows=max(prefill_len, batch))
    layers = eng.layers
    slots = list(range(batch))
    gen = torch.Generator().manual_seed(0)

    def decode_ms(mode: str, j: int) -> float:
        eng.layers = layers[:j]
        try:
            for s_ in slots:
                eng.seq_len[s_] = context
            if gpu:
                g = DecodeGraph(eng, batch, mode, slots=slots)
                g.tokens.copy_(torch.randint(3, cfg.vocab_size, (batch,), generator=gen).to(torch.int32))
                g.capture()
            else:
                g = EagerDecode(eng, batch, mode, slots=slots)
            for _ in range(3):
                g.replay()
            if gpu:
                torch.cuda.synchronize()
            return _timed_replays(g.replay, replays, gpu)
        finally:
            eng.layers = layers

    def prefill_ms(j: int) -> float:
        eng.layers = layers[:j]
        try:
            ids = torch.randint(3, cfg.vocab_size, (prefill_len,), generator=gen)

            def run():
                eng.reset([0])
                sl, po = eng.prefill_rows([0], [prefill_len])
                eng.forward(eng.embed(ids.to(dev)), sl, po)
            run()
            if gpu:
                torch.cuda.synchronize()
            return _timed_replays(run, max(3, replays // 4), gpu)
        finally:
            eng.layers = layers

    mid1, midn = decode_ms("mid", 1), decode_ms("mid", n)
    first_n, full_n = decode_ms("first", n), decode_ms("full", n)
    p1, pn = prefill_ms(1), prefill_ms(n)
    # per-layer cost from the 1- vs n-layer difference; a host whose speed drifted between the two
    # measurements can make that difference <= 0, and a zero layer cost would make the planner
    # treat layers as free: then the n-layer time split evenly over its layers (an upper bound)
    layer = (midn - mid1) / (n - 1)
    layer = layer if layer > 0 else midn / n
    lp = (pn - p1) / (n - 1)
    lp = lp if lp > 0 else pn / n
    out = {
        "batch": batch, "context": context, "profiled_layers": n, "prefill_len": prefill_len,
        "device": str(dev), "graph": gpu,
        "layer_decode_ms": layer,
        "stage_overhead_ms": max(0.0, mid1 - layer),
        "embed_decode_ms": max(0.0, first_n - midn),
        "head_decode_ms": max(0.0, full_n - first_n),
        "layer_prefill_ms": lp,
        "prefill_overhead_ms": max(0.0, p1 - lp),
        "decode_c_k": layer * cfg.num_hidden_layers / batch * 1e-3,  # s per token per whole model
    }
    del eng
    if gpu:
        torch.cuda.empty_cache()
    return out


def predict_stage_ms(prof: dict, n_layers: int, first: bool = False, last: bool = False,
                     head_frac: float = 1.0) -> float:
    """Decode step time of a stage of ``n_layers`` layers from :func:`profile_stage_costs`."""
    t = prof["stage_overhead_ms"] + n_layers * prof["layer_decode_ms"]
    if first:
        t += prof["embed_decode_ms"]
    if last:
        t += head_frac * prof["head_decode_ms"]
    return t


def costs_for_planner(cfg: LlamaConfig, prof: dict) -> dict:
    """``plan_stages`` keyword arguments from a stage-cost profile (ms per decode step)."""
    return {"layer_costs": [prof["layer_decode_ms"]] * cfg.num_hidden_layers,
            "embed_cost": prof["embed_decode_ms"], "head_cost": prof["head_decode_ms"],
            "stage_overhead": prof["stage_overhead_ms"]}


class NodeProfiler:
    PROFILE_INTERVAL_SLEEP_TIME = 1
    PROFILE_REPEAT_NUM = 3
    PROFILE_PREFILL_INPUT_TOKEN_LENGTHS = [8, 16, 32, 64, 128, 256, 512]
    PROFILE_DECODE_OUTPUT_TOKEN_LENGTHS = [8, 16, 32, 64, 128, 256, 512]
    PROFILE_PREFILL_PROMPT_FRAGMENT = (
        "Distributed inference splits a language model across multiple edge devices so that "
        "each device processes part of the network while cooperating with the others. "
    )
    PROFILE_DECODE_REQUEST = "The capital of France is"

    ASSISTED_COMMAND_KEY = "profile_command"
    ASSISTED_PREFILL_ACK_COMMAND = "prefill_ack"
    ASSISTED_DECODE_DONE_COMMAND = "decode_done"

    def __init__(self, shards_path: str, device="cpu", dtype=torch.float16, backend: str = "tcp",
                 plot_dir: str = os.path.join("results", "profiling"), verbose: bool = True,
                 worker_kwargs: Optional[dict] = None):
        self.shards_path = shards_path
        self.device = torch.device(device)
        self.dtype = dtype
        self.backend = backend
        self.config = LlamaConfig.from_pretrained(shards_path)
        self.layer_num = self.config.num_hidden_layers
        self.plot_dir = plot_dir
        self.verbose = verbose
        self.worker_kwargs = dict(worker_kwargs or {})
        self.shards: list = []

    def _log(self, *a, **kw) -> None:
        if self.verbose:
            print(*a, flush=True, **kw)

    def _worker(self, src_addr, dst_addr, can_receive_user_request) -> NodeWorker:
        kw = {"max_seq": 2048, "verbose": False}
        kw.update(self.worker_kwargs)
        return NodeWorker(src_addr, dst_addr, can_receive_user_request, self.shards_path, device=self.device,
                          dtype=self.dtype, backend=self.backend, **kw)

    def _sleep(self) -> None:
        if self.PROFILE_INTERVAL_SLEEP_TIME:
            time.sleep(self.PROFILE_INTERVAL_SLEEP_TIME)

    def profile_pipeline_costs(self, batch: int = 1, context: int = 128, n_layers: int = 4,
                               prefill_len: int = 128, replays: int = 20) -> dict:
        """Graph-replay cost model of the deployed pipeline engine on this device, from this
        node's shard folder (:func:`profile_stage_costs`); what ``MasterNode.deploy_pipeline
        (profiles=...)`` plans with."""
        from ..runtime.engine import ShardFolderSource
        res = profile_stage_costs(self.config, ShardFolderSource(self.shards_path, self.config), self.device,
                                  batch=batch, context=context, n_layers=n_layers, prefill_len=prefill_len,
                                  replays=replays, dtype=self.dtype)
        self._log(f"[INFO] stage costs (batch {batch}, context {context}): layer {res['layer_decode_ms']:.4f} ms, "
                  f"embed {res['embed_decode_ms']:.4f} ms, head {res['head_decode_ms']:.4f} ms, "
                  f"stage overhead {res['stage_overhead_ms']:.4f} ms; prefill layer {res['layer_prefill_ms']:.4f} ms")
        return res

    # ---------------------------------------------------------------------- C8a
    def profile_max_layer_num(self, memory_limit_bytes: Optional[float] = None,
                              src_addr: str = "tcp://*:0", dst_addr: str = "tcp://127.0.0.1:40801") -> int:
        """Largest ``i`` such that embedding + layers [0, i) load (reference :46-62)."""
        node = self._worker(src_addr, dst_addr, True)
        max_layer_num = 0
        try:
            for i in range(self.layer_num):
                node.load_shards(0, i + 1)
                if memory_limit_bytes is not None:
                    used = node.engine.memory_bytes() + node.embed_tokens.numel() * node.embed_tokens.element_size()
                    if used > memory_limit_bytes:
                        break
                max_layer_num = i + 1
        except torch.cuda.OutOfMemoryError:
            pass
        finally:
            node.close()
        self._log(f"[INFO] max layer num: {max_layer_num}")
        return max_layer_num

    # ---------------------------------------------------------------------- C8b
    def _fit_latency_models(self, token_lengths, latencies, scatter_token_lengths, scatter_latencies,
                            x_label: str, y_label: str, plot_title: str, plot_filename: str,
                            plot_note: Optional[str] = None) -> dict:
        if len(token_lengths) != len(latencies):
            raise ValueError("[ERROR] token_lengths length must be equal to latencies length.")
        if len(token_lengths) < 3:
            raise ValueError("[ERROR] at least 3 points are needed for quadratic fitting.")
        if len(scatter_token_lengths) != len(scatter_latencies):
            raise ValueError("[ERROR] scatter_token_lengths length must be equal to scatter_latencies length.")
        S = torch.tensor(token_lengths, dtype=torch.float64)
        T = torch.tensor(latencies, dtype=torch.float64)
        Xl = torch.stack((S, torch.ones_like(S)), 1)
        Xq = torch.stack((S ** 2, S, torch.ones_like(S)), 1)
        lin = torch.linalg.lstsq(Xl, T[:, None]).solution[:, 0]
        quad = torch.linalg.lstsq(Xq, T[:, None]).solution[:, 0]

        def metrics(fit):
            r = T - fit
            rmse = torch.sqrt(torch.mean(r ** 2)).item()
            sst = torch.sum((T - T.mean()) ** 2)
            r2 = float("nan") if sst.item() == 0 else (1 - torch.sum(r ** 2) / sst).item()
            return rmse, r2

        lr, lr2 = metrics(Xl @ lin)
        qr, qr2 = metrics(Xq @ quad)
        self._log(f"[INFO] linear latency model: T(S) = {lin[0]:.6e} * S + {lin[1]:.6e}; "
                  f"RMSE = {lr:.6e} sec, R^2 = {lr2:.6f}")
        self._log(f"[INFO] quadratic latency model: T(S) = {quad[0]:.6e} * S^2 + {quad[1]:.6e} * S + "
                  f"{quad[2]:.6e}; RMSE = {qr:.6e} sec, R^2 = {qr2:.6f}")
        plot_path = None
        try:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
            xs = torch.linspace(min(token_lengths), max(token_lengths), 200, dtype=torch.float64)
            os.makedirs(self.plot_dir, exist_ok=True)
            plot_path = os.path.join(self.plot_dir, plot_filename)
            plt.figure(figsize=(8, 5))
            plt.scatter(scatter_token_lengths, scatter_latencies, label="measured latency")
            plt.plot(xs.tolist(), (lin[0] * xs + lin[1]).tolist(), label="linear fit")
            plt.plot(xs.tolist(), (quad[0] * xs ** 2 + quad[1] * xs + quad[2]).tolist(), label="quadratic fit")
            plt.xlabel(x_label)
            plt.ylabel(y_label)
            plt.title(plot_title)
            if plot_note is not None:
                plt.figtext(0.5, 0.01, plot_note, ha="center", fontsize=8)
            plt.grid(alpha=0.3)
            plt.legend()
            plt.tight_layout(rect=(0, 0.04, 1, 1) if plot_note else (0, 0, 1, 1))
            plt.savefig(plot_path, dpi=150)
            plt.close()
            self._log(f"[INFO] latency fit plot saved to {plot_path}")
        except ImportError:
            self._log("[WARNING] matplotlib not available: skipping the plot")
        return {"linear_coefficients": lin, "quadratic_coefficients": quad, "linear_rmse": lr,
                "linear_r_squared": lr2, "quadratic_rmse": qr, "quadratic_r_squared": qr2, "plot": plot_path}

    # ---------------------------------------------------------------------- C8c
    def _report_prefill_decode_similarity(self, prefill_comp_capa_avg: float, decode_comp_capa_avg: float,
                                          prefill_linear_slope: float, decode_linear_slope: float,
                                          prefill_quadratic_coefficients, decode_quadratic_coefficients,
                                          comparison_token_lengths, similarity_threshold: float = 0.30) -> dict:
        if prefill_comp_capa_avg == 0 or prefill_linear_slope == 0:
            self._log("[WARNING] prefill capability is zero; skip relative similarity comparison.")
            return {}
        avg_ratio = decode_comp_capa_avg / prefill_comp_capa_avg
        avg_rel = abs(decode_comp_capa_avg - prefill_comp_capa_avg) / prefill_comp_capa_avg
        slope_ratio = decode_linear_slope / prefill_linear_slope
        slope_rel = abs(decode_linear_slope - prefill_linear_slope) / prefill_linear_slope
        S = torch.tensor(comparison_token_lengths, dtype=torch.float64)
        pa, pb, _ = prefill_quadratic_coefficients.tolist()
        da, db, _ = decode_quadratic_coefficients.tolist()
        pm, dm = 2 * pa * S + pb, 2 * da * S + db
        q_avg = q_max = None
        if not torch.any(pm == 0):
            r = torch.abs(dm - pm) / torch.abs(pm)
            q_avg, q_max = r.mean().item(), r.max().item()
        self._log(f"[INFO] average capability comparison: decode / prefill = {avg_ratio:.6f}, "
                  f"relative difference = {avg_rel:.2%}")
        self._log(f"[INFO] fitted-slope comparison: decode / prefill = {slope_ratio:.6f}, "
                  f"relative difference = {slope_rel:.2%}")
        if q_avg is not None:
            self._log(f"[INFO] quadratic-fit marginal-cost comparison: mean relative difference = {q_avg:.2%}, "
                      f"max relative difference = {q_max:.2%}")
        similar = slope_rel <= similarity_threshold
        self._log(f"[INFO] according to the linear-fit slopes, prefill and decode compute capabilities "
                  f"{'CAN' if similar else 'are NOT'} be regarded as approximately similar under the "
                  f"{similarity_threshold:.0%} threshold.")
        return {"average_ratio": avg_ratio, "average_relative_difference": avg_rel, "slope_ratio": slope_ratio,
                "slope_relative_difference": slope_rel, "quadratic_marginal_mean": q_avg,
                "quadratic_marginal_max": q_max, "similar": similar}

    # ---------------------------------------------------------------------- C8d helpers
    def _synchronize_device(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    @classmethod
    def _build_assisted_command(cls, command: str) -> dict:
        return {cls.ASSISTED_COMMAND_KEY: command}

    @classmethod
    def _is_assisted_command(cls, data, command: Optional[str] = None) -> bool:
        if not isinstance(data, dict) or cls.ASSISTED_COMMAND_KEY not in data:
            return False
        return command is None or data[cls.ASSISTED_COMMAND_KEY] == command

    def _resolve_profile_loaded_layer_num(self, max_layer_num: int) -> int:
        if max_layer_num == -1:
            return self.layer_num
        loaded = max_layer_num - 1  # keep room for the KV cache (reference :323-329)
        if loaded <= 0:
            raise ValueError("[ERROR] max_layer_num is too small to reserve space for KV cache.")
        return loaded

    def _resolve_assisted_target_loaded_layer_num(self, target_max_layer_num: Optional[int]) -> int:
        if target_max_layer_num is None:
            self._log("[WARNING] max_layer_num needed; probing it with profile_max_layer_num().")
            target_max_layer_num = self.profile_max_layer_num()  # Q11 fixed: use the probed value
        if target_max_layer_num == -1:
            raise ValueError("[ERROR] assisted profiling is only needed when target device can only load partial "
                             "layers, but max_layer_num == -1 means the device can load all model layers.")
        loaded = target_max_layer_num - 1
        if loaded <= 0:
            raise ValueError("[ERROR] target_max_layer_num is too small to reserve space for KV cache.")
        if loaded >= self.layer_num:
            raise ValueError("[ERROR] the device can load all model layers, pls do NOT use assisted profiling mode.")
        return loaded

    def _build_profile_input_ids(self, tokenizer) -> tuple:
        lengths = list(self.PROFILE_PREFILL_INPUT_TOKEN_LENGTHS)
        if max(lengths) > self.config.max_position_embeddings:
            raise ValueError("[ERROR] requested prompt length exceeds model max_position_embeddings.")
        prompt = self.PROFILE_PREFILL_PROMPT_FRAGMENT
        ids = tokenizer(prompt, return_tensors="pt")["input_ids"]
        while ids.shape[1] < max(lengths):
            prompt += self.PROFILE_PREFILL_PROMPT_FRAGMENT
            ids = tokenizer(prompt, return_tensors="pt")["input_ids"]
        return lengths, [ids[:, :n].clone() for n in lengths]

    # ---------------------------------------------------------------------- C8e reports
    def _report_prefill_profile_results(self, input_token_lengths, repeated_computation_latencies,
                                        computation_latencies, loaded_layer_num: int) -> tuple:
        if len(computation_latencies) != len(input_token_lengths):
            raise ValueError("[ERROR] tested computation latency number is not equal to request number.")
        scale = self.layer_num / loaded_layer_num
        norm = [x * scale for x in computation_latencies]
        self._log("[INFO] tested prompt token lengths=", input_token_lengths)
        self._log(f"[INFO] first-token latencies (each repeated {self.PROFILE_REPEAT_NUM} times):")
        for r in repeated_computation_latencies:
            self._log(r)
        self._log("[INFO] normalized first-token latencies=", norm)
        caps = [lat / n for n, lat in zip(input_token_lengths, norm)]
        avg = sum(caps) / len(caps)
        self._log("[INFO] each compute capability c_k=", " / ".join(str(c) for c in caps))
        self._log("[INFO] average compute capability c_k=", str(avg), f" sec / (token * {self.layer_num}layer)")
        fit = self._fit_latency_models(input_token_lengths, norm, input_token_lengths, norm,
                                       "Input token length", "First-token latency (sec, full-model equivalent)",
                                       "Prefill first-token latency fit", "profile_prefill_compute_capability.png")
        return avg, fit

    def _report_decode_profile_results(self, cumulative_decode_latencies, displayed_output_token_lengths,
                                       loaded_layer_num: int):
        mx = max(displayed_output_token_lengths)
        if len(cumulative_decode_latencies) < mx:
            self._log("[WARNING] decode profiling stopped early because EOS was generated before "
                      f"output token length reached {mx}.")
        if len(cumulative_decode_latencies) < 3:
            self._log("[WARNING] too few decode points were collected; skip decode fitting and stage comparison.")
            return None
        scale = self.layer_num / loaded_layer_num
        norm = [x * scale for x in cumulative_decode_latencies]
        lengths = list(range(1, len(norm) + 1))
        sampled = [n for n in displayed_output_token_lengths if n <= len(norm)]
        if not sampled:
            self._log("[WARNING] no decode sample reached the configured comparison checkpoints.")
            return None
        sampled_lat = [norm[n - 1] for n in sampled]
        self._log("[INFO] sampled decode output token lengths=", sampled)
        self._log("[INFO] cumulative decode latencies=", sampled_lat)
        caps = [lat / n for n, lat in zip(sampled, sampled_lat)]
        avg = sum(caps) / len(caps)
        self._log("[INFO] average decode compute capability c_k=", str(avg), f" sec / (token * {self.layer_num}layer)")
        fit = self._fit_latency_models(lengths, norm, sampled, sampled_lat, "Output token length",
                                       "Cumulative decode latency (sec, full-model equivalent)",
                                       "Decode cumulative latency fit", "profile_decode_compute_capability.png",
                                       plot_note="Fit uses cumulative latency from every generated output token, "
                                                 "not only sampled checkpoints.")
        return avg, fit, sampled

    # ---------------------------------------------------------------------- C8g rounds
    def _assisted_target_prefill_round(self, node: NodeWorker, measure_latency: bool = False):
        data = node.communicator.receive_data()
        if self._is_assisted_command(data):
            raise RuntimeError("[ERROR] received an assisted command where prefill state was expected.")
        self._synchronize_device()
        t0 = time.perf_counter()
        node.pass_through_shard(data)
        self._synchronize_device()
        t1 = time.perf_counter()
        node.clear_KV_cache()
        node.communicator.transfer_data(self._build_assisted_command(self.ASSISTED_PREFILL_ACK_COMMAND))
        return (t1 - t0) if measure_latency else None

    def _assisted_target_decode_round(self, node: NodeWorker, measure_latency: bool = False) -> list:
        cum, acc = [], 0.0
        while True:
            data = node.communicator.receive_data()
            if self._is_assisted_command(data, self.ASSISTED_DECODE_DONE_COMMAND):
                break
            if self._is_assisted_command(data):
                raise RuntimeError("[ERROR] received unknown assisted command during decode profiling.")
            self._synchronize_device()
            t0 = time.perf_counter()
            out = node.pass_through_shard(data)
            self._synchronize_device()
            t1 = time.perf_counter()
            if measure_latency:
                acc += t1 - t0
                cum.append(acc)
            node.communicator.transfer_data(out)
        node.clear_KV_cache()
        return cum

    def _assistor_assist_prefill_round(self, node: NodeWorker, input_ids: torch.Tensor) -> None:
        node.communicator.transfer_data(node.receive_user_request(input_ids=input_ids))
        data = node.communicator.receive_data()
        if not self._is_assisted_command(data, self.ASSISTED_PREFILL_ACK_COMMAND):
            raise RuntimeError(f"[ERROR] expected assisted profiling command {self.ASSISTED_PREFILL_ACK_COMMAND}, "
                               f"but received {type(data)}.")
        node.clear_KV_cache()

    def _assistor_assist_decode_round(self, node: NodeWorker, max_new_tokens: int) -> None:
        data = node.receive_user_request(request=self.PROFILE_DECODE_REQUEST)
        reached_end = False
        while not reached_end:
            node.communicator.transfer_data(data)
            target_out = node.communicator.receive_data()
            if self._is_assisted_command(target_out):
                raise RuntimeError("[ERROR] received assisted command where target decode state was expected.")
            processed = node.pass_through_shard(target_out)
            reached_end, data = node.receive_next_token(processed, max_new_tokens=max_new_tokens)
        node.communicator.transfer_data(self._build_assisted_command(self.ASSISTED_DECODE_DONE_COMMAND))
        node.clear_KV_cache()

    # ---------------------------------------------------------------------- C8f
    def profile_compute_capability(self, max_layer_num: Optional[int] = None, assisted: bool = False,
                                   src_addr: str = "tcp://*:40800", dst_addr: str = "tcp://172.16.0.1:40800") -> dict:
        if assisted:
            return self._profile_compute_capability_assisted_target(max_layer_num, src_addr, dst_addr)
        if max_layer_num is None:
            self._log("[WARNING] max_layer_num needed; probing it with profile_max_layer_num().")
            max_layer_num = self.profile_max_layer_num()
        node = self._worker("tcp://*:0", "tcp://127.0.0.1:1", True)
        loaded = self._resolve_profile_loaded_layer_num(max_layer_num)
        node.load_shards(0, loaded)
        lengths, reqs = self._build_profile_input_ids(node.tokenizer)
        self._log("[INFO] warming up prefill profiling path...")
        for ids in (reqs[-1], reqs[0]):
            node.pass_through_shard(node.receive_user_request(input_ids=ids))
            self._synchronize_device()
            node.clear_KV_cache()
            self._sleep()
        rep_lat, lat = [], []
        total, done = len(lengths) * self.PROFILE_REPEAT_NUM, 0
        for i in range(len(lengths)):
            cur = []
            for _ in range(self.PROFILE_REPEAT_NUM):
                self._synchronize_device()
                t0 = time.perf_counter()
                node.pass_through_shard(node.receive_user_request(input_ids=reqs[i]))
                self._synchronize_device()
                cur.append(time.perf_counter() - t0)
                node.clear_KV_cache()
                done += 1
                if done < total:
                    self._sleep()
            rep_lat.append(cur)
            lat.append(sum(cur) / len(cur))
        p_avg, p_fit = self._report_prefill_profile_results(lengths, rep_lat, lat, loaded)
        result = {"prefill_lengths": lengths, "prefill_latencies": lat, "prefill_c_k": p_avg, "prefill_fit": p_fit,
                  "loaded_layer_num": loaded}
        if loaded != self.layer_num:
            self._log("[WARNING] decode profiling needs the full model on one device. Pass max_layer_num=-1 on a "
                      "device with enough memory to validate whether prefill and decode compute capabilities "
                      "are similar.")
            node.close()
            return result
        shown = list(self.PROFILE_DECODE_OUTPUT_TOKEN_LENGTHS)
        self._log("[INFO] warming up decode profiling path...")
        d0 = node.receive_user_request(request=self.PROFILE_DECODE_REQUEST)
        end = False
        while not end:
            end, d0 = node.receive_next_token(node.pass_through_shard(d0), max_new_tokens=shown[0])
        self._synchronize_device()
        node.clear_KV_cache()
        self._sleep()
        d0 = node.receive_user_request(request=self.PROFILE_DECODE_REQUEST)
        self._synchronize_device()
        t_start = time.perf_counter()
        cum, end = [], False
        while not end:
            end, d0 = node.receive_next_token(node.pass_through_shard(d0), max_new_tokens=max(shown))
            self._synchronize_device()
            cum.append(time.perf_counter() - t_start)
        node.clear_KV_cache()
        node.close()
        rep = self._report_decode_profile_results(cum, shown, loaded)
        result["decode_cumulative_latencies"] = cum
        if rep is None:
            return result
        d_avg, d_fit, sampled = rep
        result.update({"decode_c_k": d_avg, "decode_fit": d_fit})
        result["similarity"] = self._report_prefill_decode_similarity(
            p_avg, d_avg, p_fit["linear_coefficients"][0].item(), d_fit["linear_coefficients"][0].item(),
            p_fit["quadratic_coefficients"], d_fit["quadratic_coefficients"], sampled)
        return result

    def _profile_compute_capability_assisted_target(self, max_layer_num, src_addr, dst_addr) -> dict:
        loaded = self._resolve_assisted_target_loaded_layer_num(max_layer_num)
        lengths = list(self.PROFILE_PREFILL_INPUT_TOKEN_LENGTHS)
        node = self._worker(src_addr, dst_addr, False)
        node.load_shards(0, loaded)
        self._log("[INFO] assisted target warming up prefill profiling path...")
        for _ in range(2):
            self._assisted_target_prefill_round(node, False)
            self._sleep()
        rep_lat, lat = [], []
        total, done = len(lengths) * self.PROFILE_REPEAT_NUM, 0
        for _ in lengths:
            cur = []
            for _ in range(self.PROFILE_REPEAT_NUM):
                cur.append(self._assisted_target_prefill_round(node, True))
                done += 1
                if done < total:
                    self._sleep()
            rep_lat.append(cur)
            lat.append(sum(cur) / len(cur))
        p_avg, p_fit = self._report_prefill_profile_results(lengths, rep_lat, lat, loaded)
        result = {"prefill_lengths": lengths, "prefill_latencies": lat, "prefill_c_k": p_avg, "prefill_fit": p_fit,
                  "loaded_layer_num": loaded}
        shown = list(self.PROFILE_DECODE_OUTPUT_TOKEN_LENGTHS)
        self._assisted_target_decode_round(node, False)
        self._sleep()
        cum = self._assisted_target_decode_round(node, True)
        node.close()
        rep = self._report_decode_profile_results(cum, shown, loaded)
        result["decode_cumulative_latencies"] = cum
        if rep is not None:
            d_avg, d_fit, sampled = rep
            result.update({"decode_c_k": d_avg, "decode_fit": d_fit})
            result["similarity"] = self._report_prefill_decode_similarity(
                p_avg, d_avg, p_fit["linear_coefficients"][0].item(), d_fit["linear_coefficients"][0].item(),
                p_fit["quadratic_coefficients"], d_fit["quadratic_coefficients"], sampled)
        return result

    def assist_profile_compute_capability(self, target_max_layer_num: int, src_addr: str = "tcp://*:40800",
                                          dst_addr: str = "tcp://172.16.0.2:40800") -> None:
        loaded = self._resolve_assisted_target_loaded_layer_num(target_max_layer_num)
        node = self._worker(src_addr, dst_addr, True)
        node.load_shards(loaded, self.layer_num)
        _, reqs = self._build_profile_input_ids(node.tokenizer)
        for ids in (reqs[-1], reqs[0]):
            self._assistor_assist_prefill_round(node, ids)
            self._sleep()
        total, done = len(reqs) * self.PROFILE_REPEAT_NUM, 0
        for ids in reqs:
            for _ in range(self.PROFILE_REPEAT_NUM):
                self._assistor_assist_prefill_round(node, ids)
                done += 1
                if done < total:
                    self._sleep()
        shown = list(self.PROFILE_DECODE_OUTPUT_TOKEN_LENGTHS)
        self._assistor_assist_decode_round(node, shown[0])
        self._sleep()
        self._assistor_assist_decode_round(node, max(shown))
        node.communicator.flush()
        node.close()
        self._log("[INFO] assist compute capability profiling finished.")

    # ---------------------------------------------------------------------- C8h
    def profile_cold_start_latency(self, max_layer_num: Optional[int] = None) -> dict:
        if max_layer_num is None:
            max_layer_num = self.profile_max_layer_num()
        node = self._worker("tcp://*:0", "tcp://127.0.0.1:1", False)
        loaded = self.layer_num if max_layer_num == -1 else max_layer_num
        if loaded <= 0:
            raise ValueError("[ERROR] invalid max_layer_num")
        self._synchronize_device()
        t0 = time.perf_counter()
        node.load_shards(0, loaded)
        self._synchronize_device()
        dt = time.perf_counter() - t0
        node.close()
        self._log(f"[INFO] overall cold start time ({loaded} layer): ", str(dt))
        self._log("[INFO] load latency per layer: ", str(dt / loaded))
        return {"cold_start_s": dt, "per_layer_s": dt / loaded, "layers": loaded}

    # ---------------------------------------------------------------------- C8i / C8j
    def go_through_every_shards(self, out_token_num: int = 50, n_stages: int = 4, base_port: int = 40800,
                                request: str = "Why the sky blue", input_ids=None) -> list:
        """``n_stages`` NodeWorkers in ONE process on loopback ports base_port.., stepped by hand."""
        L = self.layer_num
        bounds = [round(k * L / n_stages) for k in range(n_stages + 1)]
        nodes = []
        for k in range(n_stages):
            w = self._worker(f"tcp://*:{base_port + k}", f"tcp://127.0.0.1:{base_port + (k + 1) % n_stages}", k == 0)
            w.load_shards(bounds[k], bounds[k + 1])
            nodes.append(w)
        data0 = nodes[0].receive_user_request(request=request, input_ids=input_ids)
        for _ in range(out_token_num):
            nodes[0].communicator.transfer_data(nodes[0].pass_through_shard(data0))
            for k in range(1, n_stages):
                d = nodes[k].communicator.receive_data(timeout_ms=60000)
                nodes[k].communicator.transfer_data(nodes[k].pass_through_shard(d))
            tok = nodes[0].communicator.receive_data(timeout_ms=60000)
            reached_end, data0 = nodes[0].receive_next_token(tok, max_new_tokens=out_token_num)
            if reached_end:
                break
        out = nodes[0].output_ids()[0].tolist()
        for n in nodes:
            n.close()
        return out

    def go_through_every_shards_only_by_profiler(self, out_token_num: int = 50, request: str = "Write a poem "
                                                 "about the blue sky.", input_ids=None) -> list:
        """One engine per layer, no networking (the reference's golden forward, C8j)."""
        from ..runtime.engine import ShardFolderSource, StageEngine
        cfg, dev = self.config, self.device
        dt = torch.bfloat16 if dev.type == "cuda" else self.dtype
        src = ShardFolderSource(self.shards_path, cfg)
        L = self.layer_num
        self.shards = [StageEngine(cfg, i, i + 1, dev, dt, has_embed=(i == 0), has_head=(i == L - 1), source=src,
                                   max_seq=2048) for i in range(L)]
        tok = load_tokenizer(self.shards_path)
        ids = tok(request, return_tensors="pt")["input_ids"][0] if input_ids is None else input_ids.reshape(-1)
        generated = ids.tolist()
        cur = ids
        for _ in range(out_token_num):
            S = cur.numel()
            h = self.shards[0].embed(cur.to(dev))
            for e in self.shards:
                slot, pos = e.prefill_rows([0], [S])
                h = e.forward(h, slot, pos)
                e.advance([0], [S])
            nxt = self.shards[-1].head(h, [S - 1]).cpu()
            generated.append(int(nxt[0]))
            self._log(repr(tok.decode(int(nxt[0]))), end=" ")
            if int(nxt[0]) in cfg.eos_ids:
                break
            cur = nxt
        self._log()
        self._log("output: ", tok.decode(generated))
        return generated


if __name__ == "__main__":
    import sys
    p = NodeProfiler(sys.argv[1] if len(sys.argv) > 1 else "shards/Llama-2-7b-chat-hf_bfloat16",
                     device="cuda:0" if torch.cuda.is_available() else "cpu", dtype=torch.bfloat16)
    p.go_through_every_shards()
