"""Reference-compatible pipeline-stage runtime and node control plane.

API parity with ``/root/reference/utils/node_worker.py``:

* :class:`Communicator` (re-exported, C1 ``:13-67``) - native TCP PUSH/PULL, in-memory framing.
* :class:`NodeWorker` (C2 ``:70-382``) - ``load_shards``, ``receive_user_request``,
  ``pass_through_shard``, ``receive_next_token``, ``clear_KV_cache``, the clear-KV ring command
  builders/predicates and the ``CLEAR_KV_CACHE_*`` constants, with the same message dicts
  (``input_token_info``, ``next_state_info``, next-token Tensor).
* :class:`NodeController` (C3 ``:385-559``) - config receive on ``tcp://*:<listen_port>``, the
  worker event loop with the reference's dispatch rules, hot re-configuration, request
  forwarding to the chain head.

MI355X-native underneath: the stage forward is a :class:`StageEngine` (fused HIP kernels,
packed weights, static KV cache, fused final-norm/lm_head/argmax) instead of HF modules and a
``DynamicCache``; on the GPU every decode step (seq_len 1) replays a captured hipGraph of the
stage (``use_graph=True``, one graph per batch size; the reference runs its HF modules eagerly,
``:227-309``). Reference quirks fixed on purpose: causal prefill by
default (Q1, ``noncausal_prefill=True`` restores the unmasked reference behaviour); batch > 1
(Q2: next tokens embed to ``[B, 1, H]``); lm_head only on the last position (Q3); EOS by id as
well as by string (Q4); no disk staging (Q5); blocking receive with timeout instead of a busy
poll (Q6); a real request ingress (Q7: ``{"command": "user_request", ...}`` on the config port,
or :meth:`NodeController.receive_request`); no AttributeError when a non-ingress node keeps
its role (Q8); sockets closed on a role change (Q9).

Pipeline mode (the master's RCCL deployment, ``MasterNode.deploy_pipeline``): a config with
``"mode": "pipeline"`` plus ``rank`` / ``world_size`` (the controller's torchrun rank) makes the
controller build a :class:`..parallel.server.PipelineServer` for its layer range instead of a
NodeWorker - micro-batched continuous batching, hidden states over RCCL on one communicator
per ring edge, hipGraph decode replays, tokens on the device. Rank 0 is the ingress: its config
port takes the reference ``user_request`` messages (optionally with ``reply_to``) and
``shutdown``. No cos/sin tables travel (every stage derives positions from its own KV state).
A pipeline that loses a rank is dropped by the survivors - on a peer's closed connection, or on
the master's ``abort_pipeline`` (then, if still blocked inside a communicator op after
``ABORT_GRACE_S``, by aborting its process groups) - which release their stages and groups and
wait for the master's re-deployment as a ZMQ chain (``MasterNode.failover``).

On ROCm devices the engine computes in bfloat16: ``dtype=torch.float16`` is accepted (the
reference default) and mapped to bfloat16 with a notice.
"""
from __future__ import annotations

import json
import threading
import os
import sys
import time
from typing import Optional

import torch

from ..config import LlamaConfig
from ..models.rope import full_cos_sin
from ..models.tokenizer import load_tokenizer
from ..parallel import protocol
from ..parallel.communicator import Again, Communicator
from ..parallel.transport import PullSocket, PushSocket, local_ip
from ..runtime.engine import DecodeGraph, ShardFolderSource, StageEngine, WeightSource
from .forwarding_utils import build_position_ids  # noqa: F401 - re-exported as in the reference module


def _log(msg: str) -> None:
    print(msg, flush=True)


class _EngineKV:
    """``past_key_value`` view of the worker's static cache (``get_seq_length``)."""

    def __init__(self, worker: "NodeWorker"):
        self.w = worker

    def get_seq_length(self, layer_idx: int = 0) -> int:
        return 0 if self.w.engine is None else int(self.w.engine.seq_len[0])


class NodeWorker:
    CLEAR_KV_CACHE_COMMAND = "clear_KV_cache"
    CLEAR_KV_CACHE_ORIGIN_KEY = "origin_node"

    def __init__(self, src_addr: str, dst_addr: str, can_receive_user_request: bool, shards_path: str,
                 device="cpu", dtype=torch.float16, backend: str = "tcp", max_batch: int = 8,
                 max_seq: int = 4096, noncausal_prefill: bool = False,
                 source: Optional[WeightSource] = None, verbose: bool = True,
                 rccl_ranks: Optional[tuple] = None, ship_rope: bool = False, use_graph: bool = True):
        # backend "rccl": envelopes over TCP, tensors device-to-device over torch.distributed
        self.communicator = Communicator(src_addr=src_addr, dst_addr=dst_addr, backend=backend,
                                         device=torch.device(device), rccl_ranks=rccl_ranks)
        self.can_receive_user_request = can_receive_user_request
        self.shards_path = shards_path
        self.device = torch.device(device)
        if self.device.type == "cuda" and dtype != torch.bfloat16:
            if verbose:
                _log(f"[INFO] {dtype} requested on {self.device}: the MI355X kernels compute in torch.bfloat16")
            dtype = torch.bfloat16
        self.dtype = dtype
        self.config = LlamaConfig.from_pretrained(shards_path)
        self.layer_num = self.config.num_hidden_layers
        self.max_batch, self.max_seq = max_batch, max_seq
        self.noncausal_prefill = noncausal_prefill
        self.source = source or ShardFolderSource(shards_path, self.config)
        self.verbose = verbose
        self.ship_rope = ship_rope  # send real cos/sin tables in next_state_info (reference wire parity)
        # GPU decode steps (seq_len 1) replay a captured hipGraph of the stage (one per batch
        # size) instead of launching every kernel from Python
        self.use_graph = use_graph
        self._graphs: dict = {}
        self._graph_pos: dict = {}

        self.tokenizer = None
        self.embed_tokens = None   # embedding table [V, H] (ingress / head stage)
        self.engine: Optional[StageEngine] = None
        self.rope = None           # (cos, sin) tables [max_pos, Hd/2] (every stage)
        self.shard = None          # alias of the engine (reference attribute name)
        self.lm_head = None
        self.past_key_value = None
        self.start = 0
        self.end = 0
        self.batch_size = 0
        if can_receive_user_request:
            self.generated_ids: list = []
            self._load_embedding()
            self.input_token_length = None

    # ------------------------------------------------------------------ loading
    def _load_embedding(self) -> None:
        if self.verbose:
            _log("[INFO] loading tokenizer...")
        self.tokenizer = load_tokenizer(self.shards_path)
        if self.verbose:
            _log("[INFO] loading embedding layer...")
        self.embed_tokens = self.source.embedding(self.device, self.dtype).contiguous()
        if self.verbose:
            _log("[INFO] embedding layer loaded.")

    def load_shards(self, start: int, end: int) -> None:
        if start < 0 or start >= end or end > self.layer_num:
            raise ValueError("[ERROR] start or end is invalid")
        self.start, self.end = start, end
        self.engine = self.shard = self.lm_head = None
        self._graphs, self._graph_pos = {}, {}
        if self.device.type == "cuda":
            torch.cuda.empty_cache()
        if self.verbose:
            _log(f"[INFO] loading hidden layer {start}~{end}(end excluded)...")
        self.engine = StageEngine(self.config, start, end, self.device, self.dtype,
                                  has_embed=False, has_head=(end == self.layer_num), source=self.source,
                                  max_slots=self.max_batch, max_seq=self.max_seq,
                                  causal=not self.noncausal_prefill)
        self.shard = self.engine
        self.rope = (self.engine.cos, self.engine.sin)
        self.lm_head = self.engine.lm_head
        self.past_key_value = _EngineKV(self)
        if self.verbose:
            _log(f"[INFO] hidden layer {start}~{end}(end excluded) loaded.")

    # ------------------------------------------------------------------ helpers
    def _embed(self, ids: torch.Tensor) -> torch.Tensor:
        ids = ids.to(self.device)
        if self.device.type == "cuda":
            from ..ops import hip
            flat = ids.reshape(-1).to(torch.int32)
            out = torch.empty((flat.numel(), self.config.hidden_size), dtype=torch.bfloat16, device=self.device)
            hip.embed(flat, self.embed_tokens, out)
            return out.reshape(*ids.shape, -1)
        return torch.nn.functional.embedding(ids.long(), self.embed_tokens)

    # ------------------------------------------------------------------ ingress
    @torch.inference_mode()
    def receive_user_request(self, request: str = "Write a poem about the blue sky.",
                             input_ids: Optional[torch.Tensor] = None) -> dict:
        if not self.can_receive_user_request:
            raise RuntimeError("[ERROR] this node does not have embedding layer while receiving user request.")
        if input_ids is None:
            if self.verbose:
                _log("[INFO] input: " + request)
            input_ids = self.tokenizer(request, return_tensors="pt")["input_ids"]
        else:
            if input_ids.ndim != 2:
                raise ValueError("[ERROR] input_ids must be a 2D tensor with shape [batch_size, seq_len].")
            if self.verbose:
                _log("[INFO] input: inputted from direct token ids.")
        input_ids = input_ids.to(dtype=torch.long)
        self.input_token_length = int(input_ids.shape[1])
        if self.verbose:
            _log("[INFO] input token number: " + str(self.input_token_length))
        self.generated_ids = [input_ids.cpu()]
        hidden_states = self._embed(input_ids)
        B, S = int(input_ids.shape[0]), int(input_ids.shape[1])
        self.batch_size = B
        return {"hidden_states": hidden_states, "batch_size": B, "seq_len": S}

    # ------------------------------------------------------------------ stage forward
    @torch.inference_mode()
    def pass_through_shard(self, state_info: dict):
        if self.engine is None:
            raise RuntimeError("[ERROR] no shard loaded")
        if self.is_input_token_info(state_info):
            if self.start != 0:
                raise RuntimeError("[ERROR] after embedding layer, the states should first passing hidden layer 0!")
            self.batch_size = int(state_info["batch_size"])
        elif self.is_next_state_info(state_info):
            pass  # positions come from this stage's own KV length (same values as shipped cos/sin)
        else:
            attrs = [a for a in dir(state_info) if not a.startswith("__")]
            raise RuntimeError(f"[ERROR] Received unknown state_info type: {type(state_info)}; "
                               f"Attributes: {attrs if attrs else 'No attributes found'}")
        hs = state_info["hidden_states"]
        B, S, H = hs.shape
        if B > self.max_batch:
            raise ValueError(f"[ERROR] batch {B} exceeds max_batch={self.max_batch}")
        eng = self.engine
        past = eng.seq_len[0]
        slots = list(range(B))
        if S == 1 and self.use_graph and eng.gpu:
            out = self._graph_step(hs, B, H)
        else:
            slot, pos = eng.prefill_rows(slots, [S] * B)
            kv_len = [past + S] * (B * S) if (self.noncausal_prefill and S > 1) else None
            h = eng.forward(hs.reshape(B * S, H).to(self.device, eng.dtype), slot, pos, kv_len=kv_len)
            eng.advance(slots, [S] * B)
            out = eng.head(h, [b * S + S - 1 for b in range(B)]) if self.end == self.layer_num else h
        if self.end == self.layer_num:
            return out.to("cpu", torch.long)
        if eng.cos is None or not self.ship_rope:
            # every stage derives its positions from its own KV length (the reference ships the
            # first stage's tables down the chain, node_worker.py:267-271): keep the message
            # schema with empty tables - no device->host copy, no bytes on the wire
            cos = sin = torch.empty((B, S, 0), dtype=eng.dtype)
        else:  # ship_rope=True: the reference's [B, S, head_dim] tables (slice on device first)
            position_ids = torch.arange(0, S, dtype=torch.long)[None].expand(B, S)
            cos, sin = full_cos_sin(eng.cos[past:past + S].cpu(), eng.sin[past:past + S].cpu(), position_ids,
                                    dtype=eng.dtype)
        return {"hidden_states": out.reshape(B, S, H).clone(), "cos": cos, "sin": sin}

    def _graph_step(self, hs: torch.Tensor, B: int, H: int) -> torch.Tensor:
        """One decode step of rows 0..B-1 by hipGraph replay (DecodeGraph "mid", or "last" with
        the fused head + argmax): the hidden state goes into the graph's input buffer, the
        positions live on the device and advance inside the graph; they are re-uploaded only
        when the host's KV lengths moved without the graph (prefill, clear_KV_cache)."""
        eng = self.engine
        last = self.end == self.layer_num
        g = self._graphs.get(B)
        if g is None:
            # captured outside inference mode: the graph's own tensors (and the CUDA generator's
            # graph-safe RNG state, created at the process's first capture) stay normal tensors
            # that later captures elsewhere may update in place
            with torch.inference_mode(False):
                g = DecodeGraph(eng, B, "last" if last else "mid").capture()
            self._graphs[B] = g
            self._graph_pos[B] = None
        want = [int(eng.seq_len[r]) for r in range(B)]
        if self._graph_pos[B] != want:
            g.set_positions()
        g.h_in.copy_(hs.reshape(B, H).to(self.device, eng.dtype))
        g.replay()
        eng.advance(list(range(B)), [1] * B)
        self._graph_pos[B] = [p + 1 for p in want]
        return g.tokens if last else g.out_hidden

    # ------------------------------------------------------------------ autoregression
    @torch.inference_mode()
    def receive_next_token(self, next_token_id: torch.Tensor, max_new_tokens: int = 1024) -> tuple:
        if not self.can_receive_user_request:
            raise RuntimeError('[ERROR] this node does not store the "generated token id" list, but received a next_token_id.')
        next_token_id = next_token_id.reshape(-1).to("cpu", torch.long)
        self.generated_ids.append(next_token_id.unsqueeze(-1))
        tid = int(next_token_id[0])
        next_token = self.tokenizer.decode(tid)
        if self.verbose:
            print(repr(next_token), end=" ", flush=True)
        eos_ids = set(self.config.eos_ids)
        if getattr(self.tokenizer, "eos_token_id", None) is not None:
            eos_ids.add(int(self.tokenizer.eos_token_id))
        reached_eos = next_token == getattr(self.tokenizer, "eos_token", None) or bool(
            all(int(t) in eos_ids for t in next_token_id))
        reached_max = len(self.generated_ids) > max_new_tokens
        if reached_eos or reached_max:
            if self.verbose:
                print()
                final_ids = torch.cat(self.generated_ids, dim=-1)
                _log("output: " + self.tokenizer.decode(final_ids[0]))
                _log("\n[INFO] output token number: " + str(len(self.generated_ids) - 1))
            return True, None
        hidden_states = self._embed(next_token_id.unsqueeze(-1))  # [B, 1, H]
        return False, {"hidden_states": hidden_states, "batch_size": self.batch_size, "seq_len": 1}

    def output_ids(self) -> torch.Tensor:
        return torch.cat(self.generated_ids, dim=-1)

    # ------------------------------------------------------------------ protocol predicates
    @staticmethod
    def is_input_token_info(data) -> bool:
        return isinstance(data, dict) and "batch_size" in data and "seq_len" in data

    @staticmethod
    def is_next_state_info(data) -> bool:
        return isinstance(data, dict) and "cos" in data and "sin" in data

    def clear_KV_cache(self) -> None:
        """Reset the per-request state; weights stay resident (reference ``:319-355``)."""
        if self.engine is not None:
            self.engine.reset()
        self.batch_size = 0
        if self.can_receive_user_request:
            self.generated_ids = []
            self.input_token_length = None
        if self.verbose:
            _log("\n[INFO] KV cache and all states caused by prev user are cleared.")

    def _get_clear_KV_cache_origin(self) -> dict:
        return {"src_addr": self.communicator.src_addr, "dst_addr": self.communicator.dst_addr,
                "shards_start": self.start, "shards_end": self.end}

    def build_clear_KV_cache_command(self) -> dict:
        return {"command": self.CLEAR_KV_CACHE_COMMAND,
                self.CLEAR_KV_CACHE_ORIGIN_KEY: self._get_clear_KV_cache_origin()}

    @classmethod
    def is_clear_KV_cache_command(cls, data) -> bool:
        return isinstance(data, dict) and data.get("command") == cls.CLEAR_KV_CACHE_COMMAND

    def is_clear_KV_cache_command_origin(self, data) -> bool:
        return (self.is_clear_KV_cache_command(data)
                and data.get(self.CLEAR_KV_CACHE_ORIGIN_KEY) == self._get_clear_KV_cache_origin())

    def close(self) -> None:
        self.communicator.close()


CONFIG_KEYS = ("src_addr", "dst_addr", "can_receive_user_request", "first_node_addr", "shards_start", "shards_end")


class _StageRef:
    """What rank 0's ingress thread holds instead of the PipelineServer itself (so a dropped
    stage can be freed while the listener still runs): ``submit`` forwards to the live stage."""

    def __init__(self, ctrl):
        self._ctrl = ctrl

    def submit(self, *a, **kw):
        # under the controller's submit lock: a request either reaches the live server before the
        # drop starts (and is then answered by the drop's unfinished() sweep) or is rejected here
        with self._ctrl._submit_lock:
            srv = self._ctrl.server
            if srv is None or self._ctrl._aborted or getattr(self._ctrl, "phase", "serving") != "serving":
                raise ValueError("pipeline dropped (a rank was lost)")
            return srv.submit(*a, **kw)


class NodeController:
    """Node-side control plane (reference C3). Config JSON arrives on ``tcp://*:listen_port``."""

    def __init__(self, shards_path: str, device, dtype=torch.float16, listen_port: int = 40700,
                 backend: str = "tcp", wait_config: bool = True, config: Optional[dict] = None,
                 worker_kwargs: Optional[dict] = None, poll_ms: int = 20, verbose: bool = True):
        self.shards_path = shards_path
        self.device = device
        self.dtype = dtype
        self._submit_lock = threading.Lock()  # ingress submits vs the pipeline drop (_StageRef)
        self.backend = backend
        self.poll_ms = poll_ms
        self.verbose = verbose
        self.worker_kwargs = dict(worker_kwargs or {})
        self.listen_addr = "tcp://*:" + str(listen_port)
        self.recv_config_socket = PullSocket(self.listen_addr)
        self.listen_port = self.recv_config_socket.port
        self.send_request_socket = None
        self.first_node_addr = ""
        self.pending_requests: list = []
        self.running = False
        self.finished_outputs: list = []
        self.node_worker: Optional[NodeWorker] = None
        self.server = None  # PipelineServer (pipeline mode)
        self.forwarded = 0
        self.t_boot = time.monotonic()
        self.received_config = config if config is not None else (self._receive_config() if wait_config else None)
        if self.received_config is not None:
            self._apply_new_role(self.received_config)
            if self.verbose:
                _log("[INFO] Node is ready.")

    # ------------------------------------------------------------------ config
    def _receive_config(self, no_block: bool = False) -> Optional[dict]:
        while True:
            if no_block:
                try:
                    raw = self.recv_config_socket.recv_bytes(0)
                except Again:
                    return None
            else:
                if self.verbose:
                    _log("[CONFIG] Waiting for configuration file from master node...")
                raw = self.recv_config_socket.recv_bytes(-1)
            msg = json.loads(raw.decode())
            if isinstance(msg, dict) and msg.get("command") in ("user_request", "shutdown", "ping"):
                self._handle_command(msg)
                continue
            if isinstance(msg, dict) and "command" in msg:
                # commands of another mode (abort_pipeline / replan outside a pipeline): acknowledged
                # (so a master waiting on them does not stall) and otherwise ignored - never a config
                _log(f"[WARNING] command {msg['command']!r} ignored: no pipeline deployed here")
                self._pong(msg)
                continue
            if self.verbose:
                _log("[CONFIG] Received configuration file from master node:")
                for k, v in msg.items():
                    _log(f"  - {k}: {v}")
            return msg

    def _handle_command(self, msg: dict) -> None:
        if msg["command"] == "shutdown":
            self.running = False
        elif msg["command"] == "user_request":
            self.pending_requests.append(msg)
        elif msg["command"] == "ping":
            self._pong(msg)

    def status(self) -> dict:
        """Liveness / role snapshot (answered to ``ping``; SURVEY.md §5.3 stage-liveness)."""
        if self.server is not None:
            c = self.received_config or {}
            return {"listen_port": self.listen_port, "configured": True, "mode": "pipeline",
                    "shards": [self.server.start, self.server.end], "replans": self.server.replans,
                    "rank": c.get("rank"),
                    "ingress": c.get("rank") == 0, "finished_requests": len(self.finished_outputs),
                    "phase": getattr(self, "phase", "serving"), "uptime_s": time.monotonic() - self.t_boot}
        w = self.node_worker
        return {"listen_port": self.listen_port, "configured": w is not None,
                "pipeline_lost": getattr(self, "pipeline_lost", None),
                "shards": [w.start, w.end] if w is not None else None,
                "ingress": bool(w.can_receive_user_request) if w is not None else False,
                "forwarded": self.forwarded, "finished_requests": len(self.finished_outputs),
                "phase": getattr(self, "phase", "chain"), "uptime_s": time.monotonic() - self.t_boot}

    def _pong(self, msg: dict) -> None:
        reply_to = msg.get("reply_to")
        if not reply_to:
            return
        try:
            s = PushSocket(reply_to)
            s.send_bytes(json.dumps({"command": "pong", "nonce": msg.get("nonce"), **self.status()}).encode())
            s.close(linger_ms=2000)
        except OSError as e:
            _log(f"[WARNING] pong to {reply_to} failed: {e}")

    def _apply_new_role(self, cfg: dict) -> None:
        for k in CONFIG_KEYS:
            if k not in cfg:
                raise KeyError(f"[ERROR] configuration misses {k!r}")
        if cfg.get("mode") == "pipeline":
            self._apply_pipeline_role(cfg)
            return
        if self.node_worker is not None:
            self.node_worker.close()  # Q9: release the old sockets before rebinding
            self.node_worker = None
        self._set_first_node_addr(cfg)
        kw = dict(self.worker_kwargs)
        if cfg.get("rccl_ranks") is not None:  # optional extension key: (src_rank, dst_rank)
            kw["rccl_ranks"] = tuple(cfg["rccl_ranks"])
        self.node_worker = NodeWorker(cfg["src_addr"], cfg["dst_addr"], cfg["can_receive_user_request"],
                                      self.shards_path, device=self.device, dtype=self.dtype, backend=self.backend,
                                      verbose=self.verbose, **kw)
        self.node_worker.load_shards(cfg["shards_start"], cfg["shards_end"])

    def _apply_pipeline_role(self, cfg: dict) -> None:
        """Build this rank's PipelineServer (collective: every rank of the job does it when its
        config arrives - the control gloo group and the per-edge RCCL groups are created here)."""
        import torch.distributed as dist
        from ..parallel.server import PipelineServer
        if not dist.is_initialized():
            raise RuntimeError("[ERROR] pipeline mode needs torch.distributed (start_node.py --backend rccl "
                               "under torch.distributed.run)")
        r, n = dist.get_rank(), dist.get_world_size()
        if int(cfg["rank"]) != r or int(cfg["world_size"]) != n:
            raise RuntimeError(f"[ERROR] pipeline config for rank {cfg['rank']}/{cfg['world_size']} delivered to "
                               f"rank {r}/{n}")
        if self.server is not None:
            raise RuntimeError("[ERROR] a pipeline is already deployed here: re-plan it through rank 0 "
                               "(MasterNode.replan) or shut it down first")
        if self.node_worker is not None:
            self.node_worker.close()
            self.node_worker = None
        mcfg = LlamaConfig.from_pretrained(self.shards_path)
        source = ShardFolderSource(self.shards_path, mcfg)
        ctrl = dist.new_group(backend="gloo")  # rank 0's command headers (never blocks a GPU)
        self.server = PipelineServer(mcfg, source, r, n, int(cfg["shards_start"]), int(cfg["shards_end"]),
                                     self.device, batch=int(cfg.get("batch", 8)),
                                     microbatches=int(cfg.get("microbatches", max(2, n))),
                                     max_seq=int(cfg.get("max_seq", 2048)),
                                     prefill_budget=int(cfg.get("prefill_budget", 2048)),
                                     use_graph=bool(cfg.get("use_graph", True)), dtype=self.dtype, ctrl_group=ctrl,
                                     causal=not self.worker_kwargs.get("noncausal_prefill", False),
                                     streams=int(cfg.get("streams", 1)))
        self.tokenizer = None
        if r == 0:
            try:
                self.tokenizer = load_tokenizer(self.shards_path)
            except Exception as e:  # noqa: BLE001 - token-id requests still work
                _log(f"[WARNING] no tokenizer ({e}); only input_ids requests are served")
        if self.verbose:
            _log(f"[INFO] pipeline stage {r}/{n}: layers [{cfg['shards_start']}, {cfg['shards_end']}) on {self.device}")

    def _run_pipeline(self, max_new_tokens: int) -> bool:
        """Pipeline mode: rank 0 reads requests from its config port on a thread and schedules;
        the other ranks follow rank 0's commands until it stops (``shutdown``). Returns True if
        the pipeline was dropped because a rank was lost (a peer's error, or the master's
        ``abort_pipeline`` from :meth:`MasterNode.failover`).

        Failover ordering (no message may be lost between the pipeline and the chain): the
        listener thread is the ONLY reader of the config socket until it is joined; while the
        stage is dropped it keeps answering pings (phase ``dropping``), refuses new requests with
        an error reply and queues any config that arrives early (``self._early_configs``).
        Only after the join does the phase become ``awaiting_redeploy`` - the state the master
        waits for before it sends the chain configs - and :meth:`_await_redeploy` drains the
        early queue before it reads the socket itself."""
        import threading
        from ..parallel.ingress import Replies, run_ingress
        lost = None
        stop = threading.Event()
        serving = threading.Event()
        serving.set()
        self._aborted = False
        self._abort_timer = None
        self._abort_lock = threading.Lock()
        self._early_configs = []
        self.phase = "serving"
        # no local (thread argument, timer argument, closure) may keep the stage alive: its
        # process groups must be freed by _drop_pipeline so their connections close and the
        # peers blocked on this rank fail over too
        first = self.server.first

        def other(msg):
            if not isinstance(msg, dict):
                return
            cmd = msg.get("command")
            if cmd == "ping":
                self._pong(msg)
            elif cmd == "abort_pipeline":
                # the master lost a rank of this torchrun world (MasterNode.failover): rank 0 stops
                # scheduling, every rank drops its pipeline and waits for a chain re-deployment
                with self._abort_lock:
                    # the timer exists BEFORE _aborted is set: the serving loop returns on
                    # _aborted and must find the timer to cancel it (it reads it under this lock)
                    if not self._aborted and serving.is_set():
                        # a rank still inside an RCCL op with the dead peer after the grace period
                        # cannot see a closed connection (gloo can): abort its communicators so the
                        # op fails instead of waiting for the watchdog
                        t = threading.Timer(self.ABORT_GRACE_S, self._abort_groups, args=(serving,))
                        t.daemon = True
                        t.start()
                        self._abort_timer = t
                    self._aborted = True
                self._pong(msg)
            elif cmd == "replan" or (msg.get("mode") == "pipeline" and "stages" in msg):
                # live re-shard of the deployed pipeline (reference hot re-config, node_worker.py
                # :445-474): rank 0 owns the command stream, so the new split is applied there,
                # in order, once the requests in flight have finished
                if self.server is None or not self.server.first or self._aborted:
                    _log("[WARNING] replan ignored: send it to rank 0 (the ingress) of a running pipeline")
                    return
                try:
                    self.server.request_replan(msg["stages"])
                    if self.verbose:
                        _log(f"[CONFIG] re-plan requested: {msg['stages']}")
                except ValueError as e:
                    _log(f"[ERROR] {e}")
            elif cmd == "user_request":  # non-ingress rank (rank 0's run_ingress takes its own)
                self._reject_request(msg, "this rank is not the pipeline's ingress")
            elif cmd is None and msg.get("mode") != "pipeline":
                # a chain config that arrived before this rank finished dropping its stage
                _log("[CONFIG] chain configuration queued until the pipeline is dropped")
                self._early_configs.append(msg)
            else:
                _log(f"[WARNING] message {cmd!r} ignored while a pipeline is deployed")

        def accepting():
            if self._aborted or self.phase != "serving":
                return "pipeline dropped (a rank was lost); resubmit after the master's failover"
            return None

        replies = None
        if first:
            replies = Replies(self.tokenizer, verbose=self.verbose,
                              on_done=lambda r, text: self.finished_outputs.append(list(r.output_ids)))
            th = threading.Thread(target=run_ingress, args=(_StageRef(self), self.recv_config_socket, self.tokenizer,
                                                            stop, max_new_tokens, replies, other, accepting),
                                  daemon=True)
        else:
            def pings():
                while not stop.is_set():
                    try:
                        raw = self.recv_config_socket.recv_bytes(200)
                    except Again:
                        continue
                    msg = json.loads(raw.decode())
                    if isinstance(msg, dict) and msg.get("command") == "shutdown":
                        continue  # the pipeline's STOP comes from rank 0's command stream
                    other(msg)
            th = threading.Thread(target=pings, daemon=True)
        th.start()
        try:
            if first:
                self.server.serve(stop_when_idle=False, should_stop=lambda: stop.is_set() or self._aborted)
            else:
                self.server.serve()
        except Exception as e:  # noqa: BLE001 - a peer rank died mid-collective
            lost = repr(e)
        with self._abort_lock:  # no communicator abort may start once serve() has returned
            serving.clear()
            timer = self._abort_timer  # set, if ever, together with _aborted (same lock)
        if timer is not None:
            timer.cancel()
            timer.join(timeout=5)  # its thread has exited before the phase changes
        dropped = lost is not None or self._aborted
        if dropped:
            with self._submit_lock:  # no submit can slip in between the phase change and the sweep
                self.phase = "dropping"  # the listener still answers pings and queues early configs
                pending = self.server.unfinished() if replies is not None else []
            if replies is not None:
                for r in pending:
                    replies.error(r.reply_to, "pipeline dropped (a rank was lost) before the request finished",
                                  request_id=r.rid)
            self._drop_pipeline(lost or "aborted by the master")
        stop.set()
        while th.is_alive():  # the listener must be gone before anyone else reads the socket
            th.join(timeout=5)
            if th.is_alive():
                _log("[WARNING] waiting for the config listener to stop")
        if replies is not None:
            replies.close()
        self.running = False
        if dropped:
            self.phase = "awaiting_redeploy"
        return dropped

    ABORT_GRACE_S = 10.0  # abort_pipeline -> communicator abort if this rank is still serving

    def _abort_groups(self, serving) -> None:
        """Grace period over and still inside a collective: abort every process group of the
        stage (``ProcessGroup.abort()``, the supported form - ncclCommAbort on RCCL) so the
        blocked op returns an error instead of waiting for the watchdog."""
        import torch.distributed as dist
        with self._abort_lock:
            if not serving.is_set():
                return
            groups, server = [], self.server
            if server is not None:
                groups += list(getattr(server.p2p, "groups", {}).values())
                if server.ctrl is not None:
                    groups.append(server.ctrl)
            from ..parallel import communicator
            groups += list(getattr(communicator, "_EDGE_GROUPS", {}).values())
            if dist.is_initialized():
                groups.append(dist.group.WORLD)
            _log(f"[ERROR] still blocked in the pipeline after the abort grace period: aborting "
                 f"{len(groups)} process groups with ProcessGroup.abort()")
            groups = [g for g in groups if isinstance(g, dist.ProcessGroup)]  # not NON_GROUP_MEMBER
            done = 0
            for g in groups:
                try:
                    g.abort()
                    done += 1
                except Exception as e:  # noqa: BLE001 - e.g. a backend without abort support
                    _log(f"[WARNING] ProcessGroup.abort() on {g!r}: {e}")
            self.abort_report = {"method": "ProcessGroup.abort", "groups": len(groups), "aborted": done}
            _log(f"[INFO] process-group abort: {done}/{len(groups)} aborted")

    def _drop_pipeline(self, reason: str) -> None:
        """The torchrun world lost a rank: release this rank's stage and its process groups (which
        closes its connections, so peers still blocked on it fail too and drop theirs) and fall
        back to the ZMQ chain transport for the master's re-deployment over the survivors."""
        import gc
        import torch.distributed as dist
        from ..parallel import communicator
        _log(f"[ERROR] pipeline dropped ({reason}); waiting for the master's chain re-deployment")
        self.pipeline_lost = reason
        # every reference to a process group goes (the stage's edge groups and command group,
        # the job-wide edge groups of start_node.py); gloo closes a group's connections only
        # when the group is freed, and a peer blocked in a receive from this rank (e.g. the
        # command broadcast of rank 0) fails only then
        self.server = None
        getattr(communicator, "_EDGE_GROUPS", {}).clear()
        gc.collect()
        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception as e:  # noqa: BLE001
                _log(f"[WARNING] destroy_process_group: {e}")
        gc.collect()
        self.backend = "tcp"

    def _reject_request(self, msg: dict, reason: str) -> None:
        reply_to = msg.get("reply_to")
        _log(f"[ERROR] request not served: {reason}")
        if not reply_to:
            return
        try:
            s = PushSocket(reply_to)
            s.send_bytes(protocol.encode({"request_id": None, "error": reason, "output_ids": [], "text": ""}))
            s.close(linger_ms=2000)
        except OSError as e:
            _log(f"[WARNING] error reply to {reply_to} failed: {e}")

    def _await_redeploy(self) -> bool:
        """After :meth:`_drop_pipeline` (listener joined): apply a chain config that arrived while
        the stage was being dropped, else answer pings until one arrives; False if a ``shutdown``
        came first. Requests received meanwhile are kept for the new ingress; a survivor that
        does not become the ingress answers them with an error (the client resubmits)."""
        while True:
            if self._early_configs:
                msg = self._early_configs.pop(0)
            else:
                try:
                    raw = self.recv_config_socket.recv_bytes(200)
                except Again:
                    continue
                msg = json.loads(raw.decode())
            cmd = msg.get("command") if isinstance(msg, dict) else None
            if cmd == "shutdown":
                return False
            if cmd == "user_request":
                self.pending_requests.append(msg)
                continue
            if cmd is not None:  # ping, a repeated abort_pipeline, ...
                self._pong(msg)
                continue
            if msg.get("mode") == "pipeline":
                _log("[ERROR] a pipeline config after a lost rank: restart the torchrun job to redeploy one")
                continue
            self.received_config = msg
            self._apply_new_role(msg)
            self.phase = "chain"
            if not self.node_worker.can_receive_user_request:
                for req in self.pending_requests:
                    self._reject_request(req, "this node is not the chain's ingress after the failover")
                self.pending_requests = []
            return True

    def _set_first_node_addr(self, cfg: dict) -> None:
        new = cfg.get("first_node_addr", "") if cfg.get("can_receive_user_request") else ""
        if new != self.first_node_addr:
            if self.send_request_socket is not None:
                self.send_request_socket.close()
                self.send_request_socket = None
            if new:
                self.send_request_socket = PushSocket(new)
            self.first_node_addr = new

    def _change_first_node_addr(self, new_first_node_addr: str) -> str:
        self._set_first_node_addr({"can_receive_user_request": True, "first_node_addr": new_first_node_addr})
        return self.first_node_addr

    def check_new_config(self) -> None:
        new = self._receive_config(no_block=True)
        if not new:
            return
        old = self.received_config or {}
        w = self.node_worker
        if w is None or new["can_receive_user_request"] != old.get("can_receive_user_request"):
            self._apply_new_role(new)
        else:
            w.communicator.change_src_addr(new["src_addr"])
            w.communicator.change_dst_addr(new["dst_addr"])
            if w.communicator.backend == "rccl":
                # the tensor side channel follows the new ring too: explicit (src, dst) ranks
                # from the config, else the default torchrun ring
                import torch.distributed as dist
                r, n = dist.get_rank(), dist.get_world_size()
                src, dst = new["rccl_ranks"] if new.get("rccl_ranks") is not None else ((r - 1) % n, (r + 1) % n)
                w.communicator.change_ranks(src, dst)
            self._set_first_node_addr(new)  # Q8: no-op for non-ingress nodes
            if (new["shards_start"], new["shards_end"]) != (w.start, w.end):
                w.load_shards(new["shards_start"], new["shards_end"])
            else:
                w.clear_KV_cache()
        self.received_config = new
        if self.verbose:
            _log("[INFO] The new configuration node is ready.")

    # ------------------------------------------------------------------ requests
    def _forward_request(self, data: dict, data_path: str = "results/send_request.pt", keep_data: bool = False):
        payload = protocol.encode(data)
        self.send_request_socket.send_bytes(payload)
        if keep_data:
            os.makedirs(os.path.dirname(data_path) or ".", exist_ok=True)
            with open(data_path, "wb") as f:
                f.write(payload)
            return data_path
        return None

    def receive_request(self, request: str = "Write a poem about the blue sky.",
                        input_ids: Optional[torch.Tensor] = None) -> None:
        if not self.node_worker.can_receive_user_request:
            raise RuntimeError("[ERROR] this node cannot receive user request.")
        token_info = self.node_worker.receive_user_request(request, input_ids=input_ids)
        if self.send_request_socket is None:
            raise RuntimeError("[ERROR] no first_node_addr configured for request forwarding")
        self._forward_request(token_info)

    # ------------------------------------------------------------------ loop
    def process_one(self, received_data, max_new_tokens: int = 1024) -> bool:
        """Dispatch one data-plane message (reference ``run_worker_loop`` body). Returns True
        if something was forwarded down the chain."""
        w = self.node_worker
        if w.is_clear_KV_cache_command(received_data):
            if not w.is_clear_KV_cache_command_origin(received_data):
                w.communicator.transfer_data(received_data)
                w.clear_KV_cache()
            return False
        if isinstance(received_data, torch.Tensor):
            if w.start != 0:
                raise RuntimeError('[ERROR] I\'m not the first node in the model chain, but received "next_token_id".')
            reached_end, received_data = w.receive_next_token(received_data, max_new_tokens)
            if reached_end:
                self.finished_outputs.append(w.output_ids())
                w.communicator.transfer_data(w.build_clear_KV_cache_command())
                w.clear_KV_cache()
                return False
        elif w.is_input_token_info(received_data):
            if w.start != 0:
                raise RuntimeError('[ERROR] I\'m not the first node in the model chain, but received "input_token_info".')
        elif w.is_next_state_info(received_data):
            if w.start == 0:
                raise RuntimeError('[ERROR] I\'m the first node in the model chain, but received "next_state_info".')
        else:
            attrs = [a for a in dir(received_data) if not a.startswith("__")]
            raise RuntimeError(f"[ERROR] Received unknown data type: {type(received_data)}; "
                               f"Attributes: {attrs if attrs else 'No attributes found'}")
        processed = w.pass_through_shard(received_data)
        w.communicator.transfer_data(processed)
        self.forwarded += 1
        if w.start != 0 and self.verbose:
            print("*", end=" ", flush=True)
        return True

    def run_worker_loop(self, max_new_tokens: int = 1024, max_idle_s: Optional[float] = None) -> None:
        """Serve until a ``shutdown`` command arrives (or ``max_idle_s`` without traffic)."""
        self.running = True
        if self.server is not None:
            if not self._run_pipeline(max_new_tokens) or not self._await_redeploy():
                return
            self.running = True  # re-deployed as a chain stage over the survivors
        idle_since = time.monotonic()
        while self.running:
            try:
                data = self.node_worker.communicator.receive_data(timeout_ms=self.poll_ms)
                idle_since = time.monotonic()
                self.process_one(data, max_new_tokens)
            except Again:
                pass
            while self.pending_requests and self.node_worker.can_receive_user_request:
                req = self.pending_requests.pop(0)
                ids = torch.tensor(req["input_ids"]) if req.get("input_ids") is not None else None
                self.receive_request(req.get("text", ""), input_ids=ids)
                idle_since = time.monotonic()
            self.check_new_config()
            if max_idle_s is not None and time.monotonic() - idle_since > max_idle_s:
                break
        self.running = False

    def close(self) -> None:
        if self.node_worker is not None:
            self.node_worker.close()
        if self.send_request_socket is not None:
            self.send_request_socket.close()
        self.recv_config_socket.close()


def send_user_request(node_ip: str, port: int, text: str = "", input_ids=None, max_new_tokens: int = None,
                      reply_to: Optional[str] = None) -> None:
    """Client helper: submit a request to an ingress NodeController's config port (fixes Q7).
    ``reply_to``: a PULL address that receives the finished request (pipeline mode / serve.py)."""
    msg = {"command": "user_request", "text": text}
    if max_new_tokens is not None:
        msg["max_new_tokens"] = int(max_new_tokens)
    if reply_to:
        msg["reply_to"] = reply_to
    if input_ids is not None:
        msg["input_ids"] = [list(map(int, r)) for r in (input_ids.tolist() if hasattr(input_ids, "tolist") else input_ids)]
    s = PushSocket(f"tcp://{node_ip}:{port}")
    s.send_bytes(json.dumps(msg).encode())
    s.close(linger_ms=5000)


def ping_node(node_ip: str, port: int, timeout_ms: int = 2000, command: str = "ping") -> Optional[dict]:
    """Liveness probe: send ``ping`` to a controller's config port and wait for its ``pong``
    (its :meth:`NodeController.status`). Returns None if no answer within ``timeout_ms``.
    ``command="abort_pipeline"``: the same exchange, asking a pipeline rank to drop its stage."""
    import secrets
    reply = PullSocket("tcp://127.0.0.1:0" if node_ip in ("127.0.0.1", "localhost") else "tcp://*:0")
    host = "127.0.0.1" if node_ip in ("127.0.0.1", "localhost") else local_ip()
    nonce = secrets.randbits(31)
    s = PushSocket(f"tcp://{node_ip}:{port}")
    try:
        s.send_bytes(json.dumps({"command": command, "nonce": nonce, "reply_to": f"tcp://{host}:{reply.port}"}).encode())
        deadline = time.monotonic() + timeout_ms / 1e3
        while True:
            left = int((deadline - time.monotonic()) * 1e3)
            if left <= 0:
                return None
            try:
                msg = json.loads(reply.recv_bytes(timeout_ms=left).decode())
            except Again:
                return None
            if msg.get("command") == "pong" and msg.get("nonce") == nonce:
                return msg
    finally:
        s.close(linger_ms=0)
        reply.close()


def send_shutdown(node_ip: str, port: int) -> None:
    s = PushSocket(f"tcp://{node_ip}:{port}")
    s.send_bytes(json.dumps({"command": "shutdown"}).encode())
    s.close(linger_ms=5000)


__all__ = ["Communicator", "NodeWorker", "NodeController", "send_user_request", "send_shutdown", "ping_node", "Again"]


if __name__ == "__main__":
    shards = sys.argv[1] if len(sys.argv) > 1 else "shards/Llama-2-7b-chat-hf_float16"
    NodeController(shards, device="cuda:0" if torch.cuda.is_available() else "cpu", dtype=torch.bfloat16).run_worker_loop()
