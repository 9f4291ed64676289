"""Master node: profile-driven placement + deployment of a NodeController chain.

The reference README (``/root/reference/README.md:7-8``) describes a scheduling algorithm on
the master that calls ``ConfigSender``; the repository only ships a hand-written placement
(``send_config.py:5-44``). ``MasterNode`` closes that gap:

1. devices (host, config/data ports, HBM capacity, relative speed) are described by
   :class:`DeviceSpec` - speed factors can be taken from ``NodeProfiler`` results
   (per-token compute capability ``c_k``, :meth:`MasterNode.speed_from_profiles`);
2. :func:`plan_stages` picks contiguous layer ranges minimising the bottleneck stage under
   the memory caps (exact DP);
3. :meth:`deploy` sends the reference 6-key configs (ring chain, ingress = stage 0) through
   ``ConfigSender``; :meth:`submit` / :meth:`shutdown` drive the deployed chain;
4. failure detection / elastic recovery: :meth:`health` pings every
   controller's config port (``ping`` -> ``pong`` with its status); :meth:`failover` drops
   the devices that stopped answering, re-plans the layers over the survivors and hot
   re-configures them (the reference's live re-shard path, ``node_worker.py:445-474``); a
   deployed pipeline (item 5) that lost a rank is first dropped by its survivors, which then
   serve as a ZMQ chain (a torchrun world cannot shrink);
5. the RCCL deployment on one node (BASELINE north star: "the master_node scheduler places
   shards on the 8 GPUs of one node"): :meth:`deploy_pipeline` plans the stages over the
   controllers of a torchrun job (``start_node.py --backend rccl``: controller i = rank i =
   GPU i, config port base + i) and sends each the reference config extended with
   ``mode="pipeline"``, its rank, the world size, the whole stage list and the serving
   geometry; the controllers then run the micro-batched RCCL pipeline (PipelineServer) and
   :meth:`submit` feeds requests to rank 0;
6. live re-shard of that deployed pipeline (the reference's hot re-configuration,
   ``/root/reference/utils/node_worker.py:445-474``, which there rebinds one ZMQ chain):
   :meth:`replan` re-plans the split inside the same torchrun world - new device speeds
   (e.g. fresh ``NodeProfiler`` measurements) or explicit ranges - and sends it to rank 0,
   which drains the requests in flight and moves every stage to its new ``[start, end)``
   (PipelineServer.request_replan); the ring edges stay, so no communicator is rebuilt.
"""
from __future__ import annotations

import json
import time
from dataclasses import replace
from typing import List, Optional, Sequence

from ..config import LlamaConfig
from ..parallel.scheduler import DeviceSpec, Plan, build_chain_configs, plan_stages
from ..parallel.transport import PushSocket
from .config_sender import ConfigSender
from .node_worker import ping_node, send_shutdown, send_user_request


class MasterNode:
    def __init__(self, cfg: LlamaConfig, devices: Sequence[DeviceSpec], kv_tokens: int = 4096):
        self.cfg = cfg
        self.devices = list(devices)
        self.kv_tokens = kv_tokens
        self.plan: Optional[Plan] = None
        self.senders: List[ConfigSender] = []
        self.mode = "chain"

    @classmethod
    def from_shards(cls, shards_path: str, devices: Sequence[DeviceSpec], kv_tokens: int = 4096) -> "MasterNode":
        return cls(LlamaConfig.from_pretrained(shards_path), devices, kv_tokens)

    @staticmethod
    def speed_from_profiles(profiles: Sequence[dict]) -> list:
        """Relative time multipliers from NodeProfiler results (decode c_k if present, else
        prefill c_k); the fastest device gets 1.0."""
        ck = [p.get("decode_c_k", p.get("prefill_c_k")) for p in profiles]
        base = min(ck)
        return [c / base for c in ck]

    def make_plan(self) -> Plan:
        self.plan = plan_stages(self.cfg, self.devices, kv_tokens=self.kv_tokens)
        return self.plan

    def configs(self) -> list:
        if self.plan is None:
            self.make_plan()
        return build_chain_configs(self.plan)

    def deploy(self, timeout_ms: int = 10000) -> list:
        cfgs = self.configs()
        self.senders = []
        for st, c in zip(self.plan.stages, cfgs):
            s = ConfigSender(node_port=st.device.config_port)
            s.build_config(c["shards_start"], c["shards_end"], c["can_receive_user_request"], c["src_addr"],
                           c["dst_addr"], first_node_addr=c["first_node_addr"])
            if not s.send_config(st.device.host, timeout_ms):
                raise TimeoutError(f"config not delivered to {st.device.host}:{st.device.config_port}")
            self.senders.append(s)
        return cfgs

    def plan_from_profiles(self, profiles: Sequence[dict], kv_tokens: int = 0) -> Plan:
        """Plan with MEASURED costs of the deployed engine: ``profiles[i]`` is device i's
        :func:`~.node_profiler.profile_stage_costs` result. Device 0's per-layer / embedding /
        head / per-stage costs are the cost model, every device's speed factor its per-layer
        decode time relative to device 0 (est_time of each stage = predicted ms per step)."""
        from .node_profiler import costs_for_planner
        if len(profiles) != len(self.devices):
            raise ValueError("plan_from_profiles: one profile per device")
        base = profiles[0]["layer_decode_ms"]
        self.devices = [replace(d, speed=(p["layer_decode_ms"] / base if base > 0 else 1.0))
                        for d, p in zip(self.devices, profiles)]
        self._plan_costs = costs_for_planner(self.cfg, profiles[0])
        self.plan = plan_stages(self.cfg, self.devices, kv_tokens=kv_tokens, **self._plan_costs)
        return self.plan

    def deploy_pipeline(self, batch: int = 8, microbatches: int = 0, max_seq: int = 2048,
                        prefill_budget: int = 2048, streams: int = 1, use_graph: bool = True,
                        timeout_ms: int = 10000, profiles: Optional[Sequence[dict]] = None) -> list:
        """Plan contiguous layer ranges over the devices (device i = torchrun rank i, KV cache of
        ``microbatches`` x ``batch`` sequences of ``max_seq`` tokens counted against each GPU's
        HBM) and configure every controller for the micro-batched RCCL pipeline. ``profiles``:
        per-device stage-cost profiles of the deployed engine (NodeProfiler
        .profile_pipeline_costs) - the plan then balances measured step times
        (:meth:`plan_from_profiles`). Returns the configs sent (rank order)."""
        n = len(self.devices)
        M = microbatches or max(2, n)
        if profiles is not None:
            self.plan_from_profiles(profiles, kv_tokens=max_seq * batch * M)
        else:
            self.plan = plan_stages(self.cfg, self.devices, kv_tokens=max_seq * batch * M)
        stages = [[st.start, st.end] for st in self.plan.stages]
        ing = self.plan.stages[0].device
        cfgs, self.senders = [], []
        for r, st in enumerate(self.plan.stages):
            d, nxt = st.device, self.plan.stages[(r + 1) % n].device
            s = ConfigSender(node_port=d.config_port)
            c = s.build_config(st.start, st.end, r == 0, f"tcp://*:{d.data_port}", f"tcp://{nxt.host}:{nxt.data_port}",
                               first_node_addr=f"tcp://{ing.host}:{ing.config_port}" if r == 0 else "",
                               mode="pipeline", backend="rccl", rank=r, world_size=n, stages=stages, batch=batch,
                               microbatches=M, max_seq=max_seq, prefill_budget=prefill_budget, streams=streams,
                               use_graph=use_graph)
            if not s.send_config(d.host, timeout_ms):
                raise TimeoutError(f"config not delivered to {d.host}:{d.config_port}")
            self.senders.append(s)
            cfgs.append(dict(c))
        self.mode = "pipeline"
        self._kv_tokens_pipeline = max_seq * batch * M
        return cfgs

    def replan(self, stages: Optional[Sequence] = None, speeds: Optional[Sequence[float]] = None,
               timeout_s: float = 120.0, wait: bool = True) -> list:
        """Move the deployed pipeline to a new layer split without restarting it. ``stages``:
        explicit [[start, end], ...] per rank; else ``speeds`` (relative time multipliers per
        device, e.g. :meth:`speed_from_profiles`) re-run the exact min-max planner. The split is
        sent to rank 0; with ``wait`` this returns once every rank reports its new range."""
        if self.mode != "pipeline" or self.plan is None:
            raise RuntimeError("replan: no pipeline deployed (deploy_pipeline first)")
        if stages is None:
            if speeds is not None:
                if len(speeds) != len(self.devices):
                    raise ValueError("replan: one speed per device")
                self.devices = [replace(d, speed=float(v)) for d, v in zip(self.devices, speeds)]
            self.plan = plan_stages(self.cfg, self.devices, kv_tokens=self._kv_tokens_pipeline,
                                    **getattr(self, "_plan_costs", {}))
            stages = [[st.start, st.end] for st in self.plan.stages]
        stages = [[int(a), int(b)] for a, b in stages]
        ing = self.devices[0]
        s = PushSocket(f"tcp://{ing.host}:{ing.config_port}")
        s.send_bytes(json.dumps({"command": "replan", "stages": stages}).encode())
        s.close(linger_ms=5000)
        if wait:
            deadline = time.monotonic() + timeout_s
            while True:
                st = self.health(timeout_ms=2000)
                if all(x is not None and list(x.get("shards", [])) == stages[i] for i, (_, x) in enumerate(st)):
                    break
                if time.monotonic() > deadline:
                    raise TimeoutError(f"replan: ranks did not reach {stages}: {[x for _, x in st]}")
                time.sleep(0.2)
        self.plan_ranges = stages
        return stages

    def health(self, timeout_ms: int = 2000) -> list:
        """[(DeviceSpec, status dict | None)] for every device of the current plan."""
        devs = [st.device for st in self.plan.stages] if self.plan is not None else self.devices
        return [(d, ping_node(d.host, d.config_port, timeout_ms)) for d in devs]

    def failover(self, timeout_ms: int = 2000) -> list:
        """Ping the deployed chain; if any controller is dead, re-plan over the devices that
        answered and redeploy. Returns the list of dropped devices (empty if all alive). A
        deployed pipeline that lost a rank is dropped by its survivors first
        (:meth:`_drop_pipeline`) and they are re-deployed as a chain."""
        status = self.health(timeout_ms)
        for _ in range(2):  # a silent controller is pinged twice more before it counts as dead
            if all(st is not None for _, st in status):
                break
            status = [(d, st if st is not None else ping_node(d.host, d.config_port, timeout_ms)) for d, st in status]
        dead = [d for d, st in status if st is None]
        if not dead:
            return []
        alive = [d for d, st in status if st is not None]
        if not alive:
            raise RuntimeError("[ERROR] every controller is unreachable")
        if self.mode == "pipeline":
            self._drop_pipeline(alive, timeout_ms)
        self.devices = [d for d in self.devices if d not in dead]
        self.plan = None
        for s in self.senders:
            s.close()
        self.senders = []
        self.deploy(timeout_ms=max(timeout_ms, 10000))
        return dead

    def _drop_pipeline(self, alive: list, timeout_ms: int, drop_timeout_s: float = 120.0) -> None:
        """A torchrun world cannot lose a rank and go on (a slow but live rank is re-balanced with
        :meth:`replan` instead), so the survivors leave it: ``abort_pipeline`` to every live rank
        (the others first, acknowledged, then rank 0, which stops scheduling), each rank drops its
        stage and process groups (NodeController._drop_pipeline) and waits; the caller then
        re-deploys them as a ZMQ chain. Ranks blocked on the dead one fail on its closed
        connections and drop out the same way."""
        ing = self.plan.stages[0].device if self.plan is not None else self.devices[0]
        deadline = time.monotonic() + drop_timeout_s
        for d in [d for d in alive if d is not ing] + [d for d in alive if d is ing]:
            while ping_node(d.host, d.config_port, timeout_ms, command="abort_pipeline") is None:
                if time.monotonic() > deadline:
                    raise RuntimeError(f"[ERROR] pipeline rank {d.host}:{d.config_port} did not acknowledge the "
                                       "abort; restart the torchrun job and redeploy")
        while True:
            # "awaiting_redeploy" is reported only once a rank has dropped its stage AND stopped
            # its pipeline listener, so the chain configs sent next reach the reader that
            # applies them (NodeController._run_pipeline)
            st = [ping_node(d.host, d.config_port, timeout_ms) for d in alive]
            if all(x is not None and x.get("phase") == "awaiting_redeploy" for x in st):
                break
            if time.monotonic() > deadline:
                raise RuntimeError(f"[ERROR] pipeline ranks did not drop their stages: {st}; restart the torchrun job")
            time.sleep(0.2)
        self.mode = "chain"

    def submit(self, text: str = "", input_ids=None, max_new_tokens: Optional[int] = None,
               reply_to: Optional[str] = None) -> None:
        ing = self.plan.stages[0].device
        send_user_request(ing.host, ing.config_port, text=text, input_ids=input_ids, max_new_tokens=max_new_tokens,
                          reply_to=reply_to)

    def shutdown(self) -> None:
        # pipeline mode: rank 0 stops the whole job (its STOP header reaches every stage)
        stages = self.plan.stages[:1] if self.mode == "pipeline" else self.plan.stages
        for st in stages:
            send_shutdown(st.device.host, st.device.config_port)
        for s in self.senders:
            s.close()
