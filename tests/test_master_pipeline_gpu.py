"""The master -> ConfigSender -> NodeController pipeline-mode path on one MI355X: a one-rank
torch.distributed job (the controller thread), the master deploying it, requests submitted to
the controller's config port and answered on a reply address. The controller's PipelineServer
runs the HIP kernels and hipGraph decode; its outputs must equal the same server driven
directly in-process (identical kernels, batch geometry and order: bitwise equal)."""
import socket
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_master_pipeline_mode_on_gpu(tiny_shards_bf16):
    import torch.distributed as dist
    from llm_sharding_amd.config import LlamaConfig
    from llm_sharding_amd.parallel import protocol
    from llm_sharding_amd.parallel.communicator import init_edge_groups
    from llm_sharding_amd.parallel.scheduler import DeviceSpec
    from llm_sharding_amd.parallel.server import PipelineServer
    from llm_sharding_amd.parallel.transport import PullSocket
    from llm_sharding_amd.runtime.engine import ShardFolderSource
    from llm_sharding_amd.utils.master_node import MasterNode
    from llm_sharding_amd.utils.node_worker import NodeController

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1)
    try:
        init_edge_groups()
        cport = _port()
        box = {}

        def node():
            try:
                ctrl = NodeController(tiny_shards_bf16, device="cuda:0", dtype=torch.bfloat16, listen_port=cport,
                                      backend="rccl", verbose=False)
                ctrl.run_worker_loop(max_new_tokens=8)
                box["outs"] = ctrl.finished_outputs
                ctrl.close()
            except Exception as e:  # noqa: BLE001
                box["err"] = repr(e)

        th = threading.Thread(target=node, daemon=True)
        th.start()
        reply = PullSocket("tcp://127.0.0.1:0")
        prompts = [[1, 33, 44, 55, 66], [7, 8, 9], [100, 5, 17, 200, 3, 41, 12]]
        n_new = 6
        try:
            master = MasterNode.from_shards(tiny_shards_bf16, [DeviceSpec(config_port=cport, data_port=_port())])
            master.deploy_pipeline(batch=4, microbatches=1, max_seq=64, prefill_budget=64)
            for pr in prompts:
                master.submit(input_ids=[pr], max_new_tokens=n_new, reply_to=f"tcp://127.0.0.1:{reply.port}")
            got = {}
            for _ in prompts:
                m = protocol.decode(reply.recv_bytes(timeout_ms=120000))
                got[m["request_id"]] = m["output_ids"]
            master.shutdown()
            th.join(timeout=120)
        finally:
            reply.close()
        assert "err" not in box, box.get("err")
        # the same server, driven in-process
        cfg = LlamaConfig.from_pretrained(tiny_shards_bf16)
        srv = PipelineServer(cfg, ShardFolderSource(tiny_shards_bf16, cfg), 0, 1, 0, cfg.num_hidden_layers, "cuda:0",
                             batch=4, microbatches=1, max_seq=64, prefill_budget=64, use_graph=True)
        want = srv.generate(prompts, max_new_tokens=n_new, eos_ids=tuple(cfg.eos_ids))
        for rid in range(len(prompts)):
            assert got[rid] == want[rid], (rid, got[rid], want[rid])
            assert all(0 <= t < cfg.vocab_size for t in got[rid])
    finally:
        dist.destroy_process_group()
