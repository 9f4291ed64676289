#!/usr/bin/env python3
"""Two-process check + latency probe of the IPC ring transport (parallel/ipc_ring.py) - run as
two ranks of a gloo job (both may share one GPU). Rank 0 streams messages of assorted sizes to
rank 1 in bursts of R (the ring depth) with no host synchronisation; rank 1 checks every byte and sends each
one back on the reverse edge. Then a send and a receive captured in hipGraphs are replayed with
fresh contents each time; then batch-1-sized (8 KiB) ping-pong round trips are timed.

    python scripts/ipc_ring_check.py --rank R --world 2 --port P [--device D] [--out FILE]
Prints one JSON line per rank; exit status 0 iff every check passed."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--messages", type=int, default=24)
    ap.add_argument("--pingpong", type=int, default=200)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank, world_size=a.world)
    torch.cuda.set_device(a.device)
    from llm_sharding_amd.parallel.ipc_ring import IpcRingP2P
    dev = torch.device("cuda", a.device)
    R, slot = 3, 4 << 20
    p2p = IpcRingP2P(a.rank, slot_bytes=slot, slots=R, timeout_s=20.0)
    peer = 1 - a.rank
    res = {"rank": a.rank, "ok": True}

    def pattern(i, n):
        g = torch.Generator(device=dev).manual_seed(1000 + i)
        return torch.randint(-2 ** 31, 2 ** 31 - 1, (n // 4,), generator=g, device=dev, dtype=torch.int32)

    # every size a multiple of 4 B, some not of 16 B (the dword-tail path), up to the whole slot
    sizes = [16 * (1 + (i * 7919) % ((1 << 20) // 16)) - 4 * (i % 4) for i in range(a.messages)] + [4, 8, slot]
    # 1) messages 0 -> 1 in bursts of R (every slot of the ring in flight), echoed back 1 -> 0
    if a.rank == 0:
        outs = [pattern(i, n) for i, n in enumerate(sizes)]
        backs = [torch.empty_like(t) for t in outs]
        for c in range(0, len(outs), R):
            for t in outs[c:c + R]:
                p2p.isend(t, peer)
            for b in backs[c:c + R]:
                p2p.recv(b, peer)
        torch.cuda.synchronize()
        res["stream_ok"] = all(bool(torch.equal(o, b)) for o, b in zip(outs, backs))
    else:
        ins = [torch.empty(n // 4, dtype=torch.int32, device=dev) for n in sizes]
        for i, t in enumerate(ins):
            p2p.recv(t, peer)
            p2p.isend(t, peer)
        torch.cuda.synchronize()
        res["stream_ok"] = all(bool(torch.equal(t, pattern(i, n))) for i, (t, n) in enumerate(zip(ins, sizes)))
    # 2) hipGraph-captured send / receive, replayed with new contents
    n = 4096 * 2 * 64
    buf = torch.zeros(n // 4, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        if a.rank == 0:
            p2p.isend(buf, peer)
        else:
            p2p.recv(buf, peer)
    graph_ok = True
    for it in range(5):
        if a.rank == 0:
            buf.copy_(pattern(100 + it, n))
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
        else:
            g.replay()
            torch.cuda.synchronize()
            graph_ok &= bool(torch.equal(buf, pattern(100 + it, n)))
    res["graph_ok"] = graph_ok
    # 3) 8 KiB ping-pong (batch-1 Llama-2-7B hidden state), one-way latency incl. launches
    x = torch.zeros(2048, dtype=torch.int32, device=dev)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.pingpong):
        if a.rank == 0:
            p2p.isend(x, peer)
            p2p.recv(x, peer)
        else:
            p2p.recv(x, peer)
            x.add_(1)
            p2p.isend(x, peer)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res["pingpong_ok"] = int(x[0].item()) == a.pingpong
    res["one_way_us"] = round(dt / a.pingpong / 2 * 1e6, 2)
    # 4) 4 MiB messages (the 512-row Llama-2-7B decode hand-off), one way 0 -> 1, bursts of R
    big = torch.ones(slot // 4, dtype=torch.int32, device=dev)
    nbig = 30
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(nbig):  # the sender runs at most R ahead: its kernels wait for the acks in-kernel
        if a.rank == 0:
            p2p.isend(big, peer)
        else:
            p2p.recv(big, peer)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res["bulk_4mib_us"] = round(dt / nbig * 1e6, 1)
    res["bulk_gbps"] = round(slot * nbig / dt / 1e9, 2)
    res["alloc_kinds"] = sorted(set(p2p.alloc_kinds.values()))
    res["alloc"] = os.environ.get("LSA_IPC_ALLOC", "uncached")
    p2p.check()
    p2p.close()
    res["ok"] = bool(res["stream_ok"] and res["graph_ok"] and res["pingpong_ok"])
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()
    sys.exit(0 if res["ok"] else 1)


if __name__ == "__main__":
    main()
