#!/usr/bin/env python3
"""Headline benchmark: whole-node output tokens/s (+ p50 per-token latency) of Llama-2-7B
layer-sharded over N MI355X GPUs (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W
    (N > 1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
             --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...)

Workload (synthetic prompts, random-init bf16 weights of the exact Llama-2-7B architecture,
generated on each device - no checkpoints are available offline):
  * rank r owns a contiguous layer range chosen by the master scheduler (rank 0 also holds
    the embedding, rank N-1 the final norm + lm_head), one process per GPU;
  * M = S x N micro-batches of B sequences each are in flight (S x B sequences per GPU,
    fixed -> weak scaling); every sequence was prefilled with a P-token prompt first. The
    default is one micro-batch of 512 sequences per GPU: above 128 rows a decode step's
    projections run on the hand-written stream-K / split-K MFMA GEMM (csrc/kernels/gemm_sk.hip)
    with its epilogue (RoPE + KV write, residual add, SwiGLU) fused, which beats the 128-row
    GEMV kernels on S concurrent streams; with S > 1 each GPU replays its micro-batches'
    graphs on S HIP streams;
  * one timed "step" = every in-flight sequence produces one new token (greedy, fused
    lm_head+argmax on device); hidden states move stage->stage with RCCL send/recv over
    xGMI, token ids return last->first the same way.
  * W untimed warm-up steps, then exactly K timed steps bracketed by barrier +
    torch.cuda.synchronize(); the max over ranks is reported by rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_TOK_S = 4.3  # only reference figure (~4.3 tok/s, start_node.py:20 comment; different HW/model)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--batch", type=int, default=512,
                    help="sequences per micro-batch (per GPU, <= 1024); <= 128 decode on the fused GEMV "
                         "kernels, more on the stream-K MFMA GEMM (gemm_sk.hip) with fused epilogues")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--max-seq", type=int, default=0, help="0 = prompt + warmup + steps, rounded up to 64")
    ap.add_argument("--streams", type=int, default=1,
                    help="micro-batches resident per GPU; on one GPU they replay concurrently on this many "
                         "HIP streams")
    ap.add_argument("--microbatches", type=int, default=0, help="0 = streams x pipeline stages")
    ap.add_argument("--dp", type=int, default=1,
                    help="data-parallel pipeline replicas (gpus/dp stages each); 1 = the reference's "
                         "layout, one pipeline over all GPUs")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--trace", default="", help="write per-rank Chrome-trace timelines of the timed steps here")
    ap.add_argument("--weight-dtype", default="bf16", choices=("bf16", "fp8"),
                    help="fp8: OCP e4m3 projection/lm_head weights with per-row scales (W8A16, not the headline)")
    ap.add_argument("--latency-steps", type=int, default=32,
                    help="after the throughput pass, time this many batch-1 decode steps through the same "
                         "pipeline (b1_p50_tpot_ms / b1_tok_s in the JSON line); 0 = skip")
    ap.add_argument("--mid-batch", type=int, default=128,
                    help="after the batch-1 pass, time --latency-steps decode steps of this many sequences "
                         "(<= 128, the fused-GEMV regime; mid_p50_tpot_ms / mid_tok_s); 0 = skip")
    ap.add_argument("--ttft-lens", default="2048",
                    help="one GPU: after the decode passes, batch-1 time-to-first-token (embed -> all layers -> "
                         "lm_head argmax, median of 3 after a warm-up) at these prompt lengths on a separate "
                         "engine of the same model (ttft_prompt_ms in the JSON line); '' or 0 = skip")
    ap.add_argument("--extras", default="llama3.2-3b,llama2-13b,llama2-70b:10",
                    help="one GPU: after the headline, short decode runs of these models at the same batch "
                         "(MODEL or MODEL:LAYERS = one stage of that many layers with 8 micro-batches, e.g. "
                         "the 70B 8-stage plan's 10-layer stage) -> 'extra' in the JSON line; '' = skip")
    ap.add_argument("--stage-layers", type=int, default=0,
                    help="profile one pipeline stage: the model cut to this many layers (NOT the headline metric)")
    ap.add_argument("--transport", default="rccl", choices=("rccl", "ipc"),
                    help="stage hand-off: rccl (send/recv per ring edge) or ipc (decode messages through "
                         "IPC-mapped HBM rings with device flags, parallel/ipc_ring.py; prefill stays on RCCL)")
    ap.add_argument("--device", default="cuda", choices=("cuda", "cpu"),
                    help="cpu: the same schedule on gloo + the torch CPU path (multi-rank rehearsal)")
    ap.add_argument("--no-supervise", dest="supervise", action="store_false",
                    help="N > 1: run the rank's work in this process (default: a GPU-free per-rank supervisor "
                         "runs it in a fresh child and can restart it once, see --no-fallback)")
    ap.add_argument("--no-fallback", dest="fallback", action="store_false",
                    help="N > 1: do not restart with --transport ipc when the RCCL ring preflight fails")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """``--gpus N`` without a launcher: start N copies of this script as child processes, one
    rank per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in their env),
    BEFORE this process touches the GPU - the counterpart of the reference's run_this.sh
    (/root/reference/run_this.sh:11-17), which starts its N stage processes itself. Rank 0's
    output passes through; if any rank fails the others are stopped and the exit code is
    non-zero."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    _forward_termination(lambda: procs)
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONUNBUFFERED="1",
                   LSA_PARENT_PID=str(os.getpid()))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL, start_new_session=True))
    rc = 0
    pending = list(range(n))
    while pending:
        for r in list(pending):
            code = procs[r].poll()
            if code is None:
                continue
            pending.remove(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"[bench] rank {r} exited with {code}; stopping the other ranks", file=sys.stderr, flush=True)
                for q in pending:  # only the process groups started here
                    try:
                        os.killpg(procs[q].pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        time.sleep(0.2)
    return rc


PREFLIGHT_EXIT = 75  # = parallel.pipeline.PREFLIGHT_EXIT (not imported: the supervisor stays light)


def _die_with_parent() -> None:
    """Run FIRST in every child this script starts (``LSA_PARENT_PID`` in its env): the kernel
    sends this process SIGKILL when the process that started it exits (PR_SET_PDEATHSIG), however
    that happens - a launcher's killpg aimed at the parent's process group, a driver timeout,
    SIGKILL - so no GPU-holding worker outlives its supervisor in its own session. Set here in
    the child rather than between fork and exec: the supervisor already runs gloo threads when it
    starts a worker, and code run there in a multithreaded parent can deadlock on a lock another
    thread held (advisor round 5). If the parent is already gone (it died before the prctl took
    effect) the child exits at once."""
    import ctypes
    import signal
    want = os.environ.pop("LSA_PARENT_PID", None)
    if not want:
        return
    try:
        ctypes.CDLL(None, use_errno=True).prctl(1, int(signal.SIGKILL), 0, 0, 0)  # PR_SET_PDEATHSIG = 1
    except Exception:  # noqa: BLE001 - not Linux: the signal handlers below still stop the children
        return
    if os.getppid() != int(want):
        os._exit(1)


def _stop_group(proc, grace_s: float = 10.0) -> None:
    """SIGTERM the child's process group, then SIGKILL it if it is still there after ``grace_s``."""
    import signal
    if proc is None or proc.poll() is not None:
        return
    try:
        os.killpg(proc.pid, signal.SIGTERM)
        proc.wait(timeout=grace_s)
    except ProcessLookupError:
        return
    except Exception:  # noqa: BLE001 - TimeoutExpired
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        proc.wait()


def _forward_termination(children) -> None:
    """SIGTERM / SIGINT / SIGHUP to this process stop every child process group it started
    (``children()`` lists them), then exit with 128 + signal."""
    import signal

    def handler(signum, _frame):
        signal.signal(signum, signal.SIG_DFL)
        for p in children():
            _stop_group(p)
        os._exit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, handler)


def _spawn_worker(argv: list, port: int, extra_env: dict):
    import subprocess
    env = dict(os.environ, MASTER_PORT=str(port), LSA_BENCH_ROLE="worker", PYTHONUNBUFFERED="1",
               LSA_PARENT_PID=str(os.getpid()), **extra_env)
    # the workers rendezvous on their own store (rank 0's worker hosts it), not torchrun's agent store
    env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
    return subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env, start_new_session=True)


def _watch(proc, store, rank: int, world: int, attempt: int) -> int:
    """Wait for this rank's worker; if another rank's worker of the same attempt has already
    failed, stop ours too (it would only wait on the dead peer until the collective timeout)."""
    import signal
    others = [r for r in range(world) if r != rank]
    while True:
        code = proc.poll()
        if code is not None:
            return code
        for r in others:
            key = f"lsa_bench/{attempt}/exit/{r}"
            if store.check([key]) and int(store.get(key)) != 0:
                time.sleep(2.0)  # let our worker print its own view first
                if proc.poll() is None:
                    try:
                        os.killpg(proc.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
                    try:
                        return proc.wait(timeout=20)
                    except Exception:  # noqa: BLE001
                        os.killpg(proc.pid, signal.SIGKILL)
                        return proc.wait()
                return proc.poll()
        time.sleep(0.2)


def supervise(a, argv: list) -> int:
    """Per-rank supervisor of a multi-GPU run (never touches the GPU). The rank's real work runs
    in a FRESH child process; if any rank's child fails the ring-edge preflight
    (parallel/pipeline.preflight_edges: a dead RCCL edge, named, within LSA_PREFLIGHT_TIMEOUT_S),
    every supervisor starts one more fresh child with ``--transport ipc`` (IPC rings over xGMI,
    gloo control; no RCCL communicator) and the JSON line says ``"fallback": true``. Any other
    failure is returned as is. Coordination uses the launcher's rendezvous store (gloo group on
    the CPU); the children rendezvous on a port rank 0 picks per attempt."""
    import datetime

    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", timeout=datetime.timedelta(hours=2))
    store = dist.distributed_c10d._get_default_store()
    attempts = [([], {})]
    current = []  # the running worker: stopped with this supervisor (signal handlers + PDEATHSIG)
    _forward_termination(lambda: current)
    if a.transport == "rccl" and a.fallback:
        attempts.append((["--transport", "ipc"], {"LSA_BENCH_FALLBACK": "1"}))
    code = 0
    for i, (extra, env) in enumerate(attempts):
        if rank == 0:
            store.set(f"lsa_bench/{i}/port", str(_free_port()))
        port = int(store.get(f"lsa_bench/{i}/port"))
        if i and rank == 0:
            print(f"[bench] ring preflight failed on the RCCL transport: restarting every rank once with "
                  f"--transport ipc", file=sys.stderr, flush=True)
        proc = _spawn_worker(argv + extra, port, env)
        current[:] = [proc]
        code = _watch(proc, store, rank, world, i)
        store.set(f"lsa_bench/{i}/exit/{rank}", str(code))
        keys = [f"lsa_bench/{i}/exit/{r}" for r in range(world)]
        store.wait(keys, datetime.timedelta(minutes=30))
        codes = [int(store.get(k)) for k in keys]
        if all(c == 0 for c in codes):
            code = 0
            break
        if PREFLIGHT_EXIT not in codes or i + 1 == len(attempts):
            code = code or next(c for c in codes if c != 0)
            break
    dist.barrier()
    dist.destroy_process_group()
    return code if code >= 0 else 1


def ttft_probe(model: str, lengths: list, seed: int = 0, repeats: int = 3) -> dict:
    """Batch-1 prefill latency of the whole model at each prompt length (outside the timed
    decode region; scripts/latency_sweep.py is the full sweep). Returns {length: ms}."""
    import statistics

    import torch

    from llm_sharding_amd.config import get_preset
    from llm_sharding_amd.runtime.engine import RandomSource, StageEngine

    cfg = get_preset(model)
    dev = torch.device("cuda", 0)
    eng = StageEngine(cfg, 0, cfg.num_hidden_layers, dev, torch.bfloat16, has_embed=True, has_head=True,
                      source=RandomSource(cfg, seed), max_slots=1, max_seq=max(lengths) + 8,
                      max_prefill_rows=max(lengths))
    g = torch.Generator().manual_seed(seed)
    out = {}
    for P in lengths:
        ts = []
        for _ in range(repeats + 1):
            ids = torch.randint(3, cfg.vocab_size, (P,), generator=g).to(dev)
            eng.reset()
            torch.cuda.synchronize()
            t = time.perf_counter()
            sl, po = eng.prefill_rows([0], [P])
            tok = eng.head(eng.forward(eng.embed(ids), sl, po), [P - 1])
            int(tok[0])
            ts.append((time.perf_counter() - t) * 1e3)
        out[str(P)] = round(statistics.median(ts[1:]), 3)
    del eng
    torch.cuda.empty_cache()
    return out


def extra_runs(spec: str, a) -> dict:
    """Operating-range points measured by the same run as the headline (outside its timed
    region, one GPU): other model families at the bench batch, and one pipeline stage of a
    model too big for one GPU (the 70B 10-layer stage of the 8-stage plan, 8 micro-batches)."""
    import gc

    import torch

    from llm_sharding_amd.parallel.pipeline import run_decode_benchmark
    out = {}
    for item in [x.strip() for x in spec.split(",") if x.strip()]:
        model, _, layers = item.partition(":")
        nl = int(layers) if layers else 0
        key = f"{model}_stage{nl}_mb8" if nl else model
        try:
            r = run_decode_benchmark(model=model, n_gpus=1, steps=8 if nl else 16, warmup=2 if nl else 4,
                                     batch=a.batch, prompt_len=a.prompt_len, seed=a.seed, verbose=False,
                                     stage_layers=nl, microbatches=8 if nl else 0)
            out[key] = {"tok_s": round(r["tok_s"], 1), "ms_per_step": round(r["ms_per_step"], 3),
                        "global_batch": r["global_batch"]}
            if nl:  # tok_s = the whole pipeline's rate if every stage ran like this one
                out[key]["kind"] = "stage_profile"
        except Exception as e:  # a side measurement never costs the headline line
            out[key] = {"error": f"{type(e).__name__}: {e}"[:200]}
        gc.collect()
        torch.cuda.empty_cache()
    return out


def main():
    _die_with_parent()  # a child of spawn_ranks / supervise: die with that parent
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus != world and world != 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(spawn_ranks(a.gpus))
    if world > 1 and os.environ.get("LSA_BENCH_ROLE") != "worker" and a.supervise:
        raise SystemExit(supervise(a, sys.argv[1:]))
    if a.trace:
        os.environ["LSA_TRACE"] = a.trace
    from llm_sharding_amd.parallel.pipeline import run_decode_benchmark
    res = run_decode_benchmark(model=a.model, n_gpus=a.gpus, steps=a.steps, warmup=a.warmup,
                               batch=a.batch, prompt_len=a.prompt_len, max_seq=a.max_seq,
                               microbatches=a.microbatches, seed=a.seed, use_graph=not a.no_graph,
                               weight_dtype=a.weight_dtype, streams=a.streams, dp=a.dp,
                               latency_steps=a.latency_steps, device=a.device, stage_layers=a.stage_layers,
                               transport=a.transport, mid_batch=a.mid_batch)
    if res is None:  # non-zero ranks
        return
    line = {
        "metric": "stage_profile_tokens_per_sec" if a.stage_layers else "output_tokens_per_sec_whole_node",
        "value": round(res["tok_s"], 2),
        "unit": "tokens/s",
        "n_gpus": a.gpus,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(res["ms_per_step"], 4),
        "higher_is_better": True,
        "scaling": "weak",
        # the reference publishes no benchmark number (its only figure is a ~4.3 tok/s
        # code-comment anecdote on other hardware, kept below as reference_anecdote_tok_s)
        "vs_baseline": None,
        "dtype": "bf16" if a.weight_dtype == "bf16" else "bf16 activations, fp8-e4m3 weights (W8A16)",
        "data": f"synthetic prompts, random-init weights ({res['model_name']} architecture)",
        "config": {"model": res["model_name"], "global_batch": res["global_batch"],
                   "seq_len": a.prompt_len + a.warmup + a.steps,
                   "parallelism": f"dp{res['dp']}_pp{res['pp']}" if res["dp"] > 1 else f"pp{res['pp']}", "microbatches": res["microbatches"],
                   "batch_per_microbatch": a.batch, "prompt_len": a.prompt_len,
                   "concurrent_streams": res["streams"], "max_seq": res["max_seq"]},
        "p50_tpot_ms": round(res["p50_tpot_ms"], 4),
        "p90_tpot_ms": round(res["p90_tpot_ms"], 4),
        "ttft_ms": round(res["ttft_ms"], 3),
        "b1_p50_tpot_ms": None if res["b1_p50_tpot_ms"] is None else round(res["b1_p50_tpot_ms"], 4),
        "b1_tok_s": None if res["b1_tok_s"] is None else round(res["b1_tok_s"], 2),
        "mid_batch": res["mid_batch"],
        "mid_p50_tpot_ms": None if res["mid_p50_tpot_ms"] is None else round(res["mid_p50_tpot_ms"], 4),
        "mid_tok_s": None if res["mid_tok_s"] is None else round(res["mid_tok_s"], 2),
        "mem_pred_gb": res["mem_pred_gb"], "mem_peak_gb": res["mem_peak_gb"],
        "reference_anecdote_tok_s": BASELINE_TOK_S,
    }
    if res.get("transport"):
        line["config"]["transport"] = res["transport"]
        line["transport"] = res["transport"]
        line["fallback"] = os.environ.get("LSA_BENCH_FALLBACK") == "1"
        line["preflight_us"] = res.get("preflight_us")
    topo = res.get("topology")
    if topo:  # proof of placement: process-group size, each rank's device UUID / PCI id, edge transports
        line["dist"] = topo
    lens = [int(x) for x in str(a.ttft_lens).split(",") if x.strip() and int(x) > 0]
    if lens and a.gpus == 1 and a.device == "cuda" and not a.stage_layers:
        try:
            line["ttft_prompt_ms"] = ttft_probe(a.model, lens, seed=a.seed)
        except Exception as e:  # never lose the headline line to the side measurement
            line["ttft_prompt_ms"] = None
            line["ttft_error"] = f"{type(e).__name__}: {e}"[:200]
    if a.extras and a.gpus == 1 and a.device == "cuda" and not a.stage_layers:
        line["extra"] = extra_runs(a.extras, a)
    from llm_sharding_amd.utils.runtime_config import knobs_in_effect
    line["knobs"] = knobs_in_effect()  # LSA_* switches set for this run ({} = the product defaults)
    if res.get("tokens_mb0"):  # parity digest across layouts (same prompts -> same tokens)
        import hashlib
        line["tokens_mb0_sha16"] = hashlib.sha256(json.dumps(res["tokens_mb0"]).encode()).hexdigest()[:16]
    print(json.dumps(line), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(line, f)


if __name__ == "__main__":
    main()
