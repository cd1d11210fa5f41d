#!/usr/bin/env python3
"""Headline benchmark: output tokens/s + p50 TTFT of the Llama-3-8B *service*
(BASELINE.json metric: "Llama-3-8B K8s service") on N MI355X GPUs of one node.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 the
driver launches one rank per GPU with torch.distributed.run.  One *step* is one
serving wave: ``--num-prompts`` requests (synthetic random token prompts of
``--input-len`` tokens, ``--output-len`` generated tokens each, ignore_eos, temperature
1.0 sampling) arrive at once and are served until every request has finished -- the
vLLM ``benchmark_serving`` request-rate=inf shape.

``--mode service`` (default) measures what a client of ``svc/vllm-router-service``
gets (/root/reference/old_README.md:1175,1473-1476): every replica-leading rank starts
the OpenAI API server (engine core + API processes) and a router in front of it as
fresh child processes (this process never touches the GPU, so nothing GPU-initialised
is ever forked or exec'd), then streams the waves over HTTP/SSE through the router.
TTFT is client send -> first SSE event.  The timed region is bracketed by a barrier
over all ranks on both sides; it ends when the last stream of the last wave has been
read, i.e. after the engine's final step has finished on the GPU and its tokens have
reached the client (the service-level equivalent of synchronize()).  The engine-level
figures of the same requests (arrival at the engine core -> first token / finish,
from ``GET /kgc/engine_stats``) are reported next to them as ``engine_*`` keys.

``--mode engine`` drives ``LLMEngine.step()`` in-process instead (no HTTP): the
engine-only ceiling of the same waves.

Parallelism: ``dpN`` (default) runs one engine replica per GPU, like the reference's
``replicaCount`` DP deployment behind the router (values-01-minimal-example2.yaml:10);
per-GPU work is fixed, so scaling is weak.  ``--tp N`` runs one tensor-parallel
engine over N GPUs (RCCL/xGMI all-reduce) per replica instead.
Weights are random-init bf16 of the real architecture (no checkpoints offline).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = "output tokens/sec + p50 TTFT, Llama-3-8B K8s service at 1/2/4/8 MI355X"
_METRIC_NAMES = {"llama-3-8b": "Llama-3-8B", "llama-3-70b": "Llama-3-70B",
                 "mixtral-8x7b": "Mixtral-8x7B"}


def metric_name(model: str) -> str:
    """BASELINE.json's metric string for its model; the same shape, naming the model that
    actually ran, for every other one (a 70B run is never labelled Llama-3-8B)."""
    if model == "llama-3-8b":
        return BASELINE_METRIC
    return BASELINE_METRIC.replace("Llama-3-8B", _METRIC_NAMES.get(model, model))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--num-prompts", type=int, default=256, help="requests per wave per replica")
    ap.add_argument("--input-len", type=int, default=512)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-num-batched-tokens", type=int, default=16384)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--moe-parallel", default="tp", choices=["tp", "ep"],
                    help="Mixtral expert placement over the TP group (engine --moe-parallel)")
    ap.add_argument("--enforce-eager", action="store_true")
    ap.add_argument("--gpu-memory-utilization", type=float, default=0.90)
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--num-gpu-blocks-override", type=int, default=None,
                    help="fixed KV blocks per replica (replicas sharing one GPU: KGC_BENCH_DEVICES)")
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--prefix-caching", type=int, default=1, choices=[0, 1],
                    help="automatic prefix caching (engine default: on; random prompts never hit)")
    ap.add_argument("--prefill-first", dest="prefill_first", action="store_true", default=True,
                    help="engine scheduling (default, as in deploy/values/values-llama3-8b-"
                         "tp1.yaml): decodes sit out while prompts wait for a slot")
    ap.add_argument("--no-prefill-first", dest="prefill_first", action="store_false")
    ap.add_argument("--log-level", default="WARNING",
                    help="python logging level on stderr (INFO shows the GEMM tuner's choices)")
    ap.add_argument("--mode", default="service", choices=["service", "engine"],
                    help="service: HTTP/SSE through API server + router (headline); "
                         "engine: LLMEngine.step() in-process")
    ap.add_argument("--api-server-count", type=int, default=0,
                    help="service mode: API processes per engine (0: server default)")
    ap.add_argument("--startup-timeout", type=float, default=1800)
    ap.add_argument("--no-comm-probe", dest="comm_probe", action="store_false", default=True,
                    help="service mode, N > 1: skip the RCCL / xGMI all-reduce probe that runs "
                         "after the timed waves (benchmarks/comm_probe.py)")
    ap.add_argument("--router-workers", type=int, default=0,
                    help="service mode: router processes in front of all replicas "
                         "(0: one per replica, at most 16)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: run the same harness on the fp32 CPU path (gloo) -- a test "
                         "harness for the multi-rank logic, not a measurement")
    return ap.parse_args()


def _k9_plan() -> dict:
    from kubernetes_gpu_cluster_amd.ops import gemm
    return gemm.plan()


def _k9m_plan() -> dict:
    from kubernetes_gpu_cluster_amd.ops import gemm
    return gemm.dgemm_plan()


def _k9m_top() -> dict:
    """The K9m selections at the largest decode M (the batch-256 step), "NxK:kind" ->
    [cfg, S]: which kernels the timed decode steps ran."""
    plan = _k9m_plan()
    if not plan:
        return {}
    mx = max(k[0] for k in plan)
    return {f"{n}x{k}:{kind}": list(v) for (m, n, k, kind), v in sorted(plan.items()) if m == mx}


def run_wave(engine, args, wave: int, rank: int):
    from kubernetes_gpu_cluster_amd.engine.sequence import SamplingParams
    g = torch.Generator().manual_seed(1000 * wave + rank)
    vocab = engine.mcfg.vocab_size
    sp = SamplingParams(temperature=args.temperature, top_p=1.0, max_tokens=args.output_len,
                        ignore_eos=True)
    t0 = time.monotonic()
    seqs = []
    for i in range(args.num_prompts):
        ids = torch.randint(100, vocab - 100, (args.input_len,), generator=g).tolist()
        seqs.append(engine.add_request(ids, sp, request_id=f"w{wave}-r{rank}-{i}", arrival_time=t0))
    steps = 0
    while engine.has_unfinished():
        engine.step()
        steps += 1
    t1 = time.monotonic()
    out_toks = sum(len(s.output_token_ids) for s in seqs)
    ttfts = [s.first_token_time - s.arrival_time for s in seqs]
    tpots = [(s.last_token_time - s.first_token_time) / max(1, len(s.output_token_ids) - 1)
             for s in seqs]
    return out_toks, t1 - t0, ttfts, tpots, steps


def main_engine(args):
    import logging
    logging.basicConfig(level=getattr(logging, args.log_level.upper(), logging.WARNING),
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    n = world if world > 1 else 1
    if args.gpus != n and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    cpu = args.device == "cpu"
    if cpu:
        dev = torch.device("cpu")
        args.dtype = "float32"
    else:
        assert torch.cuda.is_available(), "bench.py needs a GPU (or --device cpu)"
        dev = torch.device("cuda", local_rank)
        torch.cuda.set_device(dev)
    tp = args.tp
    if world > 1:
        if cpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    from kubernetes_gpu_cluster_amd.engine.config import EngineConfig
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLMEngine
    from kubernetes_gpu_cluster_amd.engine.worker import ExternalExecutor, Worker, worker_loop
    cfg = EngineConfig(model=args.model, dtype=args.dtype, tensor_parallel_size=tp,
                       max_model_len=args.max_model_len, max_num_seqs=args.max_num_seqs,
                       max_num_batched_tokens=args.max_num_batched_tokens,
                       gpu_memory_utilization=args.gpu_memory_utilization,
                       enforce_eager=args.enforce_eager, random_init=True, seed=0,
                       device=args.device, enable_prefix_caching=bool(args.prefix_caching),
                       prefill_first=args.prefill_first, moe_parallel=args.moe_parallel,
                       allow_phantom=args.mode == "engine")
    engine = None
    if tp > 1:
        assert world % tp == 0
        w = Worker(cfg, rank=rank, local_device=local_rank)
        if w.ps.rank == 0:
            engine = LLMEngine(cfg, ExternalExecutor(w))
        else:
            worker_loop(w)
    else:
        engine = LLMEngine(cfg)
    replicas = world // tp
    is_driver = engine is not None

    def barrier():
        if not cpu:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    res = None
    if is_driver:
        for wv in range(args.warmup):
            run_wave(engine, args, -1 - wv, rank)
    barrier() if tp == 1 else None
    t0 = time.monotonic()
    toks, ttfts, tpots, steps, wall = 0, [], [], 0, 0.0
    if is_driver:
        for wv in range(args.steps):
            o, dt, tt, tp_, st = run_wave(engine, args, wv, rank)
            toks += o
            ttfts += tt
            tpots += tp_
            steps += st
    if tp == 1:
        barrier()
    elapsed = time.monotonic() - t0
    from kubernetes_gpu_cluster_amd.parallel import comm
    # the all-reduce policy this node's start-up calibration chose (read before shutdown
    # releases the xGMI buffers)
    ar_cal = getattr(comm.get_custom_allreduce(), "calibration", None)
    host_t = engine.host_timing() if is_driver and hasattr(engine, "host_timing") else None
    if is_driver:
        engine.shutdown()
    # aggregate over replicas (drivers) -- every rank participates in the collectives
    if world > 1:
        t = torch.tensor([elapsed if is_driver else 0.0, float(toks), float(steps)],
                         dtype=torch.float64, device=dev)
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, toks, steps = tmax[0].item(), int(t[1].item()), int(t[2].item())
        gathered = [None] * world
        dist.all_gather_object(gathered, (ttfts, tpots))
        ttfts = [x for g in gathered for x in g[0]]
        tpots = [x for g in gathered for x in g[1]]
    if rank == 0:
        value = toks / elapsed
        p50_ttft = statistics.median(ttfts) * 1e3 if ttfts else None
        # KGC_TP_PHANTOM=N: ONE rank of a TP = N model on one GPU (parallel/state.py
        # init_phantom) -- a per-rank measurement, never a TP = N service figure
        phantom = int(os.environ.get("KGC_TP_PHANTOM", "0") or 0)
        out = {
            "metric": metric_name(args.model), "value": round(value, 2), "unit": "output_tokens/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": {"bfloat16": "bf16", "float16": "fp16", "float32": "fp32"}.get(args.dtype, args.dtype),
            "data": "synthetic random-token prompts, random-init weights",
            "p50_ttft_ms": round(p50_ttft, 2) if p50_ttft else None,
            "p50_tpot_ms": round(statistics.median(tpots) * 1e3, 3) if tpots else None,
            "engine_steps": steps,
            "k9_skinny_gemm_shapes": len(_k9_plan()),
            "k9m_gemm_shapes": len(_k9m_plan()),
            "k9m_plan_max_m": _k9m_top(),
            **({"host_us_per_step": host_t} if host_t else {}),
            "config": {"model": args.model, "global_batch": args.num_prompts * replicas,
                       "seq_len": args.input_len + args.output_len, "input_len": args.input_len,
                       "output_len": args.output_len,
                       "parallelism": (f"tp{phantom}-phantom-rank0" if phantom > 1 else
                                       f"dp{replicas}" if tp == 1 else
                                       f"tp{tp}" + (f"xdp{replicas}" if replicas > 1 else "")),
                       "max_num_seqs": args.max_num_seqs,
                       "max_num_batched_tokens": args.max_num_batched_tokens,
                       "cuda_graphs": not args.enforce_eager,
                       "scheduling": "prefill-first" if args.prefill_first else "decode-first"},
        }
        if tp > 1:
            out["ar_calibration"] = ar_cal
        if phantom > 1:
            out["phantom_tp"] = phantom
            out["data"] += "; ONE phantom TP rank (peers contribute zeros): per-rank timing only"
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _note(msg: str) -> None:
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


_port_locks: list = []


def _free_port(local_rank: int, slot: int) -> int:
    """A free port from this rank's own range (ranks of one node never race for the
    same number): 18000 + 64 * local_rank + slot, stepping by 1024 when busy.  The port
    is also claimed by an flock on a per-port file held for this process's lifetime: the
    API server binds with SO_REUSEPORT (its --api-server-count frontends share the port)
    and loads its model before it binds, so a second bench on the same host that probed
    the same still-unbound port would otherwise join the same port and the kernel would
    spread each job's requests over both jobs' servers (seen as a bench whose
    /kgc/engine_stats missed requests its client had completed)."""
    import fcntl
    import socket
    import tempfile
    for step in range(16):
        port = 18000 + 64 * local_rank + slot + 1024 * step
        f = open(os.path.join(tempfile.gettempdir(), f"kgc-bench-port-{port}.lock"), "a")
        try:
            fcntl.flock(f, fcntl.LOCK_EX | fcntl.LOCK_NB)
        except OSError:
            f.close()
            continue
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                f.close()
                continue
        _port_locks.append(f)
        return port
    raise RuntimeError(f"no free port for rank {local_rank}")


def _server_devices(local_rank: int, tp: int, cpu: bool):
    """HIP_VISIBLE_DEVICES of one replica: GPUs local_rank .. local_rank+tp-1 of what
    this process may see (None on the CPU path)."""
    if cpu:
        return None
    # KGC_BENCH_DEVICES="0,0": rehearse several replicas on one GPU (each replica's
    # --gpu-memory-utilization share must then fit beside the others')
    vis = (os.environ.get("KGC_BENCH_DEVICES") or os.environ.get("HIP_VISIBLE_DEVICES")
           or os.environ.get("CUDA_VISIBLE_DEVICES"))
    ids = vis.split(",") if vis else [str(i) for i in range(local_rank + tp)]
    return ",".join(ids[local_rank:local_rank + tp])


def _engine_args(args, cpu: bool) -> list:
    ea = ["--load-format", "dummy", "--dtype", args.dtype, "--seed", "0",
          "--tensor-parallel-size", str(args.tp), "--moe-parallel", args.moe_parallel,
          "--max-model-len", str(args.max_model_len), "--max-num-seqs", str(args.max_num_seqs),
          "--max-num-batched-tokens", str(args.max_num_batched_tokens),
          "--gpu-memory-utilization", str(args.gpu_memory_utilization),
          "--disable-log-requests"]
    if args.num_gpu_blocks_override:
        ea += ["--num-gpu-blocks-override", str(args.num_gpu_blocks_override)]
    if not args.prefix_caching:
        ea.append("--no-enable-prefix-caching")
    if args.enforce_eager:
        ea.append("--enforce-eager")
    if args.prefill_first:
        ea.append("--prefill-first")
    if args.api_server_count:
        ea += ["--api-server-count", str(args.api_server_count)]
    if cpu:
        ea += ["--device", "cpu"]
    return ea


def main_service(args):
    """One replica per ``tp`` ranks: the leading rank launches API server + router and
    drives its own client; every rank joins the barriers and the aggregation (gloo,
    CPU only -- this process never initialises the GPU)."""
    import asyncio
    import urllib.request
    from kubernetes_gpu_cluster_amd.benchmarks import serving_client as sc
    from kubernetes_gpu_cluster_amd.models.configs import resolve_model
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = args.device == "cpu"
    if cpu:
        args.dtype = "float32"
    tp = args.tp
    assert world % tp == 0, f"WORLD_SIZE {world} is not a multiple of --tp {tp}"
    replicas = world // tp
    leader = rank % tp == 0
    if world > 1:
        import datetime
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=args.startup_timeout + 600))
    vocab = resolve_model(args.model)[0].vocab_size
    procs, logs = [], []
    api_url = url = None
    res_all, windows, eng = [], [], {}
    elapsed = 0.0
    router = None
    cpu0 = 0.0
    try:
        if leader:
            api_port = _free_port(local_rank, 0)
            api_url = f"http://127.0.0.1:{api_port}"
            procs.append(sc.start_api_server(args.model, api_port,
                                             _server_devices(local_rank, tp, cpu),
                                             _engine_args(args, cpu)))
            _note(f"rank {rank}: API server {api_url} (tp {tp}); waiting for health")
            asyncio.run(sc.wait_healthy([api_url], args.startup_timeout, procs, _note))
        # ONE service endpoint for the whole job, as the reference deploys DP:
        # replicaCount engine pods behind one vllm-router-service
        # (/root/reference/values-01-minimal-example2.yaml:10,23-49).  Rank 0 runs the
        # router over every replica's API server; every replica's client load goes
        # through it.
        backends = [api_url]
        if world > 1:
            allu = [None] * world
            dist.all_gather_object(allu, api_url)
            backends = [u for u in allu if u]
        if rank == 0:
            workers = args.router_workers or max(1, min(16, len(backends)))
            router_port = _free_port(local_rank, 1)
            url = f"http://127.0.0.1:{router_port}"
            router = sc.start_router(router_port, backends, workers=workers)
            procs.append(router)
            _note(f"router {url}: {workers} worker process(es) over {len(backends)} "
                  f"replica(s); waiting for health")
            asyncio.run(sc.wait_healthy([url], args.startup_timeout, procs, _note))
            _note("service is up")
        if world > 1:
            box = [url]
            dist.broadcast_object_list(box, src=0)
            url = box[0]

        def make_prompts(n: int, base_seed: int):
            # generated before any timer starts (~0.1 s of Python per 256 x 512 wave)
            return [sc.random_prompts(args.num_prompts, args.input_len, vocab,
                                      seed=base_seed + 1000 * w + rank) for w in range(n)]

        async def run_all():
            """Warmup and timed waves on ONE client session (its keep-alive connections
            are reused, as a long-lived client's are); the barriers block the loop on
            purpose -- nothing else runs on it between waves."""
            warm = make_prompts(args.warmup, 7_000_000) if leader else []
            timed = make_prompts(args.steps, 0) if leader else []
            out = []
            async with sc.new_session() as s:
                for prompts in warm:
                    r, _, _ = await sc.run_wave(s, url, args.model, prompts, args.output_len,
                                                temperature=args.temperature)
                    bad = [x for x in r if not x.ok]
                    if bad:
                        raise RuntimeError(f"warmup: {len(bad)} requests failed "
                                           f"(status {bad[0].status})")
                # engine-side window opens at the LAST rank's barrier entry: every warmup
                # request arrived before it, every timed one after (a rank that leaves the
                # barrier early may send before this rank's t0)
                t_lo = time.monotonic()
                if world > 1:
                    ents = [None] * world
                    dist.all_gather_object(ents, t_lo)
                    t_lo = max(ents)
                t0 = time.monotonic()
                c0 = sc.cpu_seconds(router.pid) if router is not None else 0.0
                for prompts in timed:
                    out.append(await sc.run_wave(s, url, args.model, prompts, args.output_len,
                                                 temperature=args.temperature))
                if world > 1:
                    dist.barrier()
                t1 = time.monotonic()
                c1 = sc.cpu_seconds(router.pid) if router is not None else 0.0
                return out, t0, t1 - t0, c1 - c0, t_lo

        waves_out, t0, elapsed, router_cpu, t_lo = asyncio.run(run_all())
        for r, lo, hi in waves_out:
            res_all += r
        # one window over all timed waves: behind the shared router a replica also serves
        # other ranks' requests, whose waves need not line up with this rank's
        windows.append((min(t_lo, t0), t0 + elapsed))
        if leader:
            with urllib.request.urlopen(f"{api_url}/kgc/engine_stats?since={t_lo - 1.0}", timeout=30) as f:
                st = json.loads(f.read())
            eng = sc.engine_figures(st["requests"], windows)
            eng["steps"] = st["steps"]
    finally:
        codes = sc.stop(procs)
        if leader and procs:
            _note(f"rank {rank}: service stopped (exit codes {codes})")
    probe = None
    devs = [d for d in os.environ.get("KGC_BENCH_DEVICES", "").split(",") if d]
    shared = len(devs) > len(set(devs))
    if world > 1 and not cpu and args.comm_probe and not shared:
        # (replicas sharing one GPU: RCCL takes one rank per device, so no probe)
        probe = _comm_probe(rank, world, local_rank)
    ok = [r for r in res_all if r.ok]
    mine = {"toks": sum(r.tokens for r in ok), "failed": len(res_all) - len(ok),
            "ttft": [r.ttft for r in ok], "tpot": [(r.e2e - r.ttft) / max(1, r.tokens - 1) for r in ok],
            "itl": [x for r in ok for x in r.itl], "elapsed": elapsed if leader else 0.0,
            "eng": eng}
    parts = [mine]
    if world > 1:
        parts = [None] * world
        dist.all_gather_object(parts, mine)
    if rank == 0:
        elapsed = max(p["elapsed"] for p in parts)
        toks = sum(p["toks"] for p in parts)
        failed = sum(p["failed"] for p in parts)
        ttft = [x for p in parts for x in p["ttft"]]
        tpot = [x for p in parts for x in p["tpot"]]
        itl = [x for p in parts for x in p["itl"]]
        engs = [p["eng"] for p in parts if p["eng"]]
        e_tok = sum(e["engine_tokens"] for e in engs)
        e_span = max((e["engine_span_s"] for e in engs), default=0.0)
        e_ttft = [x for e in engs for x in e["engine_ttft"]]
        e_tpot = [x for e in engs for x in e["engine_tpot"]]
        value = toks / elapsed if elapsed > 0 else 0.0
        e_value = e_tok / e_span if e_span > 0 else None
        med = lambda xs: round(statistics.median(xs) * 1e3, 3) if xs else None  # noqa: E731
        out = {
            "metric": metric_name(args.model), "value": round(value, 2), "unit": "output_tokens/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": {"bfloat16": "bf16", "float16": "fp16", "float32": "fp32"}.get(args.dtype, args.dtype),
            "data": "synthetic random-token prompts, random-init weights",
            "mode": "service (client -> router -> OpenAI API server -> engine core, HTTP/SSE)",
            "p50_ttft_ms": med(ttft),
            "p99_ttft_ms": round(sorted(ttft)[int(0.99 * (len(ttft) - 1))] * 1e3, 2) if ttft else None,
            "p50_tpot_ms": med(tpot), "p50_itl_ms": med(itl),
            "completed": len(ttft), "failed": failed,
            "engine_tok_s": round(e_value, 2) if e_value else None,
            "engine_p50_ttft_ms": med(e_ttft), "engine_p50_tpot_ms": med(e_tpot),
            "engine_output_tokens": e_tok,
            "engine_steps": sum(e.get("steps", 0) for e in engs),
            "service_vs_engine": round(value / e_value, 4) if e_value else None,
            # router CPU-seconds per wall second over the timed waves (all its workers)
            "router_cpu_util": round(router_cpu / elapsed, 3) if elapsed > 0 else None,
            "router_workers": args.router_workers or max(1, min(16, replicas)),
            # after the timed waves, outside the timed region: RCCL all-reduce bus
            # bandwidth and the xGMI kernel vs RCCL on this node's GPUs (N > 1)
            "comm_probe": probe,
            "config": {"model": args.model, "global_batch": args.num_prompts * replicas,
                       "seq_len": args.input_len + args.output_len, "input_len": args.input_len,
                       "output_len": args.output_len,
                       "parallelism": f"dp{replicas}" if tp == 1 else f"tp{tp}" + (f"xdp{replicas}" if replicas > 1 else ""),
                       "max_num_seqs": args.max_num_seqs,
                       "max_num_batched_tokens": args.max_num_batched_tokens,
                       "cuda_graphs": not args.enforce_eager,
                       "scheduling": "prefill-first" if args.prefill_first else "decode-first",
                       "endpoint": f"one router ({replicas} replica(s)) -> /v1/completions "
                                   f"(stream)"},
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if failed_any(parts if rank == 0 else [mine]):
        sys.exit(1)


def _comm_probe(rank: int, world: int, local_rank: int, timeout_s: float = 240.0):
    """benchmarks/comm_probe.py on every rank's GPU (the API servers are stopped), as a
    child process with a hard time limit so a collective that never completes cannot
    hold up the benchmark's own result.  Returns rank 0's table (None elsewhere)."""
    import signal
    import subprocess
    import tempfile
    from kubernetes_gpu_cluster_amd.benchmarks import serving_client as sc
    box = [_free_port(local_rank, 2) if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    out = os.path.join(tempfile.gettempdir(), f"kgc_comm_probe_{os.getpid()}.json")
    cmd = [sys.executable, "-m", "kubernetes_gpu_cluster_amd.benchmarks.comm_probe",
           "--rank", str(rank), "--world", str(world), "--port", str(box[0]),
           "--device", str(local_rank)] + (["--out", out] if rank == 0 else [])
    _note(f"rank {rank}: collective probe (RCCL + xGMI all-reduce, world {world})")
    p = subprocess.Popen(cmd, env=sc._env({}), start_new_session=True,
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        _, err = p.communicate(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        return {"error": f"timed out after {timeout_s:.0f} s"} if rank == 0 else None
    if rank != 0:
        return None
    if p.returncode != 0:
        return {"error": f"exit {p.returncode}: {(err or '')[-400:]}"}
    try:
        with open(out) as f:
            return json.loads(f.read())
    except (OSError, ValueError) as e:
        return {"error": str(e)}
    finally:
        if os.path.exists(out):
            os.remove(out)


def failed_any(parts) -> bool:
    return any(p["failed"] for p in parts)


def main():
    args = parse()
    if args.mode == "engine":
        main_engine(args)
    else:
        main_service(args)


if __name__ == "__main__":
    main()
