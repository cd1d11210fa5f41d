"""Workers and executors: one process per GPU, TP x PP inside a pod.

The reference scales a model over GPUs by handing vLLM ``--tensor-parallel-size``
/ ``--pipeline-parallel-size`` (and a Ray head for multi-pod PP:
``values-01-minimal-example4.yaml:17-18,42-46``).  Here the driver process (rank 0)
owns the scheduler; every rank owns one GPU and a ``Worker`` (model shard +
``ModelRunner``).  Control commands (profile, init cache, capture, shutdown) and
per-step ``StepPlan`` blobs travel over a gloo CPU group; activations and TP
collectives go over RCCL/xGMI.

Executors:
  * LocalExecutor      TP = PP = 1, in-process.
  * MultiprocExecutor  spawns ranks 1..N-1 (``torch.multiprocessing``, spawn) for
                       the API server / offline LLM.
  * ExternalExecutor   ranks already launched by torchrun (bench.py --tp N):
                       rank 0 drives, the others call ``worker_loop``.
"""
from __future__ import annotations

import logging
import os
import pickle
import socket
import traceback
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..models import load_model, resolve_model
from ..models.moe import set_moe_mode
from ..parallel import comm
from .health import RankWatchdog, watch_parent
from ..parallel.state import (destroy_parallel, get_state, init_parallel, init_phantom,
                              phantom_tp)
from .config import EngineConfig
from .model_runner import ModelRunner, StepPlan

log = logging.getLogger("kgc.worker")

CMD_STEP, CMD_PROFILE, CMD_INIT_CACHE, CMD_CAPTURE, CMD_EXIT = 1, 2, 3, 4, 5
N_HDR = 12                  # StepPlan.header() fields


def default_max_model_len(cfg: EngineConfig) -> int:
    mcfg, _ = resolve_model(cfg.model)
    return cfg.max_model_len or mcfg.max_position


def _fault_perturb_shard(model, ps) -> None:
    """Fault injection for the TP parity oracles (tests/test_engine_gpu.py): with
    KGC_FAULT_PERTURB_TP_RANK=r, TP rank r adds noise to its shard of every o_proj weight
    after loading -- one wrong shard, which a teacher-forced comparison against TP = 1
    must catch.  Armed only together with KGC_TESTING=1 (the test sets both), so the
    variable alone -- left in a deployment by accident -- changes nothing but a warning."""
    r = os.environ.get("KGC_FAULT_PERTURB_TP_RANK")
    if r is None or ps.tp_size == 1 or int(r) != ps.tp_rank:
        return
    if os.environ.get("KGC_TESTING") != "1":
        log.warning("KGC_FAULT_PERTURB_TP_RANK ignored: fault injection needs KGC_TESTING=1")
        return
    g = torch.Generator(device="cpu").manual_seed(1234)
    with torch.no_grad():
        for name, p in model.named_parameters():
            if name.endswith("o_proj.weight"):
                noise = torch.randn(p.shape, generator=g).to(p.device, p.dtype)
                p.add_(noise * p.float().std().item())
    log.warning("fault injection: TP rank %s perturbed its o_proj shards", r)


class Worker:
    def __init__(self, cfg: EngineConfig, rank: int = 0, local_device: Optional[int] = None):
        self.cfg = cfg
        dev = cfg.resolved_device()
        if dev.type == "cuda":
            idx = local_device if local_device is not None else int(os.environ.get("LOCAL_RANK", rank))
            idx = idx % max(1, torch.cuda.device_count())
            dev = torch.device("cuda", idx)
            torch.cuda.set_device(dev)
            ops.load_extension(strict=True)
        self.device = dev
        self.rank = rank
        set_moe_mode(cfg.moe_parallel)
        init_parallel(cfg.tensor_parallel_size, cfg.pipeline_parallel_size, device=dev)
        ph = phantom_tp()
        if ph > 1:
            # KGC_TP_PHANTOM=N: this single process is rank 0 of a TP = N model (one GPU
            # stands in for a TP node's rank: parallel/state.py init_phantom)
            if not cfg.allow_phantom:
                raise ValueError(
                    "KGC_TP_PHANTOM is set: a phantom TP rank serves rank 0's shard with zero "
                    "peers (wrong completions by construction). It is a per-rank measurement "
                    "mode for bench.py --mode engine and the tests only; unset it to serve.")
            if cfg.tensor_parallel_size * cfg.pipeline_parallel_size != 1 or dev.type != "cuda":
                raise ValueError("KGC_TP_PHANTOM needs one GPU process (tp = pp = 1)")
            log.warning("PHANTOM TP rank 0 of %d: per-rank timing only, outputs are not a "
                        "model's", ph)
            init_phantom(ph, dev)
        self.ps = get_state()
        # non-driver ranks of a multi-rank engine heart-beat into the rendezvous store
        # (engine/health.py): the driver notices a rank on another node dying, and this
        # rank notices the driver's node dying
        self.heartbeat = None
        self.hb_store = None
        if self.ps.tp_size * self.ps.pp_size > 1 and dist.is_initialized():
            # one store per replica, hosted by its driver (engine/health.py replica_store);
            # created before the weights load, so no rank waits on another's loading
            from .health import Heartbeat, replica_store
            self.hb_store = replica_store(self.ps)
            if self.hb_store is not None and dist.get_rank() != getattr(self.ps, "global_base", 0):
                self.heartbeat = Heartbeat(self.hb_store, dist.get_rank()).start()
        mcfg, _ = resolve_model(cfg.model)
        self.dtype = cfg.torch_dtype(torch.bfloat16 if mcfg.arch != "opt" else torch.float16)
        if dev.type == "cpu" and self.dtype == torch.float16:
            self.dtype = torch.float32       # CPU oracle path
        self.max_model_len = default_max_model_len(cfg)
        if dev.type == "cuda":
            from ..utils.gemm_tuning import enable_tuned_gemms
            enable_tuned_gemms(mcfg.name, self.ps.tp_size)
        torch.manual_seed(cfg.seed)
        self.mcfg, self.model = load_model(cfg.model, self.dtype, dev, cfg.random_init,
                                           seed=cfg.seed)
        _fault_perturb_shard(self.model, self.ps)
        if dev.type == "cuda" and not cfg.enforce_eager:
            # packed copies of the decode-GEMM weights for the K9m tiles, made before the
            # KV cache is sized so the pool accounts for them (ops/gemm.py)
            from ..ops import gemm
            silu = list(getattr(self.model, "silu_weights", lambda: [])())
            skip = {id(x) for x in silu}
            tied = getattr(self.mcfg, "tie_embeddings", False)
            ws = [p for n, p in self.model.named_parameters() if p.dim() == 2
                  and id(p) not in skip and (tied or "embed" not in n)]
            gemm.pack_decode_weights(ws, silu)
        if dev.type == "cuda":
            # K14m's packed expert copies serve eager and graph steps alike (the same
            # kernels, so an eager engine computes exactly what the graphs compute)
            from ..models.moe import pack_moe_experts
            pack_moe_experts(self.model)
        if dev.type == "cuda":
            # gamma-folded qkv / gate_up copies for the norm-free small-M layer (eager and
            # graph steps alike, so both run the same arithmetic)
            fold = getattr(self.model, "fold_rs_weights", None)
            if fold is not None:
                fold()
        if self.ps.tp_size > 1 and dev.type == "cuda" and not cfg.disable_custom_all_reduce:
            from ..parallel.custom_allreduce import calibration_rows, maybe_init_custom_allreduce
            rows = calibration_rows(min(cfg.cuda_graph_max_bs, cfg.max_num_seqs))
            comm.set_custom_allreduce(maybe_init_custom_allreduce(
                self.ps, dev, self.mcfg.hidden_size, self.dtype, rows))
        # the cooperative sampler's error word (last PP stage samples)
        self.sampler_health = ops.SamplerHealth(dev) if dev.type == "cuda" else None
        self.ep_a2a = None
        if self.ps.tp_size > 1 and dev.type == "cuda" and cfg.moe_parallel == "ep":
            from ..models.moe import MoEBlock
            from ..parallel.expert_a2a import maybe_init_expert_a2a
            blocks = [m for m in self.model.modules() if isinstance(m, MoEBlock) and m.mode == "ep"]
            if blocks:
                self.ep_a2a = maybe_init_expert_a2a(
                    self.ps, dev, min(cfg.cuda_graph_max_bs, cfg.max_num_seqs), blocks[0].k,
                    self.mcfg.hidden_size, self.dtype)
                for b in blocks:
                    b.ep_a2a = self.ep_a2a
        self.runner = ModelRunner(self.model, self.mcfg, self.dtype, dev, cfg.block_size,
                                  self.max_model_len, cfg.max_num_seqs, cfg.token_budget(),
                                  cfg.enforce_eager, cfg.cuda_graph_max_bs,
                                  kv_dtype=cfg.kv_torch_dtype(self.dtype))
        if self.ps.pp_size > 1 and dev.type == "cuda" and not cfg.enforce_eager:
            # per-stage decode graphs: the stage handoff as kernels over peer memory (one
            # node), or point-to-point sends between the stages' replays (pods on several
            # nodes: parallel/pp_handoff.py HostPipelineLink)
            from ..parallel.pp_handoff import init_pp_link
            self.runner.pp_link = init_pp_link(self.ps, dev, self.runner.graph_max_bs,
                                               self.mcfg.hidden_size, self.dtype, cfg.nnodes)

    def profile(self) -> int:
        if self.cfg.num_gpu_blocks_override:
            return self.cfg.num_gpu_blocks_override
        return self.runner.profile_num_blocks(self.cfg.gpu_memory_utilization)

    def init_cache(self, nb: int) -> None:
        self.runner.init_kv_cache(nb)

    def capture(self) -> float:
        return self.runner.capture_graphs()

    def run(self, plan: StepPlan):
        return self.runner.run(plan)

    def release(self) -> None:
        if self.runner.pp_link is not None:
            self.runner.pp_link.close()
            self.runner.pp_link = None
        if self.ep_a2a is not None:
            self.ep_a2a.close()
            self.ep_a2a = None
        self.runner.release()


# ---------------------------------------------------------------------- plan transport
# TP only: commands and plans are broadcast over the gloo group (every rank takes part
# in every step at the same time anyway).  PP > 1: the driver SENDS them to every rank
# (non-blocking isend, FIFO per pair), so it can hand stage 0 the next micro-batch while
# the later stages are still busy with earlier ones -- a broadcast would make the driver
# wait for the slowest stage to join and serialise the pipeline.
_pending_sends: list = []     # (work, tensor): tensors kept alive until their isend completes


def _p2p_plans(s) -> bool:
    return s.pp_size > 1


def _send_to_ranks(s, tensors: list) -> None:
    base = getattr(s, "global_base", 0)
    for r in range(1, s.tp_size * s.pp_size):
        for t in tensors:
            _pending_sends.append((dist.isend(t, dst=base + r, group=s.cpu_group), t))
    _pending_sends[:] = [(w, t) for w, t in _pending_sends if not w.is_completed()]


def _drain_sends() -> None:
    for w, _ in _pending_sends:
        w.wait()
    _pending_sends.clear()


def _bcast_cmd(cmd: int, arg: int = 0, header: Optional[list[int]] = None) -> list[int]:
    s = get_state()
    h = torch.zeros(16, dtype=torch.int64)
    if s.rank == 0:
        h[0], h[1] = cmd, arg
        if header:
            h[2:2 + len(header)] = torch.tensor(header)
    if _p2p_plans(s):
        if s.rank == 0:
            _send_to_ranks(s, [h])
        else:
            dist.recv(h, src=getattr(s, "global_base", 0), group=s.cpu_group)
    else:
        dist.broadcast(h, src=getattr(s, "global_base", 0), group=s.cpu_group)
    return h.tolist()


def _bcast_plan_blobs(runner: ModelRunner, plan_hdr: list[int]) -> None:
    s = get_state()
    src = getattr(s, "global_base", 0)
    blobs = (runner.hblob,)     # the step's int64 / int32 / fp32 arrays: one byte blob
    if _p2p_plans(s):
        if s.rank == 0:      # the driver rewrites its blobs for the next micro-batch
            _send_to_ranks(s, [t.clone() for t in blobs])
        else:
            for t in blobs:
                dist.recv(t, src=src, group=s.cpu_group)
        return
    for t in blobs:
        dist.broadcast(t, src=src, group=s.cpu_group)


def _send_tokens_to_driver(tokens: torch.Tensor, sampler_health=None) -> None:
    """The last PP stage's TP leader hands the sampled ids to the driver, with ONE extra
    trailing value: this stage's sampler error flag for the step (the driver's own word
    belongs to stage 0, which never samples at PP > 1)."""
    s = get_state()
    slot = sampler_health.enqueue_err_read() if sampler_health is not None else None
    host = tokens.cpu()              # stream-ordered: the flag copy above has landed too
    flag = int(sampler_health.failed(slot)) if slot is not None else 0
    msg = torch.cat([host.to(torch.int64), torch.tensor([flag], dtype=torch.int64)])
    dist.send(msg, dst=getattr(s, "global_base", 0), group=s.cpu_group)


def _tokens_from_last_stage(t: torch.Tensor) -> list[int]:
    """Driver side of ``_send_tokens_to_driver``: the ids, or SamplerFailed."""
    vals = t.tolist()
    if vals[-1]:
        raise ops.SamplerFailed("top-k / top-p sampler on the last pipeline stage: a row's "
                                "barrier timed out; the step's tokens are invalid")
    return vals[:-1]


def _release_custom_allreduce() -> None:
    car = comm.get_custom_allreduce()
    if car is not None:
        comm.set_custom_allreduce(None)
        car.close()


def worker_loop(worker: Worker) -> None:
    """Non-driver ranks: execute commands until CMD_EXIT."""
    s = get_state()
    last_pp_leader = s.is_last_pp and s.tp_rank == 0 and s.rank != 0
    while True:
        h = _bcast_cmd(0)
        cmd, arg = h[0], h[1]
        if cmd == CMD_EXIT:
            if worker.heartbeat is not None:
                worker.heartbeat.stop()
            worker.runner.write_stage_stats()
            _release_custom_allreduce()
            worker.release()
            break
        if cmd == CMD_PROFILE:
            nb = worker.profile()
            comm.all_reduce_min_scalar(nb)
        elif cmd == CMD_INIT_CACHE:
            worker.init_cache(arg)
        elif cmd == CMD_CAPTURE:
            worker.capture()
        elif cmd == CMD_STEP:
            hdr = h[2:2 + N_HDR]
            worker.runner.next_host_bufs()
            _bcast_plan_blobs(worker.runner, hdr)
            r = worker.runner
            plan = StepPlan(*hdr, r.h64.numpy(), r.h32.numpy(), r.hf.numpy())
            out = worker.run(plan)
            if last_pp_leader and out is not None:
                _send_tokens_to_driver(out, worker.sampler_health)


class LocalExecutor:
    def __init__(self, cfg: EngineConfig):
        self.worker = Worker(cfg)

    @property
    def runner(self) -> ModelRunner:
        return self.worker.runner

    def profile(self) -> int:
        return self.worker.profile()

    def init_cache(self, nb: int) -> None:
        self.worker.init_cache(nb)

    def capture(self) -> float:
        return self.worker.capture()

    def execute(self, plan: StepPlan) -> list[int]:
        out = self.worker.run(plan)
        sh = self.worker.sampler_health
        slot = sh.enqueue_err_read() if sh is not None else None
        res = out.tolist()              # synchronises: the error word has landed
        if sh is not None:
            sh.raise_if_failed(slot)
        return res

    def execute_async(self, plan: StepPlan) -> "TokenFuture":
        out = self.worker.run(plan)
        sh = self.worker.sampler_health
        # ahead of the token copy (its event covers both), into this step's own slot
        slot = sh.enqueue_err_read() if sh is not None else None
        done = (lambda: sh.raise_if_failed(slot)) if sh is not None else None
        return TokenFuture(*self.runner.tokens_to_host(out), lp=self.runner.take_logprobs(),
                           on_done=done)

    @property
    def supports_async(self) -> bool:
        return True

    def shutdown(self) -> None:
        _release_custom_allreduce()          # a phantom TP rank's local peer buffers
        self.worker.runner.release()


class TokenFuture:
    """Sampled ids of a launched step; result() blocks until the D2H copy landed.
    ``logprobs()`` -> {sampled row: (logprob of the sampled token, [(id, logprob)] top-k)}
    for the rows whose requests asked for logprobs.  ``on_done`` runs once the step has
    completed on the device (failure checks: engine/health.py)."""

    def __init__(self, buf: torch.Tensor, ev=None, values: Optional[list[int]] = None, lp=None,
                 on_done=None):
        self.buf, self.ev, self.values, self._lp = buf, ev, values, lp
        self._on_done = on_done

    def done(self) -> bool:
        """Non-blocking: has the step (and its token copy) completed?"""
        return self.values is not None or self.ev is None or self.ev.query()

    def result(self) -> list[int]:
        if self.values is None:
            if self.ev is not None:
                self.ev.synchronize()
            self.values = self.buf.tolist()
            if self._on_done is not None:
                done, self._on_done = self._on_done, None
                done()
        return self.values

    def logprobs(self) -> dict:
        if self._lp is None:
            return {}
        rows, chosen, topv, topi = self._lp
        chosen, topv, topi = chosen.tolist(), topv.tolist(), topi.tolist()
        return {r: (chosen[i], list(zip(topi[i][:k], topv[i][:k])))
                for i, (r, k) in enumerate(rows)}


class PipelinedTokenFuture:
    """Sampled ids of a micro-batch in the pipeline (PP > 1): arrive from the last stage."""

    def __init__(self, work, buf: torch.Tensor, on_done):
        self.work, self.buf, self._on_done = work, buf, on_done
        self.values: Optional[list[int]] = None

    def done(self) -> bool:
        """Non-blocking: have the last stage's ids arrived?"""
        return self.values is not None or self.work.is_completed()

    def result(self) -> list[int]:
        if self.values is None:
            self.work.wait()
            done, self._on_done = self._on_done, None
            done()
            self.values = _tokens_from_last_stage(self.buf)
        return self.values

    def logprobs(self) -> dict:
        return {}


class _DistExecutorBase:
    """Rank 0 side of the command protocol (shared by spawned / torchrun ranks)."""
    worker: Worker
    watchdog: Optional[RankWatchdog] = None

    def _step_launched(self, begin: bool = True):
        """Book-keeping after a step's kernels are enqueued: progress for the watchdog, and
        an async copy of the xGMI all-reduce error word checked when the step completes."""
        if begin and self.watchdog is not None:
            self.watchdog.step_begin()
        # sticky error words of the peer-memory collectives (xGMI all-reduce, EP exchange),
        # and this rank's sampler word when it samples (PP > 1: the last stage reports its
        # own with the tokens, _send_tokens_to_driver)
        sh = self.worker.sampler_health if get_state().is_last_pp else None
        checks = [c for c in (comm.get_custom_allreduce(), getattr(self.worker, "ep_a2a", None),
                              self.worker.runner.pp_link, sh)
                  if c is not None]
        slots = [c.enqueue_err_read() for c in checks]
        # the error words land in pinned host memory behind this event: done() reads them
        # only after it, so a failure of this step is reported with this step's tokens
        ev = None
        if checks and self.worker.runner.is_gpu:
            ev = torch.cuda.Event()
            ev.record()

        def done():
            if ev is not None:
                ev.synchronize()
            if self.watchdog is not None:
                self.watchdog.step_end()
            for c, slot in zip(checks, slots):
                c.raise_if_failed(slot)
        return done

    @property
    def runner(self) -> ModelRunner:
        return self.worker.runner

    def profile(self) -> int:
        _bcast_cmd(CMD_PROFILE)
        nb = self.worker.profile()
        return comm.all_reduce_min_scalar(nb)

    def init_cache(self, nb: int) -> None:
        _bcast_cmd(CMD_INIT_CACHE, nb)
        self.worker.init_cache(nb)

    def capture(self) -> float:
        _bcast_cmd(CMD_CAPTURE)
        return self.worker.capture()

    @property
    def supports_async(self) -> bool:
        return get_state().pp_size == 1

    @property
    def pipeline_depth(self) -> int:
        """Micro-batches the engine keeps in flight (one per pipeline stage)."""
        return get_state().pp_size

    def execute_pipelined(self, plan: StepPlan) -> "PipelinedTokenFuture":
        """PP > 1: send the plan to every rank, run stage 0 of it here (its activations
        go to stage 1 by point-to-point), and return at once; the last stage's TP leader
        sends the sampled ids back, received by a posted irecv."""
        if self.watchdog is not None:
            self.watchdog.step_begin()
        _bcast_cmd(CMD_STEP, 0, plan.header())
        _bcast_plan_blobs(self.worker.runner, plan.header())
        self.worker.run(plan)
        # the error-word copies go behind this micro-batch's kernels, not ahead of them
        done = self._step_launched(begin=False)
        s = get_state()
        t = torch.empty(plan.S + 1, dtype=torch.int64)      # ids + the last stage's flag
        src = getattr(s, "global_base", 0) + (s.pp_size - 1) * s.tp_size
        return PipelinedTokenFuture(dist.irecv(t, src=src, group=s.cpu_group), t, done)

    def execute_async(self, plan: StepPlan) -> TokenFuture:
        if self.watchdog is not None:
            self.watchdog.step_begin()
        _bcast_cmd(CMD_STEP, 0, plan.header())
        _bcast_plan_blobs(self.worker.runner, plan.header())
        out = self.worker.run(plan)
        if self.watchdog is not None:
            self.watchdog.step_end()
        return TokenFuture(*self.runner.tokens_to_host(out), lp=self.runner.take_logprobs(),
                           on_done=self._step_launched())

    def execute(self, plan: StepPlan) -> list[int]:
        if self.watchdog is not None:
            self.watchdog.step_begin()
        _bcast_cmd(CMD_STEP, 0, plan.header())
        _bcast_plan_blobs(self.worker.runner, plan.header())
        out = self.worker.run(plan)
        done = self._step_launched()
        s = get_state()
        if s.pp_size > 1:
            t = torch.empty(plan.S + 1, dtype=torch.int64)  # ids + the last stage's flag
            src = getattr(s, "global_base", 0) + (s.pp_size - 1) * s.tp_size
            dist.recv(t, src=src, group=s.cpu_group)
            done()
            res = _tokens_from_last_stage(t)
        else:
            res = out.tolist()
            done()
        if self.watchdog is not None:
            self.watchdog.step_end()
        return res

    def shutdown(self) -> None:
        if self.watchdog is not None:
            self.watchdog.stop()          # the ranks are about to exit on purpose
        self.worker.runner.write_stage_stats()
        try:
            _bcast_cmd(CMD_EXIT)
            _drain_sends()
        except Exception:  # noqa: BLE001
            pass
        _release_custom_allreduce()


class ExternalExecutor(_DistExecutorBase):
    """All ranks launched externally (torchrun); call on rank 0 only.  The driver cannot
    see the other ranks' exit codes, so its watchdog follows their heartbeats (and the
    adaptive step timeout) instead."""

    def __init__(self, worker: Worker):
        self.worker = worker
        self.watchdog = _remote_watchdog([], worker)


def _watch_heartbeats(wd: RankWatchdog, worker: "Worker") -> None:
    """Follow the heartbeats of this engine replica's other ranks (every rank but the
    driver), in the replica's own store (engine/health.py replica_store)."""
    s = get_state()
    store = worker.hb_store
    n = s.tp_size * s.pp_size
    if store is not None and n > 1:
        base = getattr(s, "global_base", 0)
        wd.watch_heartbeats(store, range(base + 1, base + n))


def _remote_watchdog(procs, worker: "Worker") -> RankWatchdog:
    wd = RankWatchdog(procs)
    _watch_heartbeats(wd, worker)
    return wd.start()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn_entry(rank: int, cfg: EngineConfig, env: dict, local: Optional[int] = None) -> None:
    local = rank if local is None else local
    os.environ.update(env)
    os.environ["RANK"] = str(rank)
    os.environ["LOCAL_RANK"] = str(local)
    watch_parent()            # never outlive the driver (engine/health.py)
    try:
        w = Worker(cfg, rank=rank, local_device=local)
        worker_loop(w)
    except Exception:
        traceback.print_exc()
        raise
    finally:
        destroy_parallel()


def spawn_local_ranks(cfg: EngineConfig, env: dict, first: int, last: int, daemon: bool = True):
    """Start ranks [first, last) of this node as worker processes (local device =
    rank - node_rank * ranks_per_node)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    base = cfg.node_rank * cfg.ranks_per_node
    procs = []
    for r in range(first, last):
        p = ctx.Process(target=_spawn_entry, args=(r, cfg, env, r - base), daemon=daemon)
        p.start()
        procs.append(p)
    return procs


class MultiprocExecutor(_DistExecutorBase):
    """Rank 0 (the driver) plus this node's other ranks as spawned processes; with
    ``cfg.nnodes > 1`` the remaining nodes run ``entrypoints.worker_node`` and join
    the same rendezvous."""

    def __init__(self, cfg: EngineConfig):
        if cfg.node_rank != 0:
            raise ValueError("the engine (driver) runs on node 0; use entrypoints.worker_node")
        env = cfg.dist_env()
        if cfg.nnodes == 1 and not cfg.master_addr:
            env["MASTER_PORT"] = str(_free_port())
        for k in ("HSA_ENABLE_IPC_MODE_LEGACY", "KGC_DIST_BACKEND"):
            if k in os.environ:
                env[k] = os.environ[k]
        self.procs = spawn_local_ranks(cfg, env, 1, cfg.ranks_per_node)
        # a dead rank or a step stuck in a collective ends this process (engine/health.py)
        self.watchdog = RankWatchdog(self.procs).start()
        os.environ.update(env)
        os.environ["RANK"] = "0"
        os.environ["LOCAL_RANK"] = "0"
        self.worker = Worker(cfg, rank=0, local_device=0)
        _watch_heartbeats(self.watchdog, self.worker)

    def shutdown(self) -> None:
        super().shutdown()
        for p in self.procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
        self.worker.runner.release()
        destroy_parallel()
