"""One-/two-shot all-reduce over xGMI peer memory for the decode-size TP all-reduces
(call sites C1/C2 in §2.6).

Why: inside one MI355X node every GPU pair has its own xGMI link (7 per GPU).  RCCL's
ring all-reduce moves each byte over one link per step and pays a pipeline of 2(N-1)
latency-bound hops; for the 0.06-4 MB messages of a decode step it is latency bound.
Here every rank maps its TP peers' IPC buffers and one kernel (csrc/kernels/allreduce.hip)
reads them all at once:

* one-shot (<= ``one_shot_max`` bytes): each rank sums all N inputs itself;
* two-shot (<= ``cap_bytes``): reduce-scatter into the owners' buffers, then
  all-gather -- 2(N-1)/N of the bytes per rank, every link busy in parallel.

Larger messages (prefill) fall back to RCCL.  The kernel's epoch counters live in
device memory, so the all-reduce is captured into the decode hipGraphs like any
other kernel.  ``--disable-custom-all-reduce`` (reference
``values-01-minimal-example8.yaml:32``) or ``KGC_CUSTOM_AR=0`` turns it off.
"""
from __future__ import annotations

import collections
import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

from ..engine.health import AllReduceFailed

log = logging.getLogger("kgc.allreduce")

SUPPORTED_WORLD = (2, 4, 8)


def _agree(ok: bool, group) -> bool:
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t[0]))


class CustomAllReduce:
    """Collective constructor: every rank of ``cpu_group`` must call it together.
    Each step that can fail on one rank is followed by an agreement all-reduce, so a
    failure raises on every rank instead of leaving peers blocked in a collective."""

    def __init__(self, cpu_group, rank: int, world: int, device: torch.device,
                 cap_bytes: Optional[int] = None, one_shot_max: Optional[int] = None):
        if world not in SUPPORTED_WORLD:
            raise ValueError(f"xGMI all-reduce supports {SUPPORTED_WORLD} ranks, not {world}")
        self.rank, self.world, self.device = rank, world, device
        self._thresholds(cap_bytes, one_shot_max)
        self._own, self._opened = 0, []
        self._err_host: Optional[torch.Tensor] = None
        handle, err = None, None
        try:
            from .. import ops
            ops.load_extension(strict=True)
            k = torch.ops.kgc
            with torch.cuda.device(device):
                sig_bytes = int(k.ar_signal_bytes())
                # [signal | all-reduce parity 0 | parity 1 | fused one-shot parity 0 | 1 |
                #  fused two-shot parity 0 | 1 | wide two-shot parity 0 | 1]: each kernel
                #  grid has its own regions (their element -> workgroup maps differ, see
                #  allreduce.hip)
                self._own = int(k.ar_alloc(sig_bytes + 8 * self.cap))
                handle = k.ar_get_handle(self._own).tolist()
        except Exception as e:  # noqa: BLE001
            err = e
        if not _agree(err is None, cpu_group):
            self.close()
            raise RuntimeError(f"xGMI all-reduce buffer allocation failed: {err}")
        gathered: list = [None] * world
        dist.all_gather_object(gathered, handle, group=cpu_group)
        bases = []
        try:
            with torch.cuda.device(device):
                for r, h in enumerate(gathered):
                    if r == rank:
                        bases.append(self._own)
                    else:
                        p = int(k.ar_open_handle(torch.tensor(h, dtype=torch.uint8)))
                        self._opened.append(p)
                        bases.append(p)
        except Exception as e:  # noqa: BLE001
            err = e
        if not _agree(err is None, cpu_group):
            self.close()
            raise RuntimeError(f"xGMI all-reduce peer mapping failed: {err}")
        self._set_bases(bases, sig_bytes)

    def _thresholds(self, cap_bytes: Optional[int], one_shot_max: Optional[int]) -> None:
        """Thresholds (logged at start-up; env-tunable because the one-shot / two-shot
        crossover and the RCCL hand-over point depend on the node's xGMI topology and
        have only been measured at 2 / 4 ranks on one GPU): KGC_AR_CAP -- largest message
        this path takes (bytes; above it RCCL), KGC_AR_ONE_SHOT_MAX -- largest one-shot
        message (one-shot reads (N-1) x bytes, two-shot 2(N-1)/N x bytes but pays two
        barriers)."""
        world = self.world
        self.cap = int(cap_bytes if cap_bytes is not None else
                       os.environ.get("KGC_AR_CAP", 8 << 20))
        env_os = os.environ.get("KGC_AR_ONE_SHOT_MAX")
        self.one_shot_max = int(one_shot_max if one_shot_max is not None else
                                env_os if env_os else (512 << 10 if world <= 2 else 256 << 10))
        # fused all-reduce + add + RMSNorm: one-shot up to KGC_AR_RMS_MAX (default: the
        # plain one-shot limit), the row-segmented two-shot form above it up to
        # KGC_AR_RMS2_MAX.  Default: the whole buffer at 2 ranks, off from 4 ranks up --
        # measured with the ranks as processes on one GPU (tools/allreduce_rms_bench.py,
        # profiles/allreduce_rms_fused_r4.jsonl, 256 x 8192 bf16 = 4 MB): world 2 33.4 vs
        # 37.1 us for two-shot + fused_add_rms_norm, world 4 72.1 vs 56.3 us.  (One GPU
        # shares its HBM and CUs between the ranks; on an xGMI node re-measure and set
        # KGC_AR_RMS2_MAX.)
        self.wide_min = int(os.environ.get("KGC_AR_WIDE_MIN", 1 << 62))
        self.fused_max = int(os.environ.get("KGC_AR_RMS_MAX", self.one_shot_max))
        self.fused2_max = int(os.environ.get("KGC_AR_RMS2_MAX", self.cap if world <= 2 else 0))
        self.fused_calls = 0        # host-side launches (a graph capture counts once)
        self.fused2_calls = 0       # ... of them the two-shot form
        # start-up calibration (calibrate): [(bytes, plain form, fused form)] ascending,
        # consulted by every call up to its largest size; None: the thresholds above
        self.table: Optional[list] = None
        self.calibration: Optional[dict] = None
        self.launches: collections.Counter = collections.Counter()   # form -> host launches
        # ... of them decided by a calibrated table entry (the rest: sizes past the table)
        self.table_launches: collections.Counter = collections.Counter()

    def _set_bases(self, bases: list, sig_bytes: int) -> None:
        self.sig = bases
        self.data = [b + sig_bytes for b in bases]
        self.fdata = [b + sig_bytes + 2 * self.cap for b in bases]
        self.fdata2 = [b + sig_bytes + 4 * self.cap for b in bases]
        self.wdata = [b + sig_bytes + 6 * self.cap for b in bases]
        self.max_hidden = int(torch.ops.kgc.allreduce_rms_max_hidden())

    # ------------------------------------------------------------------ policy
    def _entry(self, nb: int) -> Optional[tuple]:
        """The calibrated (bytes, plain, fused) entry covering a message of nb bytes: the
        smallest calibrated size >= nb (None past the table or without one)."""
        if not self.table:
            return None
        for e in self.table:
            if nb <= e[0]:
                return e
        return None

    def plain_form(self, nb: int) -> str:
        """'one' | 'two' | 'two_wide' | 'rccl' for a plain all-reduce of nb bytes
        ('two_wide': the two-shot form on its 256-workgroup grid; the thresholds, without a
        calibration table, pick it from KGC_AR_WIDE_MIN bytes up -- default never)."""
        e = self._entry(nb)
        if e is not None:
            return e[1]
        if nb > self.cap:
            return "rccl"
        if self.table and self.table[-1][1] != "one":
            # past the calibrated sizes (prefill-sized messages): the largest calibrated
            # size's bandwidth form, not the one-shot threshold default (a larger message
            # never favours one-shot over the form that beat it at the largest size)
            return self.table[-1][1]
        if nb > self.one_shot_max:
            return "two_wide" if nb >= self.wide_min else "two"
        return "one"

    def fused_form(self, nb: int) -> str:
        """'fused1' | 'fused2' | 'split' (the plain form, then fused_add_rms_norm)."""
        e = self._entry(nb)
        if e is not None:
            return e[2]
        if self.table and self.table[-1][2] != "fused1":
            last = self.table[-1][2]
            return last if last == "split" or nb <= self.cap else "split"
        if nb <= min(self.fused_max, self.cap):
            return "fused1"
        if nb <= min(self.fused2_max, self.cap):
            return "fused2"
        return "split"

    def should_use(self, x: torch.Tensor) -> bool:
        if not x.is_cuda or x.dtype not in (torch.bfloat16, torch.float16):
            return False
        nb = x.numel() * x.element_size()
        return (x.is_contiguous() and 0 < nb <= self.cap and nb % (16 * self.world) == 0
                and self.plain_form(nb) != "rccl")

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        nb = x.numel() * x.element_size()
        form = self.plain_form(nb)
        self._launch_plain(x, form)
        self.launches[form] += 1
        if self._entry(nb) is not None:
            self.table_launches[form] += 1
        return x

    def _launch_plain(self, x: torch.Tensor, form: str) -> None:
        wide = form == "two_wide"
        torch.ops.kgc.xgmi_allreduce(x, self.wdata if wide else self.data, self.sig, self.rank,
                                     self.cap, form != "one", wide)

    def can_fuse(self, x: torch.Tensor) -> bool:
        if not x.is_cuda or x.dtype not in (torch.bfloat16, torch.float16) or x.dim() != 2:
            return False
        H = x.shape[1]
        nb = x.numel() * x.element_size()
        return (x.is_contiguous() and 0 < nb <= self.cap and H % 8 == 0
                and H <= self.max_hidden and self.fused_form(nb) != "split")

    def all_reduce_add_rms(self, x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                           eps: float, out: torch.Tensor = None):
        """One launch: h = sum over ranks of x; residual += h; out = rms_norm(residual) * w
        (same rounding as all_reduce + fused_add_rms_norm).  Returns (out, residual)."""
        if out is None:
            out = torch.empty_like(x)
        self.fused_calls += 1
        nb = x.numel() * x.element_size()
        two = self.fused_form(nb) == "fused2"
        if two:
            self.fused2_calls += 1
        self.launches["fused2" if two else "fused1"] += 1
        if self._entry(nb) is not None:
            self.table_launches["fused2" if two else "fused1"] += 1
        torch.ops.kgc.xgmi_allreduce_rms(out, x, residual, w, eps,
                                         self.fdata2 if two else self.fdata, self.sig,
                                         self.rank, self.cap, two)
        return out, residual

    # ------------------------------------------------------------------ calibration
    def calibrate(self, hidden: int, dtype: torch.dtype, rows: list[int], tp_group, cpu_group,
                  reps: int = 20, graphs: bool = True) -> dict:
        """Time every form on THIS node at each decode message size (rows x hidden) and
        make the fastest the policy (the crossovers were fixed from a
        one-GPU rehearsal).  Collective over the TP group: every rank runs the same
        launches in the same order (the kernels wait for their peers), the per-rank times
        are MAX-reduced, so every rank derives the same table.  Forms:
          plain  'one' / 'two' (xGMI one- / two-shot, 64 workgroups) / 'two_wide' (two-shot
                 on 256 workgroups: the grid sized for large messages) / 'rccl';
          fused  'fused1' / 'fused2' (one launch with the residual add + RMSNorm) /
                 'split' (the plain choice, then fused_add_rms_norm).
        ``graphs``: each form's ``reps``-call loop is captured in a hipGraph and the table is
        chosen on REPLAY times, as the decode graphs run these kernels (at
        8-64 KB the eager launch rate is comparable to the kernel time, and eager timing
        misranked K9m candidates against the graphs); the eager times are kept beside them
        (``eager_us``, ``graph_minus_eager_us``).  'rccl' is a candidate only where it can
        be captured: not over gloo (ADVICE r5 -- a host-staged gloo all-reduce inside a
        decode graph cannot be captured).  ``cpu_group`` None: a phantom rank (no peers
        to synchronise with or reduce over).
        The thresholds stay the fallback past the largest calibrated size."""
        from .. import ops
        dev = self.device
        res = {"hidden": hidden, "rows": [], "bytes": [], "us": {}, "eager_us": {},
               "timing": "graph" if graphs else "eager"}
        forms = ("one", "two", "two_wide", "rccl", "fused1", "fused2", "split")
        plain_forms = forms[:4]
        gloo = tp_group is None or dist.get_backend(tp_group) == dist.Backend.GLOO
        rccl_ok = tp_group is not None and not (graphs and gloo)

        def barrier():
            if cpu_group is not None:
                dist.barrier(group=cpu_group)

        def timed(fn):
            """(eager us, graph us) per call of fn over ``reps`` calls."""
            torch.cuda.synchronize(dev)
            barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            e1.synchronize()
            eager = e0.elapsed_time(e1) * 1e3 / reps
            if not graphs:
                return eager, eager
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize(dev)
            barrier()
            with torch.cuda.graph(g):
                for _ in range(reps):
                    fn()
            torch.cuda.synchronize(dev)
            barrier()
            g.replay()                                   # warm replay
            torch.cuda.synchronize(dev)
            ts = []
            for _ in range(3):
                barrier()
                e0.record()
                g.replay()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / reps)
            del g
            return eager, sorted(ts)[1]

        times, etimes = [], []
        w = torch.ones(hidden, dtype=dtype, device=dev)
        saved = self.table
        self.table = None
        for m in rows:
            nb = m * hidden * torch.finfo(dtype).bits // 8
            x0 = (torch.randn(m, hidden, device=dev) * 0.01).to(dtype)
            x, out = x0.clone(), torch.empty_like(x0)
            resid = torch.zeros_like(x0)
            ok_x = nb <= self.cap and nb % (16 * self.world) == 0
            ok_f = nb <= self.cap and hidden % 8 == 0 and hidden <= self.max_hidden

            def run(form, x=x, out=out, resid=resid, nb=nb):
                if form in ("one", "two", "two_wide"):
                    self._launch_plain(x, form)
                elif form == "rccl":
                    if gloo:
                        xf = x.float()              # gloo: the fp32 path comm.py takes
                        dist.all_reduce(xf, group=tp_group)
                        x.copy_(xf)
                    else:
                        dist.all_reduce(x, group=tp_group)
                elif form in ("fused1", "fused2"):
                    torch.ops.kgc.xgmi_allreduce_rms(out, x, resid, w, 1e-6,
                                                     self.fdata2 if form == "fused2" else
                                                     self.fdata, self.sig, self.rank,
                                                     self.cap, form == "fused2")
            row, erow = [], []
            for form in forms:
                if (form in ("one", "two", "two_wide") and not ok_x) or (
                        form in ("fused1", "fused2") and not ok_f) or form == "split" or (
                        form == "rccl" and not rccl_ok):
                    row.append(float("inf"))
                    erow.append(float("inf"))
                    continue
                torch.cuda.synchronize(dev)
                barrier()
                for _ in range(3):
                    x.copy_(x0)
                    run(form)
                x.copy_(x0)
                try:
                    e, g = timed(lambda form=form: run(form))
                except RuntimeError as ex:          # e.g. a backend that cannot be captured
                    log.warning("all-reduce calibration: %s not timed (%s)", form, ex)
                    e = g = float("inf")
                row.append(g)
                erow.append(e)
            # 'split' = the fastest plain form + one fused_add_rms_norm launch
            e, g = timed(lambda: ops.fused_add_rms_norm(x, resid, w, 1e-6))
            row[forms.index("split")] = min(row[:len(plain_forms)]) + g
            erow[forms.index("split")] = min(erow[:len(plain_forms)]) + e
            times.append(row)
            etimes.append(erow)
            res["rows"].append(m)
            res["bytes"].append(nb)
        t = torch.tensor([times, etimes], dtype=torch.float64)
        t[torch.isinf(t)] = 1e30
        if cpu_group is not None:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=cpu_group)
        table = []
        for i, nb in enumerate(res["bytes"]):
            tr, te = t[0, i].tolist(), t[1, i].tolist()
            plain = min(plain_forms, key=lambda f: tr[forms.index(f)])
            fused = min(("fused1", "fused2", "split"), key=lambda f: tr[forms.index(f)])
            table.append((nb, plain, fused))
            for f in forms:
                v, ve = tr[forms.index(f)], te[forms.index(f)]
                res["us"].setdefault(f, []).append(None if v >= 1e29 else round(v, 2))
                res["eager_us"].setdefault(f, []).append(None if ve >= 1e29 else round(ve, 2))
                res.setdefault("graph_minus_eager_us", {}).setdefault(f, []).append(
                    None if v >= 1e29 or ve >= 1e29 else round(v - ve, 2))
            # would eager timing have chosen differently at this size?
            pe = min(plain_forms, key=lambda f: te[forms.index(f)])
            fe = min(("fused1", "fused2", "split"), key=lambda f: te[forms.index(f)])
            res.setdefault("eager_choice_differs", []).append(pe != plain or fe != fused)
        res["table"] = [list(e) for e in table]
        self.table, self.calibration = table, res
        del saved
        torch.cuda.synchronize(dev)
        barrier()
        return res

    def check(self) -> None:
        """Raise if any barrier timed out waiting for a peer (see allreduce.hip)."""
        err = int(torch.ops.kgc.ar_read_err(self.sig[self.rank]))
        if err:
            raise AllReduceFailed(f"xGMI all-reduce: peers {bin(err)} never arrived")

    def enqueue_err_read(self) -> None:
        """Queue an async copy of the sticky error word behind the current step (no sync)."""
        if self._err_host is None:
            self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        torch.ops.kgc.ar_err_copy_async(self.sig[self.rank], self._err_host)

    def raise_if_failed(self, slot=None) -> None:
        """After the step that queued ``enqueue_err_read`` completed: raise on a timed-out
        barrier -- the step summed stale peer data, so its tokens must not be served."""
        if self._err_host is not None and int(self._err_host[0]):
            raise AllReduceFailed(
                f"xGMI all-reduce: peers {bin(int(self._err_host[0]))} never arrived "
                f"(a TP rank is dead or wedged); the engine stops")

    def close(self) -> None:
        if self._own or self._opened:
            torch.cuda.synchronize(self.device)
            for p in self._opened:
                torch.ops.kgc.ar_close_handle(p)
            if self._own:
                torch.ops.kgc.ar_free(self._own)
            self._own = 0
            self._opened = []


class PhantomAllReduce(CustomAllReduce):
    """The xGMI all-reduce of rank ``rank`` of a TP = ``world`` group whose peers do not
    exist (KGC_TP_PHANTOM, parallel/state.py init_phantom): this rank's buffer and ``world
    - 1`` peer buffers are all local allocations, and the peers' arrival flags in this
    rank's signal are raised far ahead of any epoch (kgc.ar_raise_peer_flags), so every
    kernel form -- one-shot, two-shot, fused one- / two-shot add + RMSNorm -- runs its
    full copy-in / barrier / peer-read / reduce sequence, captured in the decode graphs,
    without waiting.  The peers' data regions hold zeros: the sums are this rank's
    partials only.  Peer reads come from local HBM, not over xGMI links, so the kernels'
    TIMES are not a TP node's; what the phantom measures is every other kernel of the
    rank's step at its real per-rank shapes, and the graph / epoch machinery."""

    # far ahead of any epoch, within the barrier's wrap-safe int32 window (2^30 calls per
    # block: ~18 h of 70B TP = 8 decode at 100 steps / s)
    FLAG_VALUE = 1 << 30

    def __init__(self, rank: int, world: int, device: torch.device,
                 cap_bytes: Optional[int] = None, one_shot_max: Optional[int] = None):
        if world not in SUPPORTED_WORLD:
            raise ValueError(f"xGMI all-reduce supports {SUPPORTED_WORLD} ranks, not {world}")
        from .. import ops
        ops.load_extension(strict=True)
        k = torch.ops.kgc
        self.rank, self.world, self.device = rank, world, device
        self._thresholds(cap_bytes, one_shot_max)
        self._err_host = None
        with torch.cuda.device(device):
            sig_bytes = int(k.ar_signal_bytes())
            bases = [int(k.ar_alloc(sig_bytes + 8 * self.cap)) for _ in range(world)]
            k.ar_raise_peer_flags(bases[rank], rank, world, self.FLAG_VALUE)
            torch.cuda.synchronize(device)
        self._own, self._opened = bases[rank], []
        self._peers = [b for r, b in enumerate(bases) if r != rank]
        self._set_bases(bases, sig_bytes)

    def close(self) -> None:
        if self._own:
            torch.cuda.synchronize(self.device)
            for p in self._peers + [self._own]:
                torch.ops.kgc.ar_free(p)
            self._own, self._peers = 0, []


def _calibration_wanted() -> bool:
    """Start-up calibration of the all-reduce policy, unless KGC_AR_CALIBRATE=0 or an
    operator fixed a threshold (KGC_AR_ONE_SHOT_MAX / KGC_AR_RMS_MAX / KGC_AR_RMS2_MAX /
    KGC_AR_CAP): the environment overrides, the measurement is the default."""
    if os.environ.get("KGC_AR_CALIBRATE", "1") == "0":
        return False
    return not any(os.environ.get(k) for k in ("KGC_AR_ONE_SHOT_MAX", "KGC_AR_RMS_MAX",
                                                "KGC_AR_RMS2_MAX", "KGC_AR_CAP"))


def calibration_rows(max_rows: int) -> list[int]:
    """Decode message sizes the calibration times: powers of two up to the largest graph
    bucket (the table is a step function between them)."""
    rows, r = [], 1
    while r < max_rows:
        rows.append(r)
        r *= 2
    rows.append(max_rows)
    return rows


def maybe_init_custom_allreduce(ps, device: torch.device, hidden: int = 0,
                                dtype: torch.dtype = torch.bfloat16,
                                calibrate_rows: Optional[list] = None
                                ) -> Optional[CustomAllReduce]:
    """Build the xGMI all-reduce for this rank's TP group, or None (RCCL only).
    All TP ranks agree: if any rank cannot set it up, none uses it.  With
    ``calibrate_rows`` the per-size policy is timed on this node (CustomAllReduce.calibrate)."""
    if os.environ.get("KGC_CUSTOM_AR", "1") == "0" or ps.tp_size not in SUPPORTED_WORLD:
        return None
    if getattr(ps, "phantom", False):
        car = PhantomAllReduce(ps.tp_rank, ps.tp_size, device)
        log.info("phantom TP rank %d of %d: xGMI all-reduce against local peer buffers",
                 ps.tp_rank, ps.tp_size)
        if calibrate_rows and hidden and _calibration_wanted():
            # the same graph-timed calibration, over local peer buffers (no group to sync or
            # reduce over): the phantom's policy comes from its own replay times
            car.calibrate(hidden, dtype, calibrate_rows, None, None)
        return car
    try:
        car = CustomAllReduce(ps.tp_cpu_group, ps.tp_rank, ps.tp_size, device)
    except RuntimeError as e:
        log.warning("%s; using RCCL", e)
        return None
    if calibrate_rows and hidden and _calibration_wanted():
        cal = car.calibrate(hidden, dtype, calibrate_rows, ps.tp_group, ps.tp_cpu_group)
        log.info("xGMI all-reduce policy calibrated on this node (hidden %d): %s", hidden,
                 " ".join(f"{r}r:{p}/{f}" for r, (_, p, f) in zip(cal["rows"], cal["table"])))
    log.info("xGMI all-reduce enabled: tp=%d cap=%d KiB (KGC_AR_CAP) one-shot<=%d KiB "
             "(KGC_AR_ONE_SHOT_MAX) fused add+RMSNorm one-shot<=%d KiB (KGC_AR_RMS_MAX), "
             "two-shot<=%d KiB (KGC_AR_RMS2_MAX), %d workgroups",
             ps.tp_size, car.cap >> 10, car.one_shot_max >> 10, car.fused_max >> 10,
             car.fused2_max >> 10, int(torch.ops.kgc.allreduce_max_blocks()))
    return car
