"""Collective probe over the node's GPUs: RCCL all-reduce bus bandwidth and the xGMI
all-reduce kernel (parallel/custom_allreduce.py) against RCCL at the decode message
sizes, measured on the machine the job runs on.

``bench.py --gpus N`` (N > 1) runs it once per rank after the timed waves, in a child
process per GPU with a hard time limit, and reports rank 0's table in its JSON line
("comm_probe"), so the driver's 1/2/4/8-GPU scaling runs also record what RCCL and the
xGMI kernel do at that world size.  The one-shot / two-shot / RCCL hand-over points
(KGC_AR_ONE_SHOT_MAX, KGC_AR_CAP) can then be set from ``crossover``.

    python -m kubernetes_gpu_cluster_amd.benchmarks.comm_probe --rank R --world N \\
        --port P --device D [--out result.json]

Each rank pins cuda:D.  Sizes are bf16 messages; RCCL times are per call from device
events around ``iters`` back-to-back calls (bus bandwidth = algbw * 2(N-1)/N, the ring
all-reduce convention); the xGMI kernel is timed the same way, one-shot and two-shot.
"""
from __future__ import annotations

import argparse
import datetime
import json
import sys

import torch
import torch.distributed as dist

RCCL_SIZES = (256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20)
XGMI_SIZES = (64 << 10, 256 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20)


def _time(fn, iters: int) -> float:
    """Mean seconds per call of ``iters`` back-to-back calls after 3 warm-up calls."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / 1e3 / iters


def probe(rank: int, world: int, dev: torch.device, iters: int = 20) -> dict:
    """Collective timings on an initialised world (nccl default group + a gloo group for
    the xGMI kernel's IPC-handle exchange).  Every rank must call it."""
    out = {"world": world, "backend": dist.get_backend(), "rccl": [], "xgmi": [],
           "crossover": {}}
    # gloo (tests, ranks sharing one GPU) stages through the host: small sizes only
    for nb in RCCL_SIZES if out["backend"] == "nccl" else RCCL_SIZES[:4]:
        x = torch.ones(nb // 2, dtype=torch.bfloat16, device=dev)
        t = _time(lambda: dist.all_reduce(x), iters if nb <= (16 << 20) else 5)
        alg = nb / t / 1e9
        out["rccl"].append({"bytes": nb, "us": round(t * 1e6, 2), "algbw_GBps": round(alg, 1),
                            "busbw_GBps": round(alg * 2 * (world - 1) / world, 1)})
    ok = torch.ones(1, dtype=torch.bfloat16, device=dev)
    dist.all_reduce(ok)
    out["rccl_correct"] = bool(float(ok.item()) == float(world))
    if world in (2, 4, 8):
        from ..parallel.custom_allreduce import CustomAllReduce
        gloo = dist.new_group(backend="gloo")
        car = CustomAllReduce(gloo, rank, world, dev, cap_bytes=max(XGMI_SIZES))
        try:
            for nb in XGMI_SIZES:
                x = torch.ones(nb // 2, dtype=torch.bfloat16, device=dev)
                row = {"bytes": nb}
                for mode, os_max in (("one_shot", nb), ("two_shot", 0)):
                    car.one_shot_max = os_max
                    row[mode + "_us"] = round(_time(lambda: car.all_reduce(x), iters) * 1e6, 2)
                y = torch.ones(nb // 2, dtype=torch.bfloat16, device=dev)
                row["rccl_us"] = round(_time(lambda: dist.all_reduce(y), iters) * 1e6, 2)
                x.fill_(1.0)
                car.one_shot_max = nb
                car.all_reduce(x)
                torch.cuda.synchronize()
                row["correct"] = bool((x.float() == world).all().item())
                out["xgmi"].append(row)
            car.check()
        finally:
            car.close()
        best = [min(("one_shot", r["one_shot_us"]), ("two_shot", r["two_shot_us"]),
                    ("rccl", r["rccl_us"]), key=lambda kv: kv[1])[0] for r in out["xgmi"]]
        one = [r["bytes"] for r, b in zip(out["xgmi"], best) if b == "one_shot"]
        kern = [r["bytes"] for r, b in zip(out["xgmi"], best) if b != "rccl"]
        out["crossover"] = {"best_per_size": best,
                            "largest_one_shot_win_bytes": max(one) if one else 0,
                            "largest_xgmi_win_bytes": max(kern) if kern else 0}
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--backend", default="nccl",
                    help="nccl (= RCCL; one GPU per rank) or gloo (tests: ranks sharing a GPU)")
    a = ap.parse_args()
    dev = torch.device("cuda", a.device)
    torch.cuda.set_device(dev)
    kw = {"device_id": dev} if a.backend == "nccl" else {}
    dist.init_process_group(a.backend, init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank,
                            world_size=a.world, timeout=datetime.timedelta(seconds=60), **kw)
    try:
        res = probe(a.rank, a.world, dev, a.iters)
    finally:
        dist.destroy_process_group()
    if a.rank == 0:
        line = json.dumps(res)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
        print(line, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
