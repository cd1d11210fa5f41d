"""Fused all-reduce + residual add + RMSNorm (allreduce.hip) against the unfused pair,
world = 2 / 4 ranks as processes sharing one GPU (gloo group, IPC-mapped peer buffers).

    python tools/allreduce_rms_bench.py --world 2 [--rows 256 --hidden 8192]

Per (world, M, H): the row-segmented two-shot fused kernel, the one-shot fused kernel
(where the message fits its limit), and the plain two-shot all-reduce followed by
fused_add_rms_norm -- each captured 20 times in a hipGraph, replayed after a barrier,
max over ranks.  On one GPU every rank's kernel shares the device's HBM and CUs (the
"link" is HBM), so the numbers rank the kernel forms' structure (launches, barriers,
passes over the data), not xGMI bandwidth.  Rank 0 prints one JSON line per form.
"""
import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, shapes, iters, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubernetes_gpu_cluster_amd import ops
    from kubernetes_gpu_cluster_amd.parallel.custom_allreduce import CustomAllReduce
    dev = torch.device("cuda", 0)
    car = CustomAllReduce(dist.group.WORLD, rank, world, dev, cap_bytes=8 << 20)
    try:
        for M, H in shapes:
            x = torch.randn(M, H, device=dev).to(torch.bfloat16)
            res = torch.randn(M, H, device=dev).to(torch.bfloat16)
            w = torch.ones(H, device=dev, dtype=torch.bfloat16)
            nb = x.numel() * 2
            forms = {}

            def fused(two):
                def f():
                    car.fused_max = 0 if two else nb
                    car.fused2_max = car.cap
                    car.all_reduce_add_rms(x, res, w, 1e-5)
                return f

            def unfused():
                y = car.all_reduce(x)
                ops.fused_add_rms_norm(y, res, w, 1e-5)

            forms["fused_two_shot"] = fused(True)
            if nb <= car.one_shot_max * 4:
                forms["fused_one_shot"] = fused(False)
            forms["two_shot_then_add_rms"] = unfused
            for name, fn in forms.items():
                fn()
                torch.cuda.synchronize()
                dist.barrier()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(iters):
                        fn()
                torch.cuda.synchronize()
                best = float("inf")
                for _ in range(3):
                    dist.barrier()
                    t = time.perf_counter()
                    g.replay()
                    torch.cuda.synchronize()
                    best = min(best, (time.perf_counter() - t) / iters)
                car.check()
                tt = torch.tensor([best])
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                if rank == 0:
                    q.put({"world": world, "M": M, "H": H, "bytes": nb, "form": name,
                           "us": round(tt.item() * 1e6, 2)})
                del g
        car.check()
        dist.barrier()
    finally:
        car.close()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="256x8192,64x8192,16x8192,256x4096")
    a = ap.parse_args()
    shapes = [tuple(int(v) for v in s.split("x")) for s in a.shapes.split(",")]
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(a.world, _port(), shapes, a.iters, q), nprocs=a.world,
                       join=True, start_method="spawn")
    while not q.empty():
        print(json.dumps(q.get()), flush=True)


if __name__ == "__main__":
    main()
