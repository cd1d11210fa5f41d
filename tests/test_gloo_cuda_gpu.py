"""The process-group sums the TP engine falls back to when the xGMI kernel is off
(KGC_CUSTOM_AR=0, e.g. the 8-rank engine test on one GPU): gloo over CUDA tensors, bf16 /
fp16 / fp32 sums and the int64 MAX of vocab-parallel sampling, at world 2 and 8."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    bad = []
    try:
        for dt in (torch.bfloat16, torch.float16, torch.float32):
            for n in (7, 1024, 100 * 1024):
                g = torch.Generator().manual_seed(n + rank)
                x = torch.randint(-8, 9, (n,), generator=g).to(dt)
                exp = sum(torch.randint(-8, 9, (n,), generator=torch.Generator().manual_seed(n + r))
                          .to(torch.float32) for r in range(world)).to(dt)
                y = x.to(dev)
                dist.all_reduce(y)
                if not torch.equal(y.cpu(), exp):
                    bad.append((str(dt), n, float((y.cpu().float() - exp.float()).abs().max())))
        v = torch.tensor([rank * 10, -rank], dtype=torch.int64, device=dev)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        if v.tolist() != [(world - 1) * 10, 0]:
            bad.append(("int64 max", v.tolist()))
    finally:
        q.put((rank, bad))
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_allreduce_cuda_tensors(gpu, world):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(world, _port(), q), nprocs=world, join=True,
                       start_method="spawn")
    res = dict(q.get() for _ in range(world))
    assert all(not b for b in res.values()), res
