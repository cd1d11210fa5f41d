"""xGMI all-reduce kernel (csrc/kernels/allreduce.hip) == sum of the ranks' inputs.

The GPU box for tests has ONE MI355X, so the ranks are processes sharing cuda:0: the
IPC buffers, epoch-flag barriers and parity double-buffering are exercised exactly as
across GPUs (peer pointers come from hipIpcOpenMemHandle), only the link is HBM
instead of xGMI.  Process group is gloo (RCCL refuses two ranks on one device).
"""
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


def _inputs(rank, n, seed, dtype, integer):
    g = torch.Generator().manual_seed(seed * 1000 + rank)
    if integer:   # exact in bf16 and in any summation order
        return torch.randint(-8, 9, (n,), generator=g).to(dtype)
    return torch.randn(n, generator=g).to(dtype)


def _expected(world, n, seed, dtype, integer):
    acc = torch.zeros(n, dtype=torch.float32)
    for r in range(world):
        acc += _inputs(r, n, seed, dtype, integer).float()
    return acc.to(dtype)


def _worker(rank, world, port, cap):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubernetes_gpu_cluster_amd.parallel.custom_allreduce import CustomAllReduce
    dev = torch.device("cuda", 0)
    car = CustomAllReduce(dist.group.WORLD, rank, world, dev, cap_bytes=cap)
    try:
        # one-shot (small) and two-shot (large), bf16 and fp16, exact integer data
        sizes = [8 * world, 4096, 64 * 4096, cap // 2 // 2, cap // 2]
        seed = 0
        for dtype in (torch.bfloat16, torch.float16):
            for n in sizes:
                for integer in (True, False):
                    seed += 1
                    x = _inputs(rank, n, seed, dtype, integer).to(dev)
                    assert car.should_use(x), (n, dtype)
                    car.all_reduce(x)
                    ref = _expected(world, n, seed, dtype, integer)
                    got = x.cpu()
                    if integer:
                        assert torch.equal(got, ref), (n, dtype, (got - ref).abs().max())
                    else:
                        torch.testing.assert_close(got.float(), ref.float(), atol=0.06, rtol=0.02)
        # hipGraph capture: replays read fresh inputs, epochs advance on the device
        for n in (4096, 256 * 1024):
            static = torch.zeros(n, dtype=torch.bfloat16, device=dev)
            car.all_reduce(static)                       # warm up outside capture
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                car.all_reduce(static)
            for it in range(4):
                seed += 1
                static.copy_(_inputs(rank, n, seed, torch.bfloat16, True))
                g.replay()
                assert torch.equal(static.cpu(), _expected(world, n, seed, torch.bfloat16, True))
        torch.cuda.synchronize()
        car.check()
        dist.barrier()
    finally:
        car.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_allreduce_matches_sum(world, gpu):
    mp.start_processes(_worker, args=(world, _port(), 4 << 20), nprocs=world, join=True,
                       start_method="spawn")


def _timeout_worker(rank, world, port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubernetes_gpu_cluster_amd.engine.health import AllReduceFailed
    from kubernetes_gpu_cluster_amd.parallel.custom_allreduce import CustomAllReduce
    dev = torch.device("cuda", 0)
    car = CustomAllReduce(dist.group.WORLD, rank, world, dev, cap_bytes=1 << 20)
    try:
        x = torch.ones(4096, dtype=torch.bfloat16, device=dev)
        car.all_reduce(x)                       # both ranks: a healthy call
        car.enqueue_err_read()
        torch.cuda.synchronize()
        car.raise_if_failed()
        dist.barrier()
        if rank == 0:
            # rank 1 "dies": rank 0's barrier gives up after its bounded spin and the
            # engine-side check raises instead of serving the stale sum
            car.all_reduce(x)
            car.enqueue_err_read()
            torch.cuda.synchronize()
            with pytest.raises(AllReduceFailed, match="never arrived"):
                car.raise_if_failed()
        dist.barrier()
    finally:
        car.close()
        dist.destroy_process_group()


def test_xgmi_allreduce_peer_timeout_raises(gpu):
    """A missing TP peer: the barrier's bounded spin sets the sticky error word, the async
    copy behind the step brings it to the host, and raise_if_failed (called when the
    step's tokens are read, engine/worker.py) raises AllReduceFailed."""
    mp.start_processes(_timeout_worker, args=(2, _port()), nprocs=2, join=True,
                       start_method="spawn")
