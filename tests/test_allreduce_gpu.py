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
                        if not torch.equal(got, ref):
                            car.check()    # a timed-out barrier raises AllReduceFailed
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
    except AssertionError:
        torch.cuda.synchronize()
        car.check()            # a mismatch after a timed-out barrier is reported as such
        raise
    finally:
        car.close()
        dist.destroy_process_group()


def _run_world(worker, world, *args):
    mp.start_processes(worker, args=(world, _port()) + tuple(args), nprocs=world, join=True,
                       start_method="spawn")


# World 2 / 4 as real processes sharing cuda:0 (IPC-mapped peer buffers).  World 8 runs
# as ONE launch holding all eight ranks' workgroups (test_xgmi_world_emulation below):
# eight processes' spin kernels need not be co-resident on one device, so a multi-process
# 8-rank run on one GPU can only time out, never prove the NR = 8 kernels.
@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_allreduce_matches_sum(world, gpu):
    _run_world(_worker, world, 4 << 20)


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
            # rank 1 "dies": rank 0's barrier gives up after its wall-clock bound
            # (common.h KGC_PEER_SPIN_MS, steady counter) and the engine-side check raises
            # instead of serving the stale sum
            import time
            k = torch.ops.kgc
            assert int(k.wall_clock_rate_khz()) == 100000      # the rate the bound assumes
            bound = int(k.peer_spin_ms()) / 1e3
            t0 = time.monotonic()
            car.all_reduce(x)
            car.enqueue_err_read()
            torch.cuda.synchronize()
            took = time.monotonic() - t0
            print(f"xGMI all-reduce peer time-out: {took:.3f} s (bound {bound:.1f} s)", flush=True)
            assert 0.9 * bound <= took <= bound + 3.0, (took, bound)
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


def _rms_worker(rank, world, port, two_shot=False):
    """Fused all-reduce + residual add + RMSNorm == xgmi all-reduce then fused_add_rms_norm,
    interleaved with plain all-reduces (separate IPC regions), eager and graph-captured.
    two_shot: every fused call takes the row-segmented two-shot kernel."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubernetes_gpu_cluster_amd import ops
    from kubernetes_gpu_cluster_amd.parallel.custom_allreduce import CustomAllReduce
    dev = torch.device("cuda", 0)
    car = CustomAllReduce(dist.group.WORLD, rank, world, dev, cap_bytes=4 << 20,
                          one_shot_max=4 << 20)
    if two_shot:
        car.fused_max = 0           # every fused call: the row-segmented two-shot kernel
        car.fused2_max = car.cap
    try:
        for dtype in (torch.bfloat16, torch.float16):
            for M, H in ((1, 4096), (7, 8192), (130, 4096), (64, 16384), (3, 1024)):
                g = torch.Generator().manual_seed(M * 31 + H + rank)
                x = (torch.randn(M, H, generator=g) * 0.5).to(dtype).to(dev)
                gres = torch.Generator().manual_seed(M * 7 + H)         # same on every rank
                res = torch.randn(M, H, generator=gres).to(dtype).to(dev)
                w = (torch.rand(H, generator=gres) + 0.5).to(dtype).to(dev)
                assert car.can_fuse(x), (M, H)
                r_got = res.clone()
                o_got, _ = car.all_reduce_add_rms(x, r_got, w, 1e-5)
                if H <= 8192:    # unfused reference on the same GPU (rms_norm: H <= 8192)
                    y = x.clone()
                    car.all_reduce(y)
                    r_ref = res.clone()
                    o_ref, _ = ops.fused_add_rms_norm(y, r_ref, w, 1e-5)
                    if not torch.equal(r_got, r_ref):
                        torch.cuda.synchronize()
                        bad = (r_got != r_ref)
                        car.check()        # a timed-out barrier raises AllReduceFailed here
                        raise AssertionError((M, H, dtype, int(bad.sum()), bad.nonzero()[:4].tolist(),
                                              (r_got.float() - r_ref.float()).abs().max().item()))
                    torch.testing.assert_close(o_got.float(), o_ref.float(), atol=1e-2, rtol=1e-2)
                # an fp32 oracle of the whole op
                xs = [(torch.randn(M, H, generator=torch.Generator().manual_seed(M * 31 + H + r))
                       * 0.5).to(dtype).float() for r in range(world)]
                h = sum(xs).to(dtype).float()
                rr = (h + res.cpu().float()).to(dtype).float()
                oo = rr * torch.rsqrt(rr.pow(2).mean(-1, keepdim=True) + 1e-5) * w.cpu().float()
                torch.testing.assert_close(o_got.cpu().float(), oo, atol=3e-2, rtol=3e-2)
        # graph capture: fused + plain all-reduce in one graph, replays with fresh inputs
        M, H = 16, 4096
        xin = torch.zeros(M, H, dtype=torch.bfloat16, device=dev)
        res = torch.zeros(M, H, dtype=torch.bfloat16, device=dev)
        w = torch.ones(H, dtype=torch.bfloat16, device=dev)
        plain = torch.zeros(8192, dtype=torch.bfloat16, device=dev)
        car.all_reduce_add_rms(xin, res, w, 1e-5)
        car.all_reduce(plain)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            out, _ = car.all_reduce_add_rms(xin, res, w, 1e-5)
            car.all_reduce(plain)
        for it in range(3):
            xin.copy_(torch.full((M, H), float(rank + it + 1), dtype=torch.bfloat16))
            res.zero_()
            plain.fill_(float(rank + 1))
            gr.replay()
            torch.cuda.synchronize()
            tot = sum(r + it + 1 for r in range(world))
            assert torch.equal(res.cpu(), torch.full((M, H), float(tot), dtype=torch.bfloat16)), it
            torch.testing.assert_close(out.float().cpu(), torch.ones(M, H), atol=1e-2, rtol=0)
            assert torch.equal(plain.cpu(), torch.full((8192,), float(sum(range(1, world + 1))),
                                                       dtype=torch.bfloat16))
        assert (car.fused2_calls > 0) == two_shot
        car.check()
        dist.barrier()
    except AssertionError:
        torch.cuda.synchronize()
        car.check()            # a mismatch after a timed-out barrier is reported as such
        raise
    finally:
        car.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("two_shot", [False, True])
def test_xgmi_allreduce_add_rmsnorm_fused(world, two_shot, gpu):
    _run_world(_rms_worker, world, two_shot)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_xgmi_world_emulation(world, gpu):
    """Every xGMI all-reduce form at NR = 2 / 4 / 8 in world emulation: ONE launch holds
    all ranks' workgroups on this device (block-major: the workgroups that wait for each
    other are adjacent in dispatch order, so the grid always drains), each rank with its
    own uncached signal + data buffers and inputs, as on a node with one GPU per rank.
    Exact integer sums; the four kernel forms interleaved over several calls so the epoch
    parity of every region flips; the fused forms against an fp32 oracle of
    all-reduce -> residual add -> RMSNorm.  No error word may be set."""
    k = torch.ops.kgc
    from kubernetes_gpu_cluster_amd import ops
    ops.load_extension(strict=True)
    dev = gpu
    cap = 4 << 20
    sig_b = int(k.ar_signal_bytes())
    bases = [int(k.ar_alloc(sig_b + 8 * cap)) for _ in range(world)]
    try:
        sig = bases
        regions = {0: [b + sig_b for b in bases], 1: [b + sig_b for b in bases],
                   2: [b + sig_b + 2 * cap for b in bases], 3: [b + sig_b + 4 * cap for b in bases],
                   4: [b + sig_b + 6 * cap for b in bases]}
        seed = 0
        for it in range(3):
            for dtype in (torch.bfloat16, torch.float16):
                # plain one-shot / two-shot: exact integers (any order sums exactly)
                # (kind 4: the wide two-shot grid, its own epochs / flags / regions)
                for kind, n in ((0, 64 * 1024), (1, 1024 * 1024), (0, 8 * world), (1, 16 * world),
                                (4, 1024 * 1024), (4, 16 * world), (4, 8 * 4096 * 8 + 8 * world)):
                    seed += 1
                    xs = [_inputs(r, n, seed, dtype, True).to(dev) for r in range(world)]
                    k.xgmi_allreduce_emu(kind, xs, [], [], None, regions[kind], sig, cap, 1e-5)
                    ref = _expected(world, n, seed, dtype, True)
                    for r in range(world):
                        assert torch.equal(xs[r].cpu(), ref), (it, kind, n, r)
                # fused one-shot and two-shot: M rows of H, incl. M < ranks and M not a
                # multiple of the grid; residual identical on every rank
                for kind, (M, H) in ((2, (16, 8192)), (3, (256, 8192)), (3, (3, 4096)),
                                     (3, (300, 4096)), (2, (1, 16384)), (3, (40, 16384))):
                    seed += 1
                    g = torch.Generator().manual_seed(seed)
                    xs = [(torch.randn(M, H, generator=g) * 0.5).to(dtype) for _ in range(world)]
                    res = torch.randn(M, H, generator=g).to(dtype)
                    w = (torch.rand(H, generator=g) + 0.5).to(dtype)
                    ins = [x.to(dev) for x in xs]
                    outs = [torch.empty(M, H, dtype=dtype, device=dev) for _ in range(world)]
                    rss = [res.to(dev) for _ in range(world)]
                    k.xgmi_allreduce_emu(kind, ins, outs, rss, w.to(dev), regions[kind], sig, cap,
                                         1e-5)
                    h = torch.zeros(M, H)
                    for x in xs:
                        h += x.float()
                    rr = (h.to(dtype).float() + res.float()).to(dtype).float()
                    oo = rr * torch.rsqrt(rr.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
                    for r in range(world):
                        # every rank ends with the same bytes
                        assert torch.equal(rss[r].cpu(), rss[0].cpu()), (kind, M, H, r)
                        assert torch.equal(outs[r].cpu(), outs[0].cpu()), (kind, M, H, r)
                    torch.testing.assert_close(rss[0].cpu().float(), rr, atol=2e-2, rtol=1e-2)
                    torch.testing.assert_close(outs[0].cpu().float(), oo, atol=3e-2, rtol=3e-2)
        torch.cuda.synchronize()
        for b in bases:
            assert int(k.ar_read_err(b)) == 0
    finally:
        torch.cuda.synchronize()
        for b in bases:
            k.ar_free(b)


def test_comm_probe_two_ranks_on_one_gpu(gpu, tmp_path):
    """benchmarks/comm_probe.py (run by bench.py at N > 1 on the real node): two ranks on
    cuda:0 with gloo standing in for RCCL; the xGMI kernel rows must be correct and the
    table complete (one-shot, two-shot, library time per size, crossover)."""
    import json
    import subprocess
    import sys
    port = _port()
    out = tmp_path / "probe.json"
    procs = [subprocess.Popen([sys.executable, "-m", "kubernetes_gpu_cluster_amd.benchmarks.comm_probe",
                               "--rank", str(r), "--world", "2", "--port", str(port), "--device", "0",
                               "--backend", "gloo", "--iters", "3"]
                              + (["--out", str(out)] if r == 0 else []))
             for r in range(2)]
    for p in procs:
        assert p.wait(timeout=110) == 0
    res = json.loads(out.read_text())
    assert res["world"] == 2 and res["rccl_correct"]
    assert len(res["rccl"]) == 4 and all(r["us"] > 0 for r in res["rccl"])
    assert len(res["xgmi"]) == 6 and all(r["correct"] for r in res["xgmi"])
    assert len(res["crossover"]["best_per_size"]) == 6


@pytest.mark.parametrize("world", [2, 8])
def test_phantom_rank_runs_every_form_without_waiting(world, gpu):
    """KGC_TP_PHANTOM's all-reduce (parallel/custom_allreduce.py PhantomAllReduce): rank 0
    of a TP = ``world`` group whose peers never run.  Their arrival flags are raised
    ahead of every epoch, so each kernel form completes its whole sequence without a
    time-out, and with zero peer data its outputs have an exact structure:
      one-shot: x (this rank's input + zeros);
      two-shot: x on this rank's owned segment, zeros on the peers' (their reduced
                segments are read from their buffers);
      fused one- / two-shot add + RMSNorm: residual + (x on the rows this rank reduces).
    Run twice per form (both data parities) and inside a captured graph."""
    from kubernetes_gpu_cluster_amd import ops
    from kubernetes_gpu_cluster_amd.parallel.custom_allreduce import PhantomAllReduce
    dev = torch.device("cuda", 0)
    car = PhantomAllReduce(0, world, dev, cap_bytes=4 << 20, one_shot_max=256 << 10)
    car.fused_max, car.fused2_max = 256 << 10, 4 << 20
    try:
        g = torch.Generator().manual_seed(3)
        for rep in range(2):
            small = torch.randint(-8, 9, (64, 512), generator=g).to(torch.bfloat16).to(dev)
            y = small.clone()
            car.all_reduce(y)
            assert torch.equal(y, small)
            big = torch.randint(-8, 9, (256, 4096), generator=g).to(torch.bfloat16).to(dev)
            flat, seg = big.view(-1), big.numel() // world
            exp = torch.zeros_like(flat)
            exp[:seg] = flat[:seg]
            for wide in (False, True):             # 2 MB > one-shot max: two-shot
                car.wide_min = 0 if wide else 1 << 62
                y = big.clone()
                car.all_reduce(y)
                assert torch.equal(y.view(-1), exp), wide
            assert car.launches["two_wide"] > 0 and car.launches["two"] > 0
            for rows in (16, 256):                 # 128 KB fused one-shot, 2 MB two-shot
                x = torch.randint(-8, 9, (rows, 4096), generator=g).to(torch.bfloat16).to(dev)
                res = torch.randint(-8, 9, (rows, 4096), generator=g).to(torch.bfloat16).to(dev)
                w = torch.ones(4096, dtype=torch.bfloat16, device=dev)
                r2 = res.clone()
                out, r2 = car.all_reduce_add_rms(x, r2, w, 1e-6)
                h = x.clone()
                if rows * 4096 * 2 > car.fused_max:
                    # row-segmented: this rank reduces the rows it owns, (row + row / 128) % NR
                    own = torch.tensor([(r + r // 128) % world == 0 for r in range(rows)],
                                       device=dev)
                    h[~own] = 0
                ref_res = (res.float() + h.float()).to(torch.bfloat16)
                assert torch.equal(r2, ref_res)
                ref_out = ops.reference.rms_norm(ref_res.float(), w.float(), 1e-6)
                torch.testing.assert_close(out.float(), ref_out, atol=2e-2, rtol=2e-2)
        # the same kernels captured and replayed (epochs come from device memory)
        x = torch.randint(-8, 9, (64, 512), generator=g).to(torch.bfloat16).to(dev)
        y = x.clone()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            y.copy_(x)
            car.all_reduce(y)
        for _ in range(3):
            gr.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, x)
        car.check()                                # no barrier ever timed out
    finally:
        car.close()
