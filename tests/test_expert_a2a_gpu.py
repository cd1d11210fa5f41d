"""Device-side expert-parallel all-to-all over IPC peer memory (csrc/kernels/ep_a2a.hip,
parallel/expert_a2a.py) == the MoE block with every expert local, eager and replayed
from a hipGraph.  Two EP ranks share cuda:0 (gloo process group, as in the xGMI
all-reduce tests): the puts, flags and parity buffers run exactly as across GPUs.
Parametrised over the owner's grouped MLP: register-staged or K14m-packed experts, and
a forced down-projection split-K whose fp32 slices ep_return sums on the way back."""
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


def _worker(rank, world, port, packed, splitk):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), KGC_DIST_BACKEND="gloo")
    if splitk:
        os.environ["KGC_MOE_SPLITK"] = splitk
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from kubernetes_gpu_cluster_amd import ops
    from kubernetes_gpu_cluster_amd.models.configs import PRESETS
    from kubernetes_gpu_cluster_amd.models.moe import MoEBlock, set_moe_mode
    from kubernetes_gpu_cluster_amd.ops import reference as ref
    from kubernetes_gpu_cluster_amd.parallel.expert_a2a import ExpertAllToAll
    from kubernetes_gpu_cluster_amd.parallel.state import destroy_parallel, get_state, init_parallel
    init_parallel(tp=world, pp=1, device=dev, rank=rank, world_size=world)
    set_moe_mode("ep")
    cfg = PRESETS["tiny-mixtral"]
    E, H, I = cfg.num_experts, cfg.hidden_size, cfg.intermediate_size
    g = torch.Generator().manual_seed(11)                  # same full weights on every rank
    w13 = (torch.randn(E, 2 * I, H, generator=g) * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, generator=g) * 0.05).to(torch.bfloat16)
    gate = (torch.randn(E, H, generator=g) * 0.5).to(torch.bfloat16)
    blk = MoEBlock(cfg, torch.bfloat16, dev)
    assert blk.mode == "ep" and blk.native
    e0, El = blk.e0, blk.E_local
    blk.w13.data.copy_(w13[e0:e0 + El])
    blk.w2.data.copy_(w2[e0:e0 + El])
    blk.gate.weight.data.copy_(gate)
    if packed:
        assert blk.pack_experts() > 0
    ps = get_state()
    a2a = ExpertAllToAll(ps.tp_cpu_group, ps.tp_rank, ps.tp_size, dev, 64 * blk.k, H,
                         torch.bfloat16)
    blk.ep_a2a = a2a
    assert blk.graph_safe

    def reference(x):
        tw, tid = ops.moe_topk_softmax(blk.gate(x), blk.k)
        return ref.moe_mlp_local(x.cpu().float(), w13.float(), w2.float(), tw.cpu(),
                                 tid.cpu()).float(), tw, tid

    try:
        for T in (1, 5, 64, 33):
            x = (torch.randn(T, H, generator=torch.Generator().manual_seed(100 * T + rank))
                 ).to(torch.bfloat16).to(dev)
            exp, _, _ = reference(x)
            got = blk(x)
            torch.testing.assert_close(got.float().cpu(), exp, atol=3e-2, rtol=3e-2)
        # hipGraph: the whole block, replayed with fresh activations
        T = 8
        xs = torch.zeros(T, H, dtype=torch.bfloat16, device=dev)
        blk(xs)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            out = blk(xs)
        for it in range(4):
            xs.copy_(torch.randn(T, H, generator=torch.Generator().manual_seed(7 * it + rank)))
            gr.replay()
            torch.cuda.synchronize()
            exp, _, _ = reference(xs)
            torch.testing.assert_close(out.float().cpu(), exp, atol=3e-2, rtol=3e-2)
        a2a.check()
        dist.barrier(group=ps.tp_cpu_group)
    finally:
        a2a.close()
        destroy_parallel()


@pytest.mark.parametrize("packed,splitk", [(False, None), (True, "2"), (False, "2")])
def test_expert_a2a_matches_local_experts(gpu, packed, splitk):
    mp.start_processes(_worker, args=(2, _port(), packed, splitk), nprocs=2, join=True,
                       start_method="spawn")
