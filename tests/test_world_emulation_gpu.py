"""8-rank peer-memory collectives on ONE GPU, without relying on co-resident processes.

The node these kernels target has one MI355X per rank; the test box has one GPU, and
eight processes' spin-waiting kernels need not be resident on it at once.  Here every
rank lives in this one process with its OWN uncached buffer (``ar_alloc``, the same
allocation the IPC path maps), and each phase of a collective is launched rank after
rank in stream order, so every flag a kernel waits for was raised by a kernel that ran
before it -- the flag / epoch / parity / credit protocols run at NR = 8 exactly as across
GPUs.  (The xGMI all-reduce, whose ranks wait for each other INSIDE one kernel, has a
single-launch emulation of its own: test_allreduce_gpu.py::test_xgmi_world_emulation.)

  * C7 expert-parallel dispatch / receive / return / combine (ep_a2a.hip) at NR = 2/4/8;
  * C5 pipeline handoff (pp_handoff.hip) along an 8-stage chain, two ring slots.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def k():
    from kubernetes_gpu_cluster_amd import ops
    ops.load_extension(strict=True)
    return torch.ops.kgc


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ep_all_to_all_world_emulation(world, gpu, k):
    """Every rank routes its tokens' top-2 experts over NR ranks (E_local experts each);
    the owners apply a per-expert map (row * (expert + 1)) to exactly the rows that
    arrived and send them back; combine == sum_j w_j * (e_j + 1) * x_t on every rank.
    Three calls: the regions' call parity flips and the device epoch advances."""
    dt, H, topk, E_local = torch.bfloat16, 256, 2, 2
    E = world * E_local
    C = 64 * topk
    sig_b = int(k.ep_signal_bytes())
    nbytes = sig_b + int(k.ep_region_bytes(world, C, H, 2))
    bases = [int(k.ar_alloc(nbytes)) for _ in range(world)]
    sig, data = bases, [b + sig_b for b in bases]
    try:
        for call, T in enumerate((5, 64, 17)):
            g = torch.Generator().manual_seed(100 + call)
            xs = [torch.randint(-4, 5, (T, H), generator=g).to(dt).to(gpu) for _ in range(world)]
            ids = [torch.stack([torch.randperm(E, generator=g)[:topk] for _ in range(T)])
                   .to(torch.int32).to(gpu) for _ in range(world)]
            ws = [torch.rand(T, topk, generator=g).to(gpu) for _ in range(world)]
            for r in range(world):
                k.ep_dispatch(xs[r], ids[r], data, sig, r, E_local, C)
            slots = world * C
            back = []
            for d in range(world):
                x_local = torch.empty(slots, H, dtype=dt, device=gpu)
                sids = torch.empty(slots, dtype=torch.int32, device=gpu)
                route = torch.empty(slots, dtype=torch.int32, device=gpu)
                k.ep_receive(x_local, sids, route, data, sig, d, E_local, C)
                valid = sids >= 0
                # owner-side check: exactly the pairs routed to d arrived, with d's experts
                assert int(valid.sum()) == sum(int(((i // E_local) == d).sum()) for i in ids)
                assert bool(((sids[valid] // E_local) == d).all())
                y = x_local * (sids.clamp(min=0) + 1).to(dt).unsqueeze(1)
                back.append((y.contiguous(), route))
            for d in range(world):
                k.ep_return(back[d][0], back[d][1], data, sig, d, C)
            for r in range(world):
                out = torch.empty(T, H, dtype=dt, device=gpu)
                k.ep_combine(out, ws[r], data, sig, r, C)
                scale = (ws[r] * (ids[r].float() + 1)).sum(1, keepdim=True)
                exp = (xs[r].float() * scale).to(dt)
                torch.testing.assert_close(out.float().cpu(), exp.float().cpu(), atol=0.1,
                                           rtol=1e-2)
        torch.cuda.synchronize()
        for b in bases:
            assert int(k.ep_read_err(b)) == 0
    finally:
        torch.cuda.synchronize()
        for b in bases:
            k.ar_free(b)


def test_pp_handoff_eight_stage_chain(gpu, k):
    """Hidden + residual rows travel stage 0 -> 7 through the handoff kernels (each stage
    adds its index to the hidden rows, as its layers would change them), two micro-batches
    in flight per link (ring of R = 2 slots), over six steps: availability and credit
    counters, slot rotation and the receiver's static tensors at every link."""
    stages, rows, H, R = 8, 16, 512, 2
    dt = torch.bfloat16
    sb = int(k.pp_signal_bytes())
    slot_bytes = (rows * H * 2 + 15) // 16 * 16
    bases = [int(k.ar_alloc(2 * sb + R * 2 * slot_bytes)) for _ in range(stages)]
    send_sig = bases
    recv_sig = [b + sb for b in bases]
    own_data = [b + 2 * sb for b in bases]
    h_in = [torch.zeros(rows, H, dtype=dt, device=gpu) for _ in range(stages)]
    r_in = [torch.zeros(rows, H, dtype=dt, device=gpu) for _ in range(stages)]
    try:
        for step in range(0, 6, 2):
            # two micro-batches enter stage 0 back to back (both ring slots in use)
            mbs = []
            for j in range(2):
                g = torch.Generator().manual_seed(10 * step + j)
                h = torch.randint(-8, 8, (rows, H), generator=g).to(dt).to(gpu)
                r = torch.randint(-8, 8, (rows, H), generator=g).to(dt).to(gpu)
                mbs.append((h, r))
                k.pp_send(h, r, own_data[1], recv_sig[1], send_sig[0], slot_bytes, R)
            for s in range(1, stages):
                outs = []
                for j in range(2):
                    k.pp_recv(h_in[s], r_in[s], own_data[s], recv_sig[s], send_sig[s - 1],
                              slot_bytes, R)
                    outs.append((h_in[s] + s, r_in[s].clone()))
                    if s == stages - 1:
                        h0, r0 = mbs[j]
                        exp_h = h0.float() + sum(range(1, stages))
                        assert torch.equal(outs[-1][0].float().cpu(), exp_h.cpu()), (step, j)
                        assert torch.equal(outs[-1][1].cpu(), r0.cpu()), (step, j)
                if s < stages - 1:
                    for h, r in outs:
                        k.pp_send(h.contiguous(), r, own_data[s + 1], recv_sig[s + 1],
                                  send_sig[s], slot_bytes, R)
        torch.cuda.synchronize()
        for b in bases:
            assert int(k.pp_read_err(b)) == 0 and int(k.pp_read_err(b + sb)) == 0
    finally:
        torch.cuda.synchronize()
        for b in bases:
            k.ar_free(b)
