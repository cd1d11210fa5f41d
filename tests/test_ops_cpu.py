"""CPU paths of the fused ops wrappers: the same signatures the GPU kernels take, checked
against the composition of the reference ops they fuse (ops.reference)."""
import math

import torch

from kubernetes_gpu_cluster_amd import ops
from kubernetes_gpu_cluster_amd.ops import reference as ref


def test_paged_attention_decode_rope_cpu_equals_composition():
    torch.manual_seed(0)
    B, nq, nkv, d, bs = 3, 8, 2, 64, 16
    ctx = [5, 17, 33]
    nb = sum(math.ceil(c / bs) for c in ctx) + 2
    kc = torch.randn(nb, nkv, bs, d)
    vc = torch.randn(nb, nkv, bs // 8, d, 8)
    bt = torch.zeros(B, 4, dtype=torch.int32)
    k = 1
    for b, c in enumerate(ctx):
        n = math.ceil(c / bs)
        bt[b, :n] = torch.arange(k, k + n, dtype=torch.int32)
        k += n
    cl = torch.tensor(ctx, dtype=torch.int32)
    pos = cl.long() - 1
    slots = torch.tensor([int(bt[b, (c - 1) // bs]) * bs + (c - 1) % bs for b, c in enumerate(ctx)])
    qkv = torch.randn(B, (nq + 2 * nkv) * d)
    cs = ref.rope_cos_sin_cache(d, 128, 1e4)
    kc2, vc2 = kc.clone(), vc.clone()
    out = ops.paged_attention_decode_rope(qkv, pos, cs, kc, vc, slots, nq, nkv, d, bt, cl,
                                          d ** -0.5)
    q = ref.rope_qk_kv_write(qkv, pos, cs, kc2, vc2, slots, nq, nkv, d)
    exp = ref.paged_attention_decode(q, kc2, vc2, bt, cl, d ** -0.5)
    torch.testing.assert_close(out, exp)
    torch.testing.assert_close(kc, kc2)
    torch.testing.assert_close(vc, vc2)
