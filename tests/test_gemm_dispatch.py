"""CPU checks of the GEMM dispatch helpers in ops/gemm.py: with no tuned plan (or on
CPU tensors) ``linear_silu`` and ``linear_add_rms`` are exactly the unfused layer math
(``silu_mul(linear)`` / ``fused_add_rms_norm(linear)``), and the tail-fused model path is
never taken off the GPU.  The fused GPU kernels are checked against fp32 references in
test_kernels_gpu.py."""
import torch

from kubernetes_gpu_cluster_amd import ops
from kubernetes_gpu_cluster_amd.ops import gemm


def test_linear_silu_fallback_matches_layer_math():
    torch.manual_seed(0)
    x = torch.randn(5, 64)
    w = torch.randn(96, 64) * 0.1
    y = x @ w.t()
    exp = torch.nn.functional.silu(y[:, :48]) * y[:, 48:]
    torch.testing.assert_close(gemm.linear_silu(x, w), exp, atol=1e-5, rtol=1e-5)


def test_linear_add_rms_fallback_matches_layer_math():
    torch.manual_seed(1)
    x = torch.randn(7, 32)
    w = torch.randn(48, 32) * 0.1
    res = torch.randn(7, 48)
    gamma = torch.rand(48) + 0.5
    r_exp = res + x @ w.t()
    o_exp = ops.reference.rms_norm(r_exp, gamma, 1e-6)
    o, r = gemm.linear_add_rms(x, w, res.clone(), gamma, 1e-6)
    torch.testing.assert_close(r, r_exp, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(o, o_exp, atol=1e-5, rtol=1e-5)


def test_tail_fusion_not_taken_on_cpu():
    from kubernetes_gpu_cluster_amd.models import configs
    from kubernetes_gpu_cluster_amd.models.llama import LlamaForCausalLM
    cfg = configs.PRESETS["tiny-llama"]
    m = LlamaForCausalLM(cfg, torch.float32, torch.device("cpu"))
    gemm._plan_dg[(4, 1, 1, "tail")] = (2, 2)
    try:
        assert not m._tail_fusable(torch.zeros(4, cfg.hidden_size))
    finally:
        gemm.clear_plan()


def test_packed_weight_cache_drops_dead_weights():
    """K9m's packed-weight cache is keyed by the weight's address; an entry must die with
    its weight, so a later tensor allocated at the same address (the next engine in the
    same process) never reads another weight's packed copy."""
    import gc
    from kubernetes_gpu_cluster_amd.ops import gemm
    w = torch.zeros(128, 64)
    packed = torch.ones(3)
    gemm._packed_put(w, False, packed)
    assert gemm._packed_get(w, False) is packed and gemm.packed_weight(w) is packed
    assert gemm._packed_get(w, True) is None
    view = w[:64]                      # same address, different tensor: not the packed weight
    assert gemm._packed_get(view, False) is None
    assert gemm._packed_get(w, False) is packed    # ... and does not evict the entry
    n = len(gemm._packed)
    del w, view
    gc.collect()
    assert len(gemm._packed) == n - 1


def test_rs_plan_rejects_producers_with_too_many_row_partials():
    """the norm-free layer's consumer (SK_RSCALE, ssl[16][256] in LDS)
    sums at most 256 sum-of-squares partials per row, and the producer leaves
    N / (16 nt) of them.  At hidden 5120 (Qwen3-14B, no bias) an nt = 1 producer leaves 320
    -- within the [16 x 256] buffer at M <= 12, but past the consumer's limit: rs_plan must
    refuse it at plan time instead of letting the launch check fail in graph capture."""
    M = 8
    saved = dict(gemm._best_sk), dict(gemm._best_rs), dict(gemm._best_silu)
    try:
        for H, I in ((5120, 17408), (4096, 14336)):
            shapes = [(3 * H, H), (H, H), (2 * I, H), (H, I)]
            gemm._best_rs.clear()
            gemm._best_sk.clear()
            gemm._best_silu.clear()
            # (mt, nt, nw, ntl): one m-tile, nt = 1 on the producers, nw = 4 (M <= 16)
            gemm._best_sk[(M, 3 * H, H)] = (1, 1, 4, True)
            gemm._best_sk[(M, H, H)] = (1, 1, 4, True)
            gemm._best_sk[(M, H, I)] = (1, 1, 4, True)
            gemm._best_silu[(M, 2 * I, H)] = (1, 2, 4, True)
            p = gemm.rs_plan(M, shapes)
            if H // 16 > gemm.RS_MAX_NSS:
                assert p is None, (H, p)
                # nt = 2 halves the partials: 160 per row is a valid plan again
                gemm._best_sk[(M, H, H)] = (1, 2, 4, True)
                gemm._best_sk[(M, H, I)] = (1, 2, 4, True)
                assert gemm.rs_plan(M, shapes) is not None
            else:
                assert p is not None and H // 16 <= gemm.RS_MAX_NSS
        # the [16 x 256] buffer also bounds M * nss: 16 rows x 256 partials fits, 17 do not
        assert gemm.rs_plan(17, [(3 * 4096, 4096), (4096, 4096), (28672, 4096),
                                 (4096, 14336)]) is None
    finally:
        for d, v in zip((gemm._best_sk, gemm._best_rs, gemm._best_silu), saved):
            d.clear()
            d.update(v)
