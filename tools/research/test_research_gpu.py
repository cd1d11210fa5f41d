"""GPU numerics of the research decode GEMMs (measured slower than the shipped K9m, kept
as reproducible negative results; profiles/README.md "Round 3: K9r" / "Round 3: K9v").
They live in their own library (tools/research/build.py -> _kgc_research.so), out of the
engine's, so this file is not part of ``pytest tests/``:

    python tools/research/build.py && python -m pytest tools/research/test_research_gpu.py -q
"""
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


@pytest.fixture(scope="session")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    return torch.device("cuda:0")


def _research():
    sys.path.insert(0, HERE)
    import build as research_build
    return research_build.load()


@pytest.mark.parametrize("cfg", range(18))
def test_ring_gemm_matches_fp32(gpu, cfg):
    """K9r ring GEMM (gemm_ring.hip, every tile config) vs an fp32 matmul: bf16 output,
    fp32 split-K slices (S = 2, 3: uneven K ranges, XCD-mapped) and the SiLU epilogue over
    the 8-row gate / up interleave; M not a multiple of BM (clamped loads, masked rows)."""
    k = _research()
    bm, bn, thr, ns = k.ring_cfg_info(cfg)
    N, K = bn * 16, 640
    M = bm - 37 if bm > 64 else bm + 5
    torch.manual_seed(cfg)
    x = torch.randn(M, K, dtype=torch.bfloat16, device=gpu)
    w = torch.randn(N, K, dtype=torch.bfloat16, device=gpu) * 0.02
    ref = x.float().cpu() @ w.float().cpu().t()

    def packed(silu):
        p = torch.empty(N // bn, K // 64, bn * 64, dtype=w.dtype, device=gpu)
        k.ring_pack(p, w, silu)
        return p
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    k.ring_gemm(out, x, packed(False), cfg, 1)
    torch.testing.assert_close(out.float().cpu(), ref, atol=3e-2, rtol=2e-2)
    for S in (2, 3):
        ws = torch.full((S, M, N), float("nan"), dtype=torch.float32, device=gpu)
        k.ring_gemm(ws, x, packed(False), cfg, 0)
        torch.testing.assert_close(ws.sum(0).cpu(), ref, atol=2e-3, rtol=2e-3)
    act = torch.empty(M, N // 2, dtype=torch.bfloat16, device=gpu)
    k.ring_gemm(act, x, packed(True), cfg, 2)
    exp = torch.nn.functional.silu(ref[:, : N // 2]) * ref[:, N // 2:]
    torch.testing.assert_close(act.float().cpu(), exp, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("depth", [2, 3, 4])
@pytest.mark.parametrize("M,N,K", [(256, 1024, 4096), (200, 768, 1024), (130, 256, 128)])
def test_vreg_gemm_matches_fp32(gpu, depth, M, N, K):
    """K9v (activations in a VGPR ring) over the engine's packed weights vs fp32: bf16
    output, fp32 split-K slices (K = 128 leaves slices of one or two K-steps, fewer than the
    prefetch depth: the filler groups and the tail waits) and the SiLU epilogue."""
    r = _research()
    k = torch.ops.kgc
    from kubernetes_gpu_cluster_amd import ops
    ops.load_extension(strict=True)
    torch.manual_seed(M + N + depth)
    x = torch.randn(M, K, dtype=torch.bfloat16, device=gpu)
    w = torch.randn(N, K, dtype=torch.bfloat16, device=gpu) * 0.02
    ref = x.float().cpu() @ w.float().cpu().t()

    def packed(silu):
        p = torch.empty(N // 128, K // 64, 8192, dtype=w.dtype, device=gpu)
        k.dgemm_pack(p, w, silu)
        return p
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    r.dgemm_vreg(out, x, packed(False), depth, 1)
    torch.testing.assert_close(out.float().cpu(), ref, atol=3e-2, rtol=2e-2)
    for S in (s for s in (2, 3) if s <= K // 64):
        ws = torch.full((S, M, N), float("nan"), dtype=torch.float32, device=gpu)
        r.dgemm_vreg(ws, x, packed(False), depth, 0)
        torch.testing.assert_close(ws.sum(0).cpu(), ref, atol=2e-3, rtol=2e-3)
    act = torch.empty(M, N // 2, dtype=torch.bfloat16, device=gpu)
    r.dgemm_vreg(act, x, packed(True), depth, 2)
    exp = torch.nn.functional.silu(ref[:, : N // 2]) * ref[:, N // 2:]
    torch.testing.assert_close(act.float().cpu(), exp, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("depth", [2, 3])
@pytest.mark.parametrize("M,N,K", [(256, 1024, 4096), (200, 768, 1024), (1, 512, 128),
                                   (130, 256, 192)])
def test_wv_gemm_matches_fp32(gpu, depth, M, N, K):
    """K9w (weights private per wave in a VGPR ring, activations through LDS) over its own
    packed layout vs fp32: bf16 output, fp32 split-K slices (slices of one to three K-steps,
    fewer than the prefetch depth: filler groups and tail waits) and the SiLU epilogue."""
    r = _research()
    torch.manual_seed(M + N + depth)
    x = torch.randn(M, K, dtype=torch.bfloat16, device=gpu)
    w = torch.randn(N, K, dtype=torch.bfloat16, device=gpu) * 0.02
    ref = x.float().cpu() @ w.float().cpu().t()

    def packed(silu):
        p = torch.empty(N // 256, K // 64, 16384, dtype=w.dtype, device=gpu)
        r.wv_pack(p, w, silu)
        return p
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    r.dgemm_wv(out, x, packed(False), depth, 1)
    torch.testing.assert_close(out.float().cpu(), ref, atol=3e-2, rtol=2e-2)
    for S in (s for s in (2, 3) if s <= K // 64):
        ws = torch.full((S, M, N), float("nan"), dtype=torch.float32, device=gpu)
        r.dgemm_wv(ws, x, packed(False), depth, 0)
        torch.testing.assert_close(ws.sum(0).cpu(), ref, atol=2e-3, rtol=2e-3)
    act = torch.empty(M, N // 2, dtype=torch.bfloat16, device=gpu)
    r.dgemm_wv(act, x, packed(True), depth, 2)
    exp = torch.nn.functional.silu(ref[:, : N // 2]) * ref[:, N // 2:]
    torch.testing.assert_close(act.float().cpu(), exp, atol=3e-2, rtol=2e-2)
