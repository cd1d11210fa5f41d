// torch op registrations (namespace "kgc_research") for the measured-not-shipped decode
// GEMM variants K9r (gemm_ring.hip) and K9v (gemm_vreg.hip).  tools/ring_bench.py,
// tools/dgemm_bench.py --research and tools/research/test_research_gpu.py load this library;
// the engine never does.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "research.h"

namespace {

using at::Tensor;

hipStream_t stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "kgc_research: ", name, " must be a GPU tensor");
}

// K9r full-K ring decode GEMM.  Wp: [N/G, K/64, G*64] from ring_pack (G-row groups).
void ring_gemm(Tensor C, Tensor X, Tensor Wp, int64_t cfg, int64_t epi) {
  check_gpu(X, "X");
  c10::hip::HIPGuardMasqueradingAsCUDA g(X.device());
  TORCH_CHECK(cfg >= 0 && cfg < kgc::ring_num_cfgs(), "unknown ring tile config");
  int bm, bn, threads, slots;
  kgc::ring_cfg_info((int)cfg, &bm, &bn, &threads, &slots);
  TORCH_CHECK(epi >= 0 && epi <= 2, "epi 0 (fp32 slices), 1 (out), 2 (silu pairs)");
  TORCH_CHECK(Wp.scalar_type() == at::kBFloat16 && X.scalar_type() == at::kBFloat16, "bf16");
  TORCH_CHECK(Wp.dim() == 3 && Wp.is_contiguous() && Wp.size(2) % 512 == 0,
              "packed W [N/G, K/64, G*64] contiguous");
  const int64_t G = Wp.size(2) / 64, N = Wp.size(0) * G, K = Wp.size(1) * 64;
  TORCH_CHECK(G == bn, "W must be packed with G = the config's BN (ring_pack)");
  TORCH_CHECK(X.dim() == 2 && X.size(1) == K && X.stride(1) == 1 && X.stride(0) % 8 == 0 &&
              reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0,
              "X [M, K] bf16, 16-B aligned rows");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(Wp.data_ptr()) % 16 == 0, "W 16-B aligned");
  TORCH_CHECK(X.device() == Wp.device() && C.device() == X.device(), "same device");
  const int64_t M = X.size(0);
  TORCH_CHECK(N % bn == 0 && K >= 64, "N % BN == 0");
  TORCH_CHECK(M <= (int64_t)1 << 20 && N < ((int64_t)1 << 31) / 4, "size limits");
  int64_t S = 1, ss = 0;
  if (epi == 0) {
    TORCH_CHECK(C.scalar_type() == at::kFloat && C.dim() == 3 && C.is_contiguous() &&
                C.size(1) == M && C.size(2) == N, "C fp32 contiguous [S, M, N]");
    S = C.size(0);
    ss = C.stride(0);
    TORCH_CHECK(S >= 1 && S <= 8 && S <= K / 64, "1 <= S <= min(8, K / 64)");
  } else {
    TORCH_CHECK(C.scalar_type() == at::kBFloat16 && C.dim() == 2 && C.is_contiguous() &&
                C.size(0) == M && C.size(1) == (epi == 2 ? N / 2 : N),
                "C [M, N] (epi 1) or [M, N/2] (epi 2), contiguous bf16");
  }
  TORCH_CHECK((M + bm - 1) / bm * (N / bn) * S < ((int64_t)1 << 31), "grid too large");
  if (M == 0) return;
  kgc::launch_ring_gemm((int)cfg, (int)epi, C.data_ptr(), X.data_ptr(), Wp.data_ptr(), (int)M,
                        (int)N, (int)K, X.stride(0), (int)S, ss, stream());
}

// P [N/G, K/64, G*64] <- W [N, K] (silu: merged [gate; up], 8-row gate / up interleave)
void ring_pack(Tensor P, Tensor W, bool silu) {
  check_gpu(W, "W");
  c10::hip::HIPGuardMasqueradingAsCUDA g(W.device());
  TORCH_CHECK(W.dim() == 2 && W.is_contiguous() && W.scalar_type() == at::kBFloat16,
              "W [N, K] contiguous bf16");
  TORCH_CHECK(P.scalar_type() == at::kBFloat16 && P.dim() == 3 && P.is_contiguous() &&
              P.size(2) % 512 == 0, "P [N/G, K/64, G*64] contiguous bf16");
  const int64_t N = W.size(0), K = W.size(1), G = P.size(2) / 64;
  TORCH_CHECK(K % 64 == 0 && N % G == 0 && P.size(0) == N / G && P.size(1) == K / 64,
              "P shape [N/G, K/64, G*64] for W [N, K]");
  TORCH_CHECK(!silu || N % 32 == 0, "silu: N % 32 == 0");
  TORCH_CHECK(P.device() == W.device(), "same device");
  kgc::launch_ring_pack(silu, P.data_ptr(), W.data_ptr(), (int)N, (int)K, (int)G, stream());
}

std::vector<int64_t> ring_cfg_info(int64_t cfg) {
  TORCH_CHECK(cfg >= 0 && cfg < kgc::ring_num_cfgs(), "unknown ring tile config");
  int bm, bn, threads, slots;
  kgc::ring_cfg_info((int)cfg, &bm, &bn, &threads, &slots);
  return {bm, bn, threads, slots};
}
int64_t ring_num_cfgs() { return kgc::ring_num_cfgs(); }


// K9v over the engine's packed weights [N/128, K/64, 8192]
void dgemm_vreg(Tensor C, Tensor X, Tensor W, int64_t depth, int64_t epi) {
  check_gpu(X, "X");
  c10::hip::HIPGuardMasqueradingAsCUDA g(X.device());
  TORCH_CHECK(depth >= 2 && depth <= 4, "depth 2..4");
  TORCH_CHECK(epi >= 0 && epi <= 2, "epi 0 (fp32 slices), 1 (out), 2 (silu pairs)");
  TORCH_CHECK(W.scalar_type() == at::kBFloat16 && X.scalar_type() == at::kBFloat16, "bf16");
  TORCH_CHECK(W.dim() == 3 && W.is_contiguous() && W.size(2) == 8192,
              "packed W [N/128, K/64, 8192] contiguous");
  const int64_t N = W.size(0) * 128, K = W.size(1) * 64, M = X.size(0);
  TORCH_CHECK(X.dim() == 2 && X.size(1) == K && X.stride(1) == 1 && X.stride(0) % 8 == 0 &&
              reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0, "X [M, K], 16-B rows");
  TORCH_CHECK(M >= 1 && M <= 256, "K9v takes one 256-row tile: 1 <= M <= 256");
  TORCH_CHECK(X.device() == W.device() && C.device() == X.device(), "same device");
  int64_t S = 1, ss = 0;
  if (epi == 0) {
    TORCH_CHECK(C.scalar_type() == at::kFloat && C.dim() == 3 && C.is_contiguous() &&
                C.size(1) == M && C.size(2) == N, "C fp32 contiguous [S, M, N]");
    S = C.size(0);
    ss = C.stride(0);
    TORCH_CHECK(S >= 1 && S <= 32 && S <= K / 64, "1 <= S <= min(32, K / 64)");
  } else {
    TORCH_CHECK(C.scalar_type() == at::kBFloat16 && C.dim() == 2 && C.is_contiguous() &&
                C.size(0) == M && C.size(1) == (epi == 2 ? N / 2 : N), "C [M, N] / [M, N/2] bf16");
  }
  kgc::launch_dgemm_vreg((int)depth, (int)epi, C.data_ptr(), X.data_ptr(), W.data_ptr(), (int)M,
                         (int)N, (int)K, X.stride(0), (int)S, ss, stream());
}

// K9w: weights private per wave (VGPR ring), activations through LDS; P from wv_pack
void dgemm_wv(Tensor C, Tensor X, Tensor P, int64_t depth, int64_t epi) {
  check_gpu(X, "X");
  c10::hip::HIPGuardMasqueradingAsCUDA g(X.device());
  TORCH_CHECK(depth >= 2 && depth <= 3, "depth 2..3");
  TORCH_CHECK(epi >= 0 && epi <= 2, "epi 0 (fp32 slices), 1 (out), 2 (silu pairs)");
  TORCH_CHECK(P.scalar_type() == at::kBFloat16 && X.scalar_type() == at::kBFloat16, "bf16");
  TORCH_CHECK(P.dim() == 3 && P.is_contiguous() && P.size(2) == 16384,
              "packed W [N/256, K/64, 16384] contiguous");
  const int64_t N = P.size(0) * 256, K = P.size(1) * 64, M = X.size(0);
  TORCH_CHECK(X.dim() == 2 && X.size(1) == K && X.stride(1) == 1 && X.stride(0) % 8 == 0 &&
              reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0, "X [M, K], 16-B rows");
  TORCH_CHECK(M >= 1 && M <= 256, "K9w takes one 256-row tile: 1 <= M <= 256");
  TORCH_CHECK(X.device() == P.device() && C.device() == X.device(), "same device");
  int64_t S = 1, ss = 0;
  if (epi == 0) {
    TORCH_CHECK(C.scalar_type() == at::kFloat && C.dim() == 3 && C.is_contiguous() &&
                C.size(1) == M && C.size(2) == N, "C fp32 contiguous [S, M, N]");
    S = C.size(0);
    ss = C.stride(0);
    TORCH_CHECK(S >= 1 && S <= 32 && S <= K / 64, "1 <= S <= min(32, K / 64)");
  } else {
    TORCH_CHECK(C.scalar_type() == at::kBFloat16 && C.dim() == 2 && C.is_contiguous() &&
                C.size(0) == M && C.size(1) == (epi == 2 ? N / 2 : N), "C [M, N] / [M, N/2] bf16");
  }
  kgc::launch_dgemm_wv((int)depth, (int)epi, C.data_ptr(), X.data_ptr(), P.data_ptr(), (int)M,
                       (int)N, (int)K, X.stride(0), (int)S, ss, stream());
}

void wv_pack(Tensor P, Tensor W, bool silu) {
  check_gpu(W, "W");
  c10::hip::HIPGuardMasqueradingAsCUDA g(W.device());
  TORCH_CHECK(W.dim() == 2 && W.is_contiguous() && W.scalar_type() == at::kBFloat16,
              "W [N, K] contiguous bf16");
  const int64_t N = W.size(0), K = W.size(1);
  TORCH_CHECK(N % 256 == 0 && K % 64 == 0, "N % 256 == 0, K % 64 == 0");
  TORCH_CHECK(P.scalar_type() == at::kBFloat16 && P.is_contiguous() && P.dim() == 3 &&
              P.size(0) == N / 256 && P.size(1) == K / 64 && P.size(2) == 16384,
              "P [N/256, K/64, 16384] contiguous bf16");
  TORCH_CHECK(P.device() == W.device(), "same device");
  kgc::launch_wv_pack(silu, P.data_ptr(), W.data_ptr(), (int)N, (int)K, stream());
}

}  // namespace

TORCH_LIBRARY(kgc_research, m) {
  m.def("ring_gemm(Tensor(a!) C, Tensor X, Tensor Wp, int cfg, int epi) -> ()");
  m.def("ring_pack(Tensor(a!) P, Tensor W, bool silu) -> ()");
  m.def("ring_cfg_info(int cfg) -> int[]", &ring_cfg_info);
  m.def("ring_num_cfgs() -> int", &ring_num_cfgs);
  m.def("dgemm_vreg(Tensor(a!) C, Tensor X, Tensor W, int depth, int epi) -> ()");
  m.def("dgemm_wv(Tensor(a!) C, Tensor X, Tensor P, int depth, int epi) -> ()");
  m.def("wv_pack(Tensor(a!) P, Tensor W, bool silu) -> ()");
}

TORCH_LIBRARY_IMPL(kgc_research, CUDA, m) {
  m.impl("ring_gemm", &ring_gemm);
  m.impl("ring_pack", &ring_pack);
  m.impl("dgemm_vreg", &dgemm_vreg);
  m.impl("dgemm_wv", &dgemm_wv);
  m.impl("wv_pack", &wv_pack);
}
