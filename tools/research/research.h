// Research kernels (measured, not shipped): K9r ring GEMM and K9v VGPR-ring GEMM.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kgc {
// K9r ring decode GEMM (gemm_ring.hip), bf16: X [M, K] . W^T with tile config `cfg`
// (ring_cfg_info: BM, BN, threads, ring slots) over W packed by launch_ring_pack into
// [N/G][K/64][G*64] with G = the config's BN.  epi 0: fp32 split-K slice z of C [S, M, N];
// 1: C [M, N] bf16 (S = 1); 2: silu(gate) * up of a merged [gate; up] W packed with
// silu = true into C [M, N/2] (S = 1)
int ring_num_cfgs();
void ring_cfg_info(int cfg, int* bm, int* bn, int* threads, int* slots);
void launch_ring_gemm(int cfg, int epi, void* C, const void* X, const void* Wp, int M, int N,
                      int K, int64_t ldx, int S, int64_t slice_stride, hipStream_t s);
void launch_ring_pack(bool silu, void* P, const void* W, int N, int K, int G, hipStream_t s);
// K9v (gemm_vreg.hip), bf16, one 256-row tile (M <= 256), W packed by the engine's
// dgemm_pack ([N/128][K/64][8192]); depth = 2, 3 or 4 K-steps in flight
void launch_dgemm_vreg(int depth, int epi, void* C, const void* X, const void* W, int M, int N,
                       int K, int64_t ldx, int S, int64_t ss, hipStream_t s);
// K9w (gemm_wv.hip), bf16, one 256-row tile (M <= 256), 256-column tiles, weights packed by
// launch_wv_pack into [N/256][K/64][16384] (per wave 4 x 1-KB loads per K-step; silu: merged
// [gate; up] with gate / up columns paired per wave); depth 2 or 3 K-steps in flight
void launch_dgemm_wv(int depth, int epi, void* C, const void* X, const void* Wp, int M, int N,
                     int K, int64_t ldx, int S, int64_t ss, hipStream_t s);
void launch_wv_pack(bool silu, void* P, const void* W, int N, int K, hipStream_t s);
}  // namespace kgc
