// Host-side launchers for the gfx950 kernels.  Kernel TUs do not include torch
// headers (fast hipcc builds); csrc/bindings.cpp adapts torch tensors to these.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kgc {

enum DType { DT_BF16 = 0, DT_F16 = 1, DT_F32 = 2 };

void launch_rms_norm(int dtype, void* out, const void* x, void* residual, const void* w,
                     int rows, int H, int64_t x_stride, float eps, hipStream_t s);
void launch_layer_norm(int dtype, void* out, const void* x, const void* w, const void* b,
                       int rows, int H, float eps, hipStream_t s);
void launch_silu_mul(int dtype, void* out, const void* x, int64_t rows, int I, hipStream_t s);
// S > 0: qkv is S fp32 split-K slices [S, T, qkv_stride] (slice_stride apart), summed here
void launch_rope_kv_write(int dtype, const void* qkv, int64_t qkv_stride, int S,
                          int64_t slice_stride, const int64_t* positions, const float* cos_sin, void* q_out,
                          void* k_cache, void* v_cache, const int64_t* slot_mapping,
                          const void* q_norm_w, const void* k_norm_w, int T, int nq, int nkv,
                          int d, int bs, float eps, bool use_rope, bool kv_fp8, float k_scale,
                          float v_scale, int num_blocks, hipStream_t s);
// Z > 1: the partials hold B * nq * Z rows (row (seq, q-head) * Z + z), merged by a
// reduce launch
void launch_paged_decode(int dtype, void* out, const void* q, const void* k_cache,
                         const void* v_cache, const int* block_tables, int bt_stride,
                         const int* ctx_lens, float* max_logits, float* exp_sums,
                         float* tmp_out, int B, int nq, int nkv, int D, int bs_log2, int Z,
                         float scale, bool kv_fp8, float k_scale, float v_scale, int num_blocks,
                         hipStream_t s);
// smallest B * nkv that runs K1w (one wave per (seq, kv-head, z-slice)); -1: K1w disabled
// (KGC_DECODE_WAVE=0) and every launch takes the 4-wave workgroup kernel
int paged_decode_wave_min_pairs();
// K1 + K3/K5/K6 fused for decode-only steps: the decode kernel takes the QKV projection
// row itself (T [B, qkv_stride], or S > 0 fp32 split-K slices [S, B, qkv_stride]),
// builds q (optional per-head RMSNorm, NeoX RoPE) in the MFMA operand registers, and
// the workgroup that owns a sequence's last token writes its rotated k and its v into
// the paged cache before reading it back -- no rope_kv launch, no q round trip.
struct DecodeRope {
  const void* qkv;
  int64_t qkv_stride;        // elements between token rows (of one slice when S > 0)
  int64_t slice_stride;      // elements between slices
  int S;                     // 0: qkv holds T values
  int use_rope;
  const int64_t* positions;  // [B]
  const float* cos_sin;      // [max_pos, d]: cos(half) | sin(half)
  const int64_t* slots;      // [B]; < 0: no cache write
  const void* q_norm_w;      // nullptr: no q/k RMSNorm
  const void* k_norm_w;
  float eps, k_inv, v_inv;
  // [B] fp32 or nullptr: row b of the projection is scaled by row_scale[b] before its
  // rounding (the norm-free layer's rsqrt(mean(x^2) + eps) of a gamma-folded QKV weight)
  const float* row_scale;
};
void launch_paged_decode_rope(int dtype, const DecodeRope& rp, void* out, void* k_cache,
                              void* v_cache, const int* block_tables, int bt_stride,
                              const int* ctx_lens, float* max_logits, float* exp_sums,
                              float* tmp_out, int B, int nq, int nkv, int D, int bs_log2,
                              int Z, float scale, bool kv_fp8, float k_scale, float v_scale,
                              int num_blocks, hipStream_t s);
void launch_prefill_attention(int dtype, const void* q, void* out, const void* k_cache,
                              const void* v_cache, const int* block_tables, int bt_stride,
                              const int* query_start_loc, const int* seq_lens,
                              const int* work_seq, const int* work_mblk, int n_work, int nq,
                              int nkv, int D, int bs_log2, float scale, bool kv_fp8,
                              float k_scale, float v_scale, int num_blocks, int64_t q_stride,
                              const float* cos_sin, int cs_rows, hipStream_t s);
// debug builds: sticky bounds-check error words of the K1 / K2 / K3 translation units
// (read and cleared; always 0 in release builds)
uint32_t dbg_err_attention_decode();
uint32_t dbg_err_attention_prefill();
uint32_t dbg_err_rope_cache();
int prefill_block_m();
int sample_splits(int B);   // vocabulary splits per row; partial holds B * splits words
void launch_sample(int dtype, int64_t* out, uint64_t* partial, const void* logits,
                   int64_t row_stride, int B, int V, const float* temperature, const int* top_k,
                   const float* top_p, const int64_t* seeds, hipStream_t s);
// cooperative sampler for rows with top-k / top-p (B <= 256): ws holds
// B * sample_coop_ws_bytes() bytes, all-zero before the first call (the kernel leaves it
// zeroed), partial B * coop splits words
int sample_coop_ws_bytes();
// device address of the sampler's sticky barrier-timeout word (this device)
void* sample_err_addr();
int sample_coop_splits(int B);
void launch_sample_coop(int dtype, int64_t* out, uint64_t* partial, void* ws, const void* logits,
                        int64_t row_stride, int B, int V, const float* temperature,
                        const int* top_k, const float* top_p, const int64_t* seeds,
                        hipStream_t s);
// vocab-parallel: per-row packed (value, global index) of this rank's shard (biased for
// a signed MAX all-reduce), and the unpack after that all-reduce
void launch_sample_vp(int dtype, int64_t* packed, uint64_t* partial, const void* logits,
                      int64_t row_stride, int B, int V, const float* temperature,
                      const int64_t* seeds, int vocab_off, hipStream_t s);
void launch_sample_vp_unpack(int64_t* out, const int64_t* packed, int B, hipStream_t s);

// K9 skinny (small-M decode) GEMM: C[M, N] = X[M, K] . W[N, K]^T (+ bias), M <= 16*mt.
// epi: 0 plain, 1 RMS-normalise X rows on the fly (gamma [K], eps), 2 accumulate into C,
// 3 silu(gate) * up over a merged weight (C [M, N/2]), 4 accumulate into C then
// NO = rms_norm(C) * gamma [N] in the same launch (ticket: a zeroed u32, one per stream),
// 5 accumulate and write ssp[m][workgroup] = sum over the workgroup's columns of C[m]^2,
// 6 / 7 C = rsqrt(sum_j ssp[m][j] / K + eps) * (X W^T) (7: the silu pairs of epi 3), nss
// partials per row (W holds the norm weight folded in)
// cooperative sampler phase stamps (profiling): enable, then read 16 wall-clock stamps
void sample_stamps_enable(bool on);
void sample_stamps_read(uint64_t* out16);

void launch_skinny_gemm(int dtype, int mt, int nt, int nw, bool ntl, int epi, void* C,
                        const void* X, const void* W, const void* bias, const void* gamma,
                        float eps, int M, int N, int K, int64_t ldx, int64_t ldc, void* NO,
                        uint32_t* ticket, float* ssp, int nss, hipStream_t s);

// K13/K14 MoE: routing, expert bucketing, grouped MFMA GEMM, weighted combine.
int moe_block_n();
int moe_block_k();
void launch_moe_route(int dtype, const void* logits, int64_t stride, int ntok, int E, int k,
                      bool renorm, float* topk_w, int* topk_ids, hipStream_t s);
// router GEMM + moe_route in one launch: x [T, H] (rows ldx apart) . wg [E, H]^T, E <= 16,
// H % 512 == 0 -> topk_w fp32 / topk_ids int32 [T, k]
void launch_moe_gate_route(int dtype, const void* x, int64_t ldx, const void* wg, int H, int E,
                           int ntok, int k, bool renorm, float* topk_w, int* topk_ids,
                           hipStream_t s);
void launch_moe_align(const int* topk_ids, int npairs, int e0, int E_local, int bm, int max_rows,
                      int* sorted_ids, int* block_expert, int* meta, hipStream_t s);
// splitk > 1 (scatter only): C is S fp32 slices of slice_stride elements each
void launch_moe_gemm(int dtype, int bm, void* C, const void* A, const void* W,
                     const int* sorted_ids, const int* block_expert, const int* meta, int npairs,
                     int topk, int N, int K, int64_t lda, int64_t ldc, int max_mblocks,
                     bool gather, bool scatter, int splitk, int64_t slice_stride, hipStream_t s);
// dense split-K decode GEMM: Cs [splitk, M, N] fp32 = A [M, K] x W [N, K]^T, XCD-mapped slices
void launch_dense_gemm_splitk(int dtype, int bm, float* Cs, const void* A, const void* W, int M,
                              int N, int K, int64_t lda, int splitk, hipStream_t s);
// K9m mid-batch decode GEMM (gemm_decode.hip): X [M, K] . W^T with tile config `cfg`
// (dgemm_cfg_info: BM x BN, and whether W is the packed [N/128][K/64][128*64] layout of
// launch_dgemm_pack rather than [N, K]).  epi 0: fp32 split-K slice z of C [S, M, N];
// 1: C [M, N] in X's dtype (S = 1); 2: silu(gate) * up of a merged [gate; up] W into
// C [M, N/2] (S = 1; a packed W must have been packed with silu = true).  epi 1 / 2 with
// rsc != nullptr: output row m scaled by rsc[m] (before the SiLU).
struct DgAux {
  const float* rsc;
  // K14m (the MoE grouped GEMM on the K9m pipeline, launch_moe_dgemm): row blocks of one
  // expert each (moe_align), per-expert packed weights wexp elements apart
  const int* sorted_ids;
  const int* block_expert;
  const int* meta;
  int npairs, topk;
  int64_t wexp;
};
// K14m: one grouped MoE projection on the K9m pipeline over per-expert PACKED weights
// Wp [E][N/128][K/64][128*64]: mode 1 = gate_up (A rows gathered from x by sorted_ids / topk,
// SiLU epilogue over the SiLU-packed w13, act [rows, N/2] in sorted-row order); mode 2 =
// down (A = act rows, C rows scattered to pair order; S > 1: fp32 slices [S][npairs][N]).
// bm = 64 | 96 | 128 row blocks (moe_align's), bn = 128 | 256 column tiles, max_rows = rows
// of sorted_ids.
void launch_moe_dgemm(int dtype, int mode, void* C, const void* A, const void* Wp, int max_rows,
                      int N, int K, int64_t lda, int S, int64_t slice_stride, int bm, int bn,
                      const int* sorted_ids, const int* block_expert, const int* meta,
                      int npairs, int topk, hipStream_t s);
int dgemm_num_cfgs();
void dgemm_cfg_info(int cfg, int* bm, int* bn, int* packed);
int dgemm_block_k();
bool dgemm_cfg_has_aux(int cfg);
// epilogues a tile config runs: bit 0 fp32 slices, 1 out, 2 SiLU pairs
int dgemm_cfg_epis(int cfg);
void launch_dgemm(int dtype, int cfg, int epi, void* C, const void* X, const void* W, int M,
                  int N, int K, int64_t ldx, int S, int64_t slice_stride, const DgAux& aux,
                  hipStream_t s);
void launch_dgemm_pack(int dtype, bool silu, void* P, const void* W, int N, int K,
                       hipStream_t s);
void launch_dgemm_ablate(int mode, float* C, const void* X, const void* W, int M, int N, int K,
                         int64_t ldx, int S, int64_t ss, hipStream_t s);
// residual += sum_z Cs[z] (rounded to dtype); out = rms_norm(residual) * w, one WG per row
void launch_splitk_add_rms_norm(int dtype, void* out, const float* Cs, void* residual,
                                const void* w, int rows, int H, int S, int64_t slice_stride,
                                float eps, hipStream_t s);
void launch_splitk_reduce(int dtype, void* out, const float* Cs, int S, int64_t numel,
                          int64_t slice_stride, hipStream_t s);
// silu(gate) * up of the summed gate_up split-K slices: Cs [S, M, 2I] -> out [M, I]
void launch_splitk_reduce_silu(int dtype, void* out, const float* Cs, int S, int M, int I,
                               int64_t slice_stride, bool interleaved, const float* rsc,
                               hipStream_t s);
void launch_moe_combine(int dtype, void* out, const void* y, const float* topk_w,
                        const int* row_map, int64_t nrows, int ntok, int k, int H,
                        int splitk, int64_t slice_stride, hipStream_t s);

// K12 xGMI all-reduce: per-rank [signal | data parity 0 | data parity 1] IPC buffers.
struct ArPtrs {
  void* data[8];
  void* sig[8];
};
// per-rank operand pointers of a world-emulation launch (all ranks on one device)
struct ArWorld {
  void* a[8];
  void* b[8];
  void* c[8];
};
size_t allreduce_signal_bytes();
int allreduce_max_blocks();
// spin-wait bounds (common.h) in ms: {peer (AR/PP/EP), same-kernel (sampler)}, and the
// device's steady-counter rate the bounds assume (kHz)
int peer_spin_ms();
int coop_spin_ms();
int64_t wall_clock_rate_khz();
// wide: the two-shot form on its 256-block grid (its own epochs / flags; P.data: its own
// regions), else the 64-block grid of both forms
void launch_allreduce(int dtype, const ArPtrs& P, int nranks, int rank, void* inout,
                      int64_t nvec, int64_t cap_vec, bool two_shot, bool wide, hipStream_t s);
// fused all-reduce + residual add + RMSNorm over [M, H] rows (P.data: the fused regions
// of the chosen form); H % 8 == 0 and H <= allreduce_rms_max_hidden().  two_shot: the
// row-segmented two-shot kernel (its own regions), else one-shot
int allreduce_rms_max_hidden();
void launch_allreduce_rms(int dtype, const ArPtrs& P, int nranks, int rank, const void* in,
                          void* out, void* residual, const void* w, int M, int H, float eps,
                          int64_t cap_vec, bool two_shot, hipStream_t s);
// world emulation (tests): all nranks ranks' blocks in one launch on one device.
// kind 0 / 1: plain one- / two-shot on W.a[r] (nvec 16-B vectors); 2 / 3: fused one- /
// two-shot with in W.a[r], out W.b[r], residual W.c[r] ([M, H]) and norm weight w
void launch_allreduce_emu(int dtype, int kind, const ArPtrs& P, const ArWorld& W, int nranks,
                          int64_t nvec, const void* w, int M, int H, float eps, int64_t cap_vec,
                          hipStream_t s);
// C7 expert-parallel dispatch / combine over the same kind of IPC buffers (ep_a2a.hip)
using EpPtrs = ArPtrs;
size_t ep_signal_bytes();
int64_t ep_region_bytes(int nr, int C, int H, int esz);
int ep_max_pairs();
void ep_raise_peer_flags(void* sig, int rank, int nranks, uint32_t value, hipStream_t s);
void launch_ep_dispatch(int dtype, const EpPtrs& P, int nr, int rank, const void* x,
                        const int* topk_ids, int npairs, int k, int H, int E_local, int C,
                        hipStream_t s);
void launch_ep_receive(int dtype, const EpPtrs& P, int nr, int rank, void* x_local, int* ids,
                       int* route, int H, int E_local, int C, hipStream_t s);
void launch_ep_return(int dtype, const EpPtrs& P, int nr, int rank, const void* y, int S,
                      int64_t slice_stride, const int* route, int H, int C, hipStream_t s);
void launch_ep_combine(int dtype, const EpPtrs& P, int nr, int rank, void* out,
                       const float* topk_w, int ntok, int k, int H, int C, hipStream_t s);
uint32_t ep_read_err(void* sig);
void ep_err_copy_async(void* sig, uint32_t* host_dst, hipStream_t s);
// C5 pipeline-stage handoff over IPC peer memory (pp_handoff.hip)
size_t pp_signal_bytes();
void launch_pp_send(void* peer_data, void* peer_sig, void* own_sig, const void* h, const void* r,
                    int64_t bytes, int64_t slot_bytes, int R, hipStream_t s);
void launch_pp_recv(void* own_data, void* own_sig, void* peer_sig, void* h, void* r,
                    int64_t bytes, int64_t slot_bytes, int R, hipStream_t s);
uint32_t pp_read_err(void* sig);
void* ar_alloc(int64_t bytes);
void ar_free(void* p);
void ar_get_handle(void* p, uint8_t* out64);
void* ar_open_handle(const uint8_t* in64);
void ar_close_handle(void* p);
uint32_t ar_read_err(void* sig);
void ar_raise_peer_flags(void* sig, int rank, int nranks, uint32_t value, hipStream_t s);
void ar_err_copy_async(void* sig, uint32_t* host_dst, hipStream_t s);

}  // namespace kgc
