// torch op registrations (namespace "kgc") for the gfx950 HIP kernels.
// Every op validates shapes/dtypes/devices on the host before launching: a bad
// launch on the MI355X pool can fault the whole node, so nothing reaches a
// kernel unless the kernel's indexing assumptions hold.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "kernels/launch.h"

namespace {

using at::Tensor;

int dt_code(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kBFloat16: return kgc::DT_BF16;
    case at::kHalf: return kgc::DT_F16;
    case at::kFloat: return kgc::DT_F32;
    default: TORCH_CHECK(false, "kgc: unsupported dtype ", t.scalar_type());
  }
  return -1;
}

hipStream_t stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "kgc: ", name, " must be a GPU tensor");
}

void check_same_dev(const Tensor& a, const Tensor& b, const char* name) {
  TORCH_CHECK(a.device() == b.device(), "kgc: ", name, " on a different device");
}

int log2_exact(int64_t v, const char* what) {
  int l = 0;
  while ((int64_t(1) << l) < v) ++l;
  TORCH_CHECK((int64_t(1) << l) == v, "kgc: ", what, " must be a power of two, got ", v);
  return l;
}

void rms_norm(Tensor out, Tensor x, std::optional<Tensor> residual, Tensor w, double eps) {
  check_gpu(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2, "kgc.rms_norm: 2-D [rows, H] expected");
  const int64_t rows = x.size(0), H = x.size(1);
  TORCH_CHECK(H % 8 == 0 && H <= 8192, "kgc.rms_norm: H must be a multiple of 8 and <= 8192");
  TORCH_CHECK(x.stride(1) == 1 && x.stride(0) % 8 == 0, "kgc.rms_norm: x rows must be dense, 16B aligned");
  TORCH_CHECK(out.is_contiguous() && out.sizes() == x.sizes(), "kgc.rms_norm: out shape");
  TORCH_CHECK(w.is_contiguous() && w.numel() == H && w.scalar_type() == x.scalar_type(), "kgc.rms_norm: weight");
  TORCH_CHECK(out.scalar_type() == x.scalar_type(), "kgc.rms_norm: out dtype");
  void* rp = nullptr;
  if (residual.has_value()) {
    TORCH_CHECK(residual->is_contiguous() && residual->sizes() == x.sizes() &&
                residual->scalar_type() == x.scalar_type(), "kgc.rms_norm: residual");
    TORCH_CHECK(x.is_contiguous(), "kgc.rms_norm: fused add needs contiguous x");
    rp = residual->data_ptr();
  }
  kgc::launch_rms_norm(dt_code(x), out.data_ptr(), x.data_ptr(), rp, w.data_ptr(), (int)rows,
                       (int)H, x.stride(0), (float)eps, stream());
}

void layer_norm(Tensor out, Tensor x, Tensor w, Tensor b, double eps) {
  check_gpu(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && out.is_contiguous() && out.sizes() == x.sizes(),
              "kgc.layer_norm: contiguous 2-D");
  const int64_t H = x.size(1);
  TORCH_CHECK(H % 8 == 0 && H <= 8192, "kgc.layer_norm: H");
  TORCH_CHECK(w.numel() == H && b.numel() == H, "kgc.layer_norm: weight/bias");
  kgc::launch_layer_norm(dt_code(x), out.data_ptr(), x.data_ptr(), w.data_ptr(), b.data_ptr(),
                         (int)x.size(0), (int)H, (float)eps, stream());
}

void silu_mul(Tensor out, Tensor x) {
  check_gpu(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && out.is_contiguous(), "kgc.silu_mul: contiguous 2-D");
  const int64_t I = x.size(1) / 2;
  TORCH_CHECK(x.size(1) % 16 == 0 && out.size(0) == x.size(0) && out.size(1) == I,
              "kgc.silu_mul: shapes");
  kgc::launch_silu_mul(dt_code(x), out.data_ptr(), x.data_ptr(), x.size(0), (int)I, stream());
}

// KV cache element type: the activation dtype, or fp8 e4m3 (--kv-cache-dtype fp8)
bool kv_is_fp8(const Tensor& k_cache, const Tensor& v_cache, at::ScalarType act) {
  TORCH_CHECK(k_cache.scalar_type() == v_cache.scalar_type(), "k/v cache dtype mismatch");
  if (k_cache.scalar_type() == at::kFloat8_e4m3fn) return true;
  TORCH_CHECK(k_cache.scalar_type() == act, "kv cache dtype must be the activation dtype or fp8_e4m3fn");
  return false;
}

// qkv: [T, >= (nq+2nkv)*d] in q_out's dtype, or the K9m split-K slices fp32 [S, T, N]
void rope_kv_write(Tensor qkv, Tensor positions, Tensor cos_sin, Tensor q_out, Tensor k_cache,
                   Tensor v_cache, Tensor slot_mapping, std::optional<Tensor> q_norm_w,
                   std::optional<Tensor> k_norm_w, int64_t nq, int64_t nkv, int64_t d,
                   double eps, bool use_rope, double k_scale, double v_scale) {
  check_gpu(qkv, "qkv");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  TORCH_CHECK(d % 16 == 0 && d <= 256, "kgc.rope_kv_write: head_dim");
  const bool slices = qkv.dim() == 3;
  const int64_t T = slices ? qkv.size(1) : qkv.size(0);
  int64_t S = 0, ss = 0, stride;
  if (slices) {
    TORCH_CHECK(qkv.scalar_type() == at::kFloat && qkv.is_contiguous() &&
                qkv.size(2) >= (nq + 2 * nkv) * d && qkv.size(2) % 8 == 0 && qkv.size(0) >= 1,
                "kgc.rope_kv_write: slices fp32 [S, T, (nq+2nkv)*d] contiguous");
    S = qkv.size(0);
    ss = qkv.stride(0);
    stride = qkv.stride(1);
  } else {
    TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.size(1) >= (nq + 2 * nkv) * d &&
                qkv.stride(0) % 8 == 0, "kgc.rope_kv_write: qkv [T, (nq+2nkv)*d]");
    TORCH_CHECK(q_out.scalar_type() == qkv.scalar_type(), "kgc.rope_kv_write: dtype");
    stride = qkv.stride(0);
  }
  TORCH_CHECK(q_out.scalar_type() == at::kBFloat16 || q_out.scalar_type() == at::kHalf,
              "q_out bf16 / fp16");
  TORCH_CHECK(positions.scalar_type() == at::kLong && positions.numel() == T, "positions int64 [T]");
  TORCH_CHECK(slot_mapping.scalar_type() == at::kLong && slot_mapping.numel() == T, "slot_mapping int64 [T]");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() && cos_sin.size(1) == d,
              "cos_sin fp32 [max_pos, d]");
  // an empty q_out: write k / v only (prefill_attention_rope rotates q as it loads it)
  const bool kv_only = q_out.numel() == 0;
  TORCH_CHECK(kv_only || (q_out.is_contiguous() && q_out.numel() == T * nq * d),
              "q_out [T, nq, d] (or empty: k / v only)");
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous() && k_cache.dim() == 4 &&
              v_cache.dim() == 5 && k_cache.size(1) == nkv && k_cache.size(3) == d &&
              v_cache.size(3) == d && v_cache.size(4) == 8 &&
              v_cache.size(2) * 8 == k_cache.size(2), "kv cache layout");
  const bool kv8 = kv_is_fp8(k_cache, v_cache, q_out.scalar_type());
  TORCH_CHECK(k_scale > 0 && v_scale > 0, "kv scales must be > 0");
  const void* qn = nullptr;
  const void* kn = nullptr;
  if (q_norm_w.has_value()) {
    TORCH_CHECK(k_norm_w.has_value() && q_norm_w->numel() == d && k_norm_w->numel() == d, "qk norm weights");
    qn = q_norm_w->data_ptr();
    kn = k_norm_w->data_ptr();
  }
  kgc::launch_rope_kv_write(dt_code(q_out), qkv.data_ptr(), stride, (int)S, ss,
                            positions.data_ptr<int64_t>(), cos_sin.data_ptr<float>(),
                            kv_only ? nullptr : q_out.data_ptr(), k_cache.data_ptr(),
                            v_cache.data_ptr(), slot_mapping.data_ptr<int64_t>(), qn, kn,
                            (int)T, (int)nq, (int)nkv,
                            (int)d, (int)k_cache.size(2), (float)eps, use_rope, kv8,
                            (float)k_scale, (float)v_scale, (int)k_cache.size(0), stream());
}

void check_kv(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, int64_t nq) {
  TORCH_CHECK(k_cache.dim() == 4 && v_cache.dim() == 5 && k_cache.is_contiguous() &&
              v_cache.is_contiguous(), "k_cache 4-D / v_cache 5-D contiguous");
  const int64_t nkv = k_cache.size(1), bs = k_cache.size(2), d = k_cache.size(3);
  TORCH_CHECK(v_cache.size(0) == k_cache.size(0) && v_cache.size(1) == nkv &&
              v_cache.size(2) * 8 == bs && v_cache.size(3) == d && v_cache.size(4) == 8,
              "v_cache must be [nb, nkv, bs/8, d, 8]");
  TORCH_CHECK(d == 64 || d == 128, "head_dim must be 64 or 128");
  TORCH_CHECK(nq % nkv == 0 && nq / nkv <= 16, "GQA group must be <= 16");
  TORCH_CHECK(bs >= 16, "block_size must be >= 16");
  kv_is_fp8(k_cache, v_cache, q.scalar_type());
  TORCH_CHECK(q.scalar_type() != at::kFloat, "attention kernels take bf16/f16");
  check_same_dev(q, k_cache, "k_cache");
  check_same_dev(q, v_cache, "v_cache");
}

// Z > 1 partials: fp32, contiguous, >= B * nq * Z rows (row (seq, q-head) * Z + z)
static void check_partials(const Tensor& ml, const Tensor& es, const Tensor& tmp, int64_t B,
                           int64_t nq, int64_t d, int64_t Z, const char* who) {
  TORCH_CHECK(ml.scalar_type() == at::kFloat && es.scalar_type() == at::kFloat &&
              tmp.scalar_type() == at::kFloat, who, ": partials fp32");
  TORCH_CHECK(ml.is_contiguous() && es.is_contiguous() && tmp.is_contiguous() &&
              ml.numel() >= B * nq * Z && es.numel() >= B * nq * Z &&
              tmp.numel() >= B * nq * Z * d, who, ": partials hold fewer than B * nq * Z rows");
  TORCH_CHECK(Z >= 1 && Z <= 1024, who, ": need 1 <= Z <= 1024");
  TORCH_CHECK(ml.device() == tmp.device() && es.device() == tmp.device(), who,
              ": partials on one device");
}

void paged_decode(Tensor out, Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables,
                  Tensor ctx_lens, Tensor max_logits, Tensor exp_sums, Tensor tmp_out,
                  int64_t Z, double scale, double k_scale, double v_scale) {
  check_gpu(q, "q");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  TORCH_CHECK(q.dim() == 3 && q.is_contiguous(), "q [B, nq, d] contiguous");
  const int64_t B = q.size(0), nq = q.size(1), d = q.size(2);
  check_kv(q, k_cache, v_cache, nq);
  TORCH_CHECK(k_cache.size(3) == d, "head_dim mismatch");
  TORCH_CHECK(out.is_contiguous() && out.sizes() == q.sizes() && out.scalar_type() == q.scalar_type(), "out");
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && block_tables.dim() == 2 &&
              block_tables.size(0) >= B && block_tables.is_contiguous(), "block_tables int32 [B, max_blocks] contiguous");
  TORCH_CHECK(ctx_lens.scalar_type() == at::kInt && ctx_lens.numel() >= B, "ctx_lens int32 [B]");
  check_partials(max_logits, exp_sums, tmp_out, B, nq, d, Z, "kgc.paged_decode");
  check_same_dev(q, tmp_out, "partials");
  kgc::launch_paged_decode(dt_code(q), out.data_ptr(), q.data_ptr(), k_cache.data_ptr(),
                           v_cache.data_ptr(), block_tables.data_ptr<int>(),
                           (int)block_tables.stride(0), ctx_lens.data_ptr<int>(),
                           max_logits.data_ptr<float>(), exp_sums.data_ptr<float>(),
                           tmp_out.data_ptr<float>(), (int)B, (int)nq, (int)k_cache.size(1),
                           (int)d, log2_exact(k_cache.size(2), "block_size"), (int)Z,
                           (float)scale, k_cache.scalar_type() == at::kFloat8_e4m3fn,
                           (float)k_scale, (float)v_scale, (int)k_cache.size(0), stream());
}

// paged_decode with rope_kv_write folded in (decode-only steps): qkv is the projection
// [B, >= (nq+2nkv)*d] in the activation dtype, or its K9m fp32 split-K slices [S, B, N].
void paged_decode_rope(Tensor out, Tensor qkv, Tensor positions, Tensor cos_sin, Tensor k_cache,
                       Tensor v_cache, Tensor slot_mapping, std::optional<Tensor> q_norm_w,
                       std::optional<Tensor> k_norm_w, Tensor block_tables, Tensor ctx_lens,
                       Tensor max_logits, Tensor exp_sums, Tensor tmp_out, int64_t nq,
                       int64_t Z, double scale, double eps, bool use_rope, double k_scale,
                       double v_scale, std::optional<Tensor> row_scale) {
  check_gpu(qkv, "qkv");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  TORCH_CHECK(out.dim() == 3 && out.is_contiguous() && out.size(1) == nq,
              "kgc.paged_decode_rope: out [B, nq, d] contiguous");
  const int64_t B = out.size(0), d = out.size(2), nkv = k_cache.size(1);
  check_kv(out, k_cache, v_cache, nq);
  TORCH_CHECK(k_cache.size(3) == d, "head_dim mismatch");
  kgc::DecodeRope rp{};
  const int64_t N = (nq + 2 * nkv) * d;
  if (qkv.dim() == 3) {
    TORCH_CHECK(qkv.scalar_type() == at::kFloat && qkv.is_contiguous() && qkv.size(1) == B &&
                qkv.size(2) >= N && qkv.size(2) % 8 == 0 && qkv.size(0) >= 1,
                "kgc.paged_decode_rope: slices fp32 [S, B, (nq+2nkv)*d] contiguous");
    rp.S = (int)qkv.size(0);
    rp.slice_stride = qkv.stride(0);
    rp.qkv_stride = qkv.stride(1);
  } else {
    TORCH_CHECK(qkv.dim() == 2 && qkv.size(0) == B && qkv.stride(1) == 1 && qkv.size(1) >= N &&
                qkv.stride(0) % 8 == 0 && qkv.scalar_type() == out.scalar_type(),
                "kgc.paged_decode_rope: qkv [B, (nq+2nkv)*d] in the output dtype");
    rp.S = 0;
    rp.qkv_stride = qkv.stride(0);
  }
  TORCH_CHECK(positions.scalar_type() == at::kLong && positions.numel() == B, "positions int64 [B]");
  TORCH_CHECK(slot_mapping.scalar_type() == at::kLong && slot_mapping.numel() == B,
              "slot_mapping int64 [B]");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() && cos_sin.size(1) == d,
              "cos_sin fp32 [max_pos, d]");
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && block_tables.dim() == 2 &&
              block_tables.size(0) >= B && block_tables.is_contiguous(),
              "block_tables int32 [B, max_blocks] contiguous");
  TORCH_CHECK(ctx_lens.scalar_type() == at::kInt && ctx_lens.numel() >= B, "ctx_lens int32 [B]");
  check_partials(max_logits, exp_sums, tmp_out, B, nq, d, Z, "kgc.paged_decode_rope");
  TORCH_CHECK(k_scale > 0 && v_scale > 0, "kv scales must be > 0");
  for (const Tensor* t : {&qkv, &positions, &cos_sin, &slot_mapping, &block_tables, &ctx_lens,
                          &tmp_out})
    check_same_dev(out, *t, "paged_decode_rope operand");
  if (q_norm_w.has_value()) {
    TORCH_CHECK(k_norm_w.has_value() && q_norm_w->numel() == d && k_norm_w->numel() == d &&
                q_norm_w->scalar_type() == out.scalar_type() &&
                k_norm_w->scalar_type() == out.scalar_type(), "qk norm weights [d]");
    rp.q_norm_w = q_norm_w->data_ptr();
    rp.k_norm_w = k_norm_w->data_ptr();
  }
  if (row_scale.has_value()) {
    TORCH_CHECK(row_scale->scalar_type() == at::kFloat && row_scale->is_contiguous() &&
                row_scale->numel() >= B, "row_scale fp32 [>= B] contiguous");
    check_same_dev(out, *row_scale, "paged_decode_rope row_scale");
    rp.row_scale = row_scale->data_ptr<float>();
  }
  rp.qkv = qkv.data_ptr();
  rp.use_rope = use_rope ? 1 : 0;
  rp.positions = positions.data_ptr<int64_t>();
  rp.cos_sin = cos_sin.data_ptr<float>();
  rp.slots = slot_mapping.data_ptr<int64_t>();
  rp.eps = (float)eps;
  rp.k_inv = (float)(1.0 / k_scale);
  rp.v_inv = (float)(1.0 / v_scale);
  kgc::launch_paged_decode_rope(dt_code(out), rp, out.data_ptr(), k_cache.data_ptr(),
                                v_cache.data_ptr(), block_tables.data_ptr<int>(),
                                (int)block_tables.stride(0), ctx_lens.data_ptr<int>(),
                                max_logits.data_ptr<float>(), exp_sums.data_ptr<float>(),
                                tmp_out.data_ptr<float>(), (int)B, (int)nq, (int)nkv, (int)d,
                                log2_exact(k_cache.size(2), "block_size"), (int)Z,
                                (float)scale, k_cache.scalar_type() == at::kFloat8_e4m3fn,
                                (float)k_scale, (float)v_scale, (int)k_cache.size(0), stream());
}

void prefill_attention(Tensor out, Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables,
                       Tensor query_start_loc, Tensor seq_lens, Tensor work_seq,
                       Tensor work_mblk, double scale, double k_scale, double v_scale) {
  check_gpu(q, "q");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  TORCH_CHECK(q.dim() == 3 && q.is_contiguous(), "q [T, nq, d] contiguous");
  const int64_t nq = q.size(1), d = q.size(2);
  check_kv(q, k_cache, v_cache, nq);
  TORCH_CHECK(k_cache.size(3) == d, "head_dim mismatch");
  TORCH_CHECK(out.is_contiguous() && out.sizes() == q.sizes() && out.scalar_type() == q.scalar_type(), "out");
  const int64_t P = seq_lens.numel();
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && block_tables.dim() == 2 &&
              block_tables.size(0) >= P && block_tables.is_contiguous(), "block_tables contiguous");
  TORCH_CHECK(query_start_loc.scalar_type() == at::kInt && query_start_loc.numel() == P + 1, "query_start_loc");
  TORCH_CHECK(seq_lens.scalar_type() == at::kInt, "seq_lens int32");
  TORCH_CHECK(work_seq.scalar_type() == at::kInt && work_mblk.scalar_type() == at::kInt &&
              work_seq.numel() == work_mblk.numel(), "work list");
  TORCH_CHECK(work_seq.numel() <= 2147483647 && nq <= 65535, "grid");
  kgc::launch_prefill_attention(dt_code(q), q.data_ptr(), out.data_ptr(), k_cache.data_ptr(),
                                v_cache.data_ptr(), block_tables.data_ptr<int>(),
                                (int)block_tables.stride(0), query_start_loc.data_ptr<int>(),
                                seq_lens.data_ptr<int>(), work_seq.data_ptr<int>(),
                                work_mblk.data_ptr<int>(), (int)work_seq.numel(), (int)nq,
                                (int)k_cache.size(1), (int)d,
                                log2_exact(k_cache.size(2), "block_size"), (float)scale,
                                k_cache.scalar_type() == at::kFloat8_e4m3fn, (float)k_scale,
                                (float)v_scale, (int)k_cache.size(0), nq * d, nullptr, 0, stream());
}

// K2 on a prefill-only step with RoPE folded into the q load: qkv [T, >= (nq+2nkv)*d]
// (the unrotated QKV projection; rope_kv_write wrote only k / v), positions implicit
// (ctx0 + row, as the engine assigns them), out [T, nq, d]
void prefill_attention_rope(Tensor out, Tensor qkv, Tensor cos_sin, Tensor k_cache,
                            Tensor v_cache, Tensor block_tables, Tensor query_start_loc,
                            Tensor seq_lens, Tensor work_seq, Tensor work_mblk, int64_t nq,
                            double scale, double k_scale, double v_scale) {
  check_gpu(qkv, "qkv");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  TORCH_CHECK(out.dim() == 3 && out.is_contiguous() && out.size(1) == nq &&
              out.scalar_type() == qkv.scalar_type(), "out [T, nq, d] contiguous, qkv's dtype");
  const int64_t d = out.size(2), T = out.size(0);
  check_kv(out, k_cache, v_cache, nq);
  const int64_t nkv = k_cache.size(1);
  TORCH_CHECK(k_cache.size(3) == d, "head_dim mismatch");
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(0) == T && qkv.stride(1) == 1 &&
              qkv.size(1) >= (nq + 2 * nkv) * d && qkv.stride(0) % 8 == 0 &&
              reinterpret_cast<uintptr_t>(qkv.data_ptr()) % 16 == 0,
              "qkv [T, >= (nq + 2 nkv) d], 16-B aligned rows");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() &&
              cos_sin.dim() == 2 && cos_sin.size(1) == d, "cos_sin fp32 [max_pos, d]");
  const int64_t P = seq_lens.numel();
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && block_tables.dim() == 2 &&
              block_tables.size(0) >= P && block_tables.is_contiguous(), "block_tables contiguous");
  TORCH_CHECK(query_start_loc.scalar_type() == at::kInt && query_start_loc.numel() == P + 1, "query_start_loc");
  TORCH_CHECK(seq_lens.scalar_type() == at::kInt, "seq_lens int32");
  TORCH_CHECK(work_seq.scalar_type() == at::kInt && work_mblk.scalar_type() == at::kInt &&
              work_seq.numel() == work_mblk.numel(), "work list");
  TORCH_CHECK(work_seq.numel() <= 2147483647 && nq <= 65535, "grid");
  TORCH_CHECK(cos_sin.size(0) >= 1 && cos_sin.size(0) < ((int64_t)1 << 31), "cos_sin rows");
  kgc::launch_prefill_attention(dt_code(out), qkv.data_ptr(), out.data_ptr(), k_cache.data_ptr(),
                                v_cache.data_ptr(), block_tables.data_ptr<int>(),
                                (int)block_tables.stride(0), query_start_loc.data_ptr<int>(),
                                seq_lens.data_ptr<int>(), work_seq.data_ptr<int>(),
                                work_mblk.data_ptr<int>(), (int)work_seq.numel(), (int)nq,
                                (int)nkv, (int)d, log2_exact(k_cache.size(2), "block_size"),
                                (float)scale, k_cache.scalar_type() == at::kFloat8_e4m3fn,
                                (float)k_scale, (float)v_scale, (int)k_cache.size(0),
                                qkv.stride(0), cos_sin.data_ptr<float>(), (int)cos_sin.size(0),
                                stream());
}

void sample(Tensor out, Tensor logits, Tensor temperature, Tensor top_k, Tensor top_p, Tensor seeds,
            bool thresholds) {
  check_gpu(logits, "logits");
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits [B, V] with dense rows");
  const int64_t B = logits.size(0);
  TORCH_CHECK(out.scalar_type() == at::kLong && out.numel() >= B, "out int64 [B]");
  TORCH_CHECK(temperature.scalar_type() == at::kFloat && temperature.numel() >= B, "temperature fp32");
  TORCH_CHECK(top_k.scalar_type() == at::kInt && top_k.numel() >= B, "top_k int32");
  TORCH_CHECK(top_p.scalar_type() == at::kFloat && top_p.numel() >= B, "top_p fp32");
  TORCH_CHECK(seeds.scalar_type() == at::kLong && seeds.numel() >= B, "seeds int64");
  TORCH_CHECK(B <= 65535 * 256 && logits.size(1) < INT32_MAX, "kgc.sample: shape");
  if (B == 0) return;
  if (thresholds && kgc::sample_coop_splits((int)B) > 0) {
    // rows with top-k / top-p: the cooperative kernel splits the threshold passes over
    // the row's workgroups (per-row workspace from the caching allocator)
    Tensor partial = at::empty({B * kgc::sample_coop_splits((int)B)}, logits.options().dtype(at::kLong));
    // one persistent zeroed workspace per device (256 rows); every call leaves it zeroed
    static std::vector<Tensor> wss(64);
    const int dev = logits.device().index();
    TORCH_CHECK(dev >= 0 && dev < 64, "device index");
    if (!wss[dev].defined())
      wss[dev] = at::zeros({256 * (int64_t)kgc::sample_coop_ws_bytes()},
                           logits.options().dtype(at::kByte));
    Tensor ws = wss[dev];
    kgc::launch_sample_coop(dt_code(logits), out.data_ptr<int64_t>(),
                            reinterpret_cast<uint64_t*>(partial.data_ptr<int64_t>()), ws.data_ptr(),
                            logits.data_ptr(), logits.stride(0), (int)B, (int)logits.size(1),
                            temperature.data_ptr<float>(), top_k.data_ptr<int>(),
                            top_p.data_ptr<float>(), seeds.data_ptr<int64_t>(), stream());
    return;
  }
  // per-(row, vocab split) candidates; from the caching allocator, so graph capture
  // gives the workspace a fixed address like any other captured temporary
  Tensor partial = at::empty({B * kgc::sample_splits((int)B)}, logits.options().dtype(at::kLong));
  kgc::launch_sample(dt_code(logits), out.data_ptr<int64_t>(),
                     reinterpret_cast<uint64_t*>(partial.data_ptr<int64_t>()), logits.data_ptr(),
                     logits.stride(0), (int)B, (int)logits.size(1), temperature.data_ptr<float>(),
                     top_k.data_ptr<int>(), top_p.data_ptr<float>(), seeds.data_ptr<int64_t>(),
                     stream());
}

void sample_vp(Tensor packed, Tensor logits, int64_t V, Tensor temperature, Tensor seeds,
               int64_t vocab_off) {
  check_gpu(logits, "logits");
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits [B, Vshard] with dense rows");
  const int64_t B = logits.size(0);
  TORCH_CHECK(V >= 1 && V <= logits.size(1), "V (valid shard columns) out of range");
  TORCH_CHECK(packed.scalar_type() == at::kLong && packed.numel() >= B, "packed int64 [B]");
  TORCH_CHECK(temperature.scalar_type() == at::kFloat && temperature.numel() >= B, "temperature fp32");
  TORCH_CHECK(seeds.scalar_type() == at::kLong && seeds.numel() >= B, "seeds int64");
  TORCH_CHECK(B <= 65535 * 256 && vocab_off >= 0 && vocab_off + V < INT32_MAX, "kgc.sample_vp: shape");
  if (B == 0) return;
  Tensor partial = at::empty({B * kgc::sample_splits((int)B)}, logits.options().dtype(at::kLong));
  kgc::launch_sample_vp(dt_code(logits), packed.data_ptr<int64_t>(),
                        reinterpret_cast<uint64_t*>(partial.data_ptr<int64_t>()), logits.data_ptr(),
                        logits.stride(0), (int)B, (int)V, temperature.data_ptr<float>(),
                        seeds.data_ptr<int64_t>(), (int)vocab_off, stream());
}

void sample_vp_unpack(Tensor out, Tensor packed) {
  check_gpu(packed, "packed");
  c10::hip::HIPGuardMasqueradingAsCUDA g(packed.device());
  TORCH_CHECK(packed.scalar_type() == at::kLong && out.scalar_type() == at::kLong &&
              out.numel() >= packed.numel() && packed.is_contiguous(), "int64 [B]");
  kgc::launch_sample_vp_unpack(out.data_ptr<int64_t>(), packed.data_ptr<int64_t>(),
                               (int)packed.numel(), stream());
}

// ---- K13/K14 MoE
void moe_route(Tensor topk_w, Tensor topk_ids, Tensor logits, bool renorm) {
  check_gpu(logits, "logits");
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "router logits [T, E] dense rows");
  const int64_t T = logits.size(0), E = logits.size(1), k = topk_w.size(-1);
  TORCH_CHECK(E >= 1 && E <= 64 && k >= 1 && k <= E, "1 <= k <= E <= 64");
  TORCH_CHECK(topk_w.scalar_type() == at::kFloat && topk_w.is_contiguous() && topk_w.numel() == T * k,
              "topk_w fp32 [T, k]");
  TORCH_CHECK(topk_ids.scalar_type() == at::kInt && topk_ids.is_contiguous() &&
              topk_ids.numel() == T * k, "topk_ids int32 [T, k]");
  if (T == 0) return;
  kgc::launch_moe_route(dt_code(logits), logits.data_ptr(), logits.stride(0), (int)T, (int)E,
                        (int)k, renorm, topk_w.data_ptr<float>(), topk_ids.data_ptr<int>(), stream());
}

void moe_gate_route(Tensor topk_w, Tensor topk_ids, Tensor x, Tensor wg, bool renorm) {
  check_gpu(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "x [T, H], 16-B aligned rows");
  TORCH_CHECK(wg.dim() == 2 && wg.is_contiguous() && wg.scalar_type() == x.scalar_type() &&
                  (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "wg [E, H] contiguous, x's dtype (bf16 / fp16)");
  const int64_t T = x.size(0), H = x.size(1), E = wg.size(0), k = topk_w.size(-1);
  TORCH_CHECK(wg.size(1) == H && H % 512 == 0, "H % 512 == 0");
  TORCH_CHECK(E >= 1 && E <= 16 && k >= 1 && k <= E, "1 <= k <= E <= 16");
  TORCH_CHECK(topk_w.scalar_type() == at::kFloat && topk_w.is_contiguous() && topk_w.numel() == T * k,
              "topk_w fp32 [T, k]");
  TORCH_CHECK(topk_ids.scalar_type() == at::kInt && topk_ids.is_contiguous() &&
              topk_ids.numel() == T * k, "topk_ids int32 [T, k]");
  check_same_dev(x, wg, "moe_gate_route");
  if (T == 0) return;
  kgc::launch_moe_gate_route(dt_code(x), x.data_ptr(), x.stride(0), wg.data_ptr(), (int)H, (int)E,
                             (int)T, (int)k, renorm, topk_w.data_ptr<float>(),
                             topk_ids.data_ptr<int>(), stream());
}

void moe_align(Tensor sorted_ids, Tensor block_expert, Tensor meta, Tensor topk_ids, int64_t e0,
               int64_t E_local, int64_t bm) {
  check_gpu(topk_ids, "topk_ids");
  c10::hip::HIPGuardMasqueradingAsCUDA g(topk_ids.device());
  TORCH_CHECK(bm == 64 || bm == 96 || bm == 128, "row block 64, 96 or 128");
  const int64_t npairs = topk_ids.numel();
  const int64_t rows = sorted_ids.numel();
  TORCH_CHECK(topk_ids.scalar_type() == at::kInt && topk_ids.is_contiguous(), "topk_ids int32");
  TORCH_CHECK(E_local >= 1 && E_local <= 256, "1 <= local experts <= 256");
  TORCH_CHECK(sorted_ids.scalar_type() == at::kInt && rows % bm == 0 &&
              rows >= npairs + E_local * (bm - 1), "sorted_ids int32, >= pairs + E*(BM-1) rows");
  TORCH_CHECK(block_expert.scalar_type() == at::kInt && block_expert.numel() >= rows / bm,
              "block_expert int32 [rows / BM]");
  TORCH_CHECK(meta.scalar_type() == at::kInt && meta.numel() >= 1, "meta int32");
  kgc::launch_moe_align(topk_ids.data_ptr<int>(), (int)npairs, (int)e0, (int)E_local, (int)bm,
                        (int)rows,
                        sorted_ids.data_ptr<int>(), block_expert.data_ptr<int>(),
                        meta.data_ptr<int>(), stream());
}

void moe_gemm(Tensor C, Tensor A, Tensor W, Tensor sorted_ids, Tensor block_expert, Tensor meta,
              int64_t npairs, int64_t topk, int64_t bm, bool gather, bool scatter, int64_t splitk) {
  check_gpu(A, "A");
  c10::hip::HIPGuardMasqueradingAsCUDA g(A.device());
  TORCH_CHECK(bm == 64 || bm == 128, "row block 64 or 128");
  TORCH_CHECK(W.dim() == 3 && W.is_contiguous(), "W [E, N, K] contiguous");
  TORCH_CHECK(splitk >= 1 && splitk <= 16, "1 <= splitk <= 16");
  TORCH_CHECK(splitk == 1 || (scatter && !gather), "split-K only for the scattering second GEMM");
  TORCH_CHECK(A.scalar_type() == W.scalar_type() &&
              C.scalar_type() == (splitk > 1 ? at::kFloat : W.scalar_type()),
              "A, W share a dtype; C too (fp32 split-K slices when splitk > 1)");
  TORCH_CHECK(W.scalar_type() == at::kBFloat16 || W.scalar_type() == at::kHalf, "bf16 / fp16");
  const int64_t N = W.size(1), K = W.size(2), rows = sorted_ids.numel();
  TORCH_CHECK(N % kgc::moe_block_n() == 0 && K % kgc::moe_block_k() == 0,
              "grouped GEMM needs N % 128 == 0 and K % 64 == 0");
  TORCH_CHECK(A.dim() == 2 && A.size(1) == K && A.stride(1) == 1 && A.stride(0) % 8 == 0, "A [*, K]");
  // split-K: C [S, rows, N] contiguous fp32 slices; else C [*, N]
  const Tensor C2 = splitk > 1 ? C.select(0, 0) : C;
  TORCH_CHECK(splitk == 1 || (C.dim() == 3 && C.size(0) == splitk && C.is_contiguous()),
              "split-K output: contiguous fp32 [splitk, rows, N]");
  TORCH_CHECK(C2.dim() == 2 && C2.size(1) == N && C2.stride(1) == 1 && C2.stride(0) % 8 == 0, "C [*, N]");
  TORCH_CHECK(rows % bm == 0 && block_expert.numel() >= rows / bm, "row blocks");
  // every row index the kernel can touch must exist
  if (gather) {
    TORCH_CHECK(A.size(0) * topk >= npairs, "A has fewer token rows than pairs / k");
  } else {
    TORCH_CHECK(A.size(0) >= rows, "A must hold every padded row");
  }
  if (scatter) {
    TORCH_CHECK(C2.size(0) >= npairs, "C must hold every pair row");
  } else {
    TORCH_CHECK(C2.size(0) >= rows, "C must hold every padded row");
  }
  if (rows == 0) return;
  kgc::launch_moe_gemm(dt_code(W), (int)bm, C.data_ptr(), A.data_ptr(), W.data_ptr(),
                       sorted_ids.data_ptr<int>(), block_expert.data_ptr<int>(), meta.data_ptr<int>(),
                       (int)npairs, (int)topk, (int)N, (int)K, A.stride(0), C2.stride(0),
                       (int)(rows / bm), gather, scatter, (int)splitk,
                       splitk > 1 ? C.stride(0) : 0, stream());
}

// K14m: the grouped MoE projections on the K9m LDS-DMA pipeline over per-expert packed
// weights Wp [E, N/128, K/64, 8192] (dgemm_pack per expert; w13 SiLU-packed).
// mode 1: C = act [rows, N/2] = silu(g) * u of x's gathered rows (sorted-row order);
// mode 2: C = [npairs, N] (W's dtype) or fp32 slices [S, npairs, N], rows scattered.
void moe_dgemm(Tensor C, Tensor A, Tensor Wp, Tensor sorted_ids, Tensor block_expert,
               Tensor meta, int64_t npairs, int64_t topk, int64_t bm, int64_t mode,
               int64_t bn) {
  check_gpu(A, "A");
  c10::hip::HIPGuardMasqueradingAsCUDA g(A.device());
  TORCH_CHECK(bm == 64 || bm == 96 || bm == 128, "row block 64, 96 or 128");
  TORCH_CHECK(mode == 1 || mode == 2, "mode 1 (gate_up + SiLU, gathered) or 2 (down, scattered)");
  TORCH_CHECK(bn == 128 || bn == 256, "column tile 128 or 256");
  TORCH_CHECK(Wp.dim() == 4 && Wp.is_contiguous() && Wp.size(3) == 128 * kgc::dgemm_block_k(),
              "Wp packed [E, N/128, K/64, 8192] contiguous");
  TORCH_CHECK(Wp.scalar_type() == at::kBFloat16 || Wp.scalar_type() == at::kHalf, "bf16 / fp16");
  TORCH_CHECK(A.scalar_type() == Wp.scalar_type(), "A in W's dtype");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(Wp.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0, "16-B aligned");
  const int64_t N = Wp.size(1) * 128, K = Wp.size(2) * kgc::dgemm_block_k();
  const int64_t rows = sorted_ids.numel();
  TORCH_CHECK(N % bn == 0, "N % bn == 0");
  TORCH_CHECK(A.dim() == 2 && A.size(1) == K && A.stride(1) == 1 && A.stride(0) % 8 == 0,
              "A [*, K], 16-B aligned rows");
  TORCH_CHECK(sorted_ids.scalar_type() == at::kInt && block_expert.scalar_type() == at::kInt &&
              meta.scalar_type() == at::kInt && rows % bm == 0 &&
              block_expert.numel() >= rows / bm && meta.numel() >= 1, "moe_align outputs");
  TORCH_CHECK(npairs >= 0 && topk >= 1 && npairs <= rows, "pairs");
  int64_t S = 1, ss = 0;
  if (mode == 1) {
    TORCH_CHECK(A.size(0) * topk >= npairs, "A has fewer token rows than pairs / k");
    TORCH_CHECK(C.scalar_type() == Wp.scalar_type() && C.dim() == 2 && C.is_contiguous() &&
                C.size(0) >= rows && C.size(1) == N / 2, "act [rows, N/2] contiguous");
  } else {
    TORCH_CHECK(A.size(0) >= rows, "A must hold every padded row");
    if (C.dim() == 3) {
      TORCH_CHECK(C.scalar_type() == at::kFloat && C.is_contiguous() && C.size(1) >= npairs &&
                  C.size(2) == N, "fp32 slices [S, >= npairs, N] contiguous");
      S = C.size(0);
      ss = C.stride(0);
      TORCH_CHECK(S >= 2 && S <= 16 && S <= K / kgc::dgemm_block_k(), "2 <= S <= 16");
    } else {
      TORCH_CHECK(C.scalar_type() == Wp.scalar_type() && C.dim() == 2 && C.is_contiguous() &&
                  C.size(0) >= npairs && C.size(1) == N, "C [>= npairs, N] contiguous");
    }
  }
  if (rows == 0) return;
  kgc::launch_moe_dgemm(dt_code(Wp), (int)mode, C.data_ptr(), A.data_ptr(), Wp.data_ptr(),
                        (int)rows, (int)N, (int)K, A.stride(0), (int)S, ss, (int)bm, (int)bn,
                        sorted_ids.data_ptr<int>(), block_expert.data_ptr<int>(),
                        meta.data_ptr<int>(), (int)npairs, (int)topk, stream());
}

void moe_combine(Tensor out, Tensor y, Tensor topk_w, const c10::optional<Tensor>& row_map) {
  check_gpu(y, "y");
  c10::hip::HIPGuardMasqueradingAsCUDA g(y.device());
  const int64_t T = out.size(0), H = out.size(1), k = topk_w.size(-1);
  TORCH_CHECK(out.is_contiguous() && y.is_contiguous() && H % 8 == 0, "contiguous, H % 8 == 0");
  TORCH_CHECK(topk_w.numel() == T * k && topk_w.scalar_type() == at::kFloat, "topk_w fp32 [T, k]");
  TORCH_CHECK(T <= 65535, "at most 65535 tokens per call");
  const int* map = nullptr;
  int64_t nrows = T * k;
  if (row_map.has_value()) {
    // y: [rows, H] in out's dtype, pair p read from row row_map[p] (-1 = no row); the
    // kernel skips indices outside [0, rows)
    const Tensor& rm = *row_map;
    TORCH_CHECK(y.dim() == 2 && y.size(1) == H && y.scalar_type() == out.scalar_type(),
                "y [rows, H] in out's dtype");
    TORCH_CHECK(rm.scalar_type() == at::kInt && rm.is_contiguous() && rm.numel() == T * k &&
                    rm.device() == y.device(),
                "row_map int32 [T*k] on y's device");
    map = rm.data_ptr<int>();
    nrows = y.size(0);
  }
  // y: [T*k, H] in out's dtype, or fp32 split-K slices [S, rows >= T*k, H]
  const bool slices = y.dim() == 3;
  if (!map)
    TORCH_CHECK(slices ? (y.scalar_type() == at::kFloat && y.size(2) == H && y.size(1) >= T * k)
                       : (y.scalar_type() == out.scalar_type() && y.numel() >= T * k * H),
                "y [T*k, H] or fp32 [S, >= T*k, H]");
  if (T == 0) return;
  kgc::launch_moe_combine(dt_code(out), out.data_ptr(), y.data_ptr(), topk_w.data_ptr<float>(),
                          map, nrows, (int)T, (int)k, (int)H, slices ? (int)y.size(0) : 1,
                          slices ? y.stride(0) : 0, stream());
}

// Dense split-K decode GEMM on the grouped-GEMM tiles (XCD-mapped K-slices) + its reduction.
void dense_gemm_splitk(Tensor Cs, Tensor A, Tensor W, int64_t bm) {
  check_gpu(A, "A");
  c10::hip::HIPGuardMasqueradingAsCUDA g(A.device());
  TORCH_CHECK(bm == 64 || bm == 128, "row block 64 or 128");
  TORCH_CHECK(W.dim() == 2 && W.is_contiguous(), "W [N, K] contiguous");
  TORCH_CHECK(W.scalar_type() == at::kBFloat16 || W.scalar_type() == at::kHalf, "bf16 / fp16");
  const int64_t N = W.size(0), K = W.size(1);
  TORCH_CHECK(A.scalar_type() == W.scalar_type() && A.dim() == 2 && A.size(1) == K &&
              A.stride(1) == 1 && A.stride(0) % 8 == 0, "A [M, K] in W's dtype");
  const int64_t M = A.size(0);
  TORCH_CHECK(N % kgc::moe_block_n() == 0 && K % kgc::moe_block_k() == 0, "N % 128, K % 64");
  TORCH_CHECK(Cs.scalar_type() == at::kFloat && Cs.dim() == 3 && Cs.is_contiguous() &&
              Cs.size(1) == M && Cs.size(2) == N, "Cs fp32 contiguous [S, M, N]");
  const int64_t S = Cs.size(0);
  TORCH_CHECK(S >= 1 && S <= 16 && K / kgc::moe_block_k() >= S, "1 <= S <= 16, S <= K / 64");
  if (M == 0) return;
  kgc::launch_dense_gemm_splitk(dt_code(W), (int)bm, Cs.data_ptr<float>(), A.data_ptr(),
                                W.data_ptr(), (int)M, (int)N, (int)K, A.stride(0), (int)S,
                                stream());
}

// K9m mid-batch decode GEMM (LDS-DMA ring, XCD-mapped split-K, fused epilogues).
// W: [N, K] for the row-major configs, [N/128, K/64, 8192] (dgemm_pack) for packed ones.
static void dgemm_shape(const Tensor& W, bool packed, int64_t* N, int64_t* K) {
  if (packed) {
    TORCH_CHECK(W.dim() == 3 && W.is_contiguous() && W.size(2) == 128 * kgc::dgemm_block_k(),
                "packed W [N/128, K/64, 8192] contiguous");
    *N = W.size(0) * 128;
    *K = W.size(1) * kgc::dgemm_block_k();
  } else {
    TORCH_CHECK(W.dim() == 2 && W.is_contiguous(), "W [N, K] contiguous");
    *N = W.size(0);
    *K = W.size(1);
  }
}

void dgemm(Tensor C, Tensor X, Tensor W, int64_t cfg, int64_t epi,
           std::optional<Tensor> rscale) {
  check_gpu(X, "X");
  c10::hip::HIPGuardMasqueradingAsCUDA g(X.device());
  TORCH_CHECK(cfg >= 0 && cfg < kgc::dgemm_num_cfgs(), "unknown dgemm tile config");
  int bm, bn, packed;
  kgc::dgemm_cfg_info((int)cfg, &bm, &bn, &packed);
  TORCH_CHECK(epi >= 0 && epi <= 2, "epi 0 (fp32 slices), 1 (out), 2 (silu pairs)");
  TORCH_CHECK((kgc::dgemm_cfg_epis((int)cfg) >> epi) & 1,
              "dgemm: this tile config has no such epilogue (dgemm_cfg_epis)");
  TORCH_CHECK(W.scalar_type() == at::kBFloat16 || W.scalar_type() == at::kHalf, "bf16 / fp16");
  int64_t N, K;
  dgemm_shape(W, packed, &N, &K);
  const int64_t bk = kgc::dgemm_block_k();
  TORCH_CHECK(X.scalar_type() == W.scalar_type() && X.dim() == 2 && X.size(1) == K &&
              X.stride(1) == 1 && X.stride(0) % 8 == 0 &&
              reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0, "X [M, K] in W's dtype, "
              "16-B aligned rows");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(W.data_ptr()) % 16 == 0, "W 16-B aligned");
  const int64_t M = X.size(0);
  TORCH_CHECK(N % bn == 0 && K % bk == 0 && K >= bk, "N % BN == 0, K % 64 == 0");
  TORCH_CHECK(M <= (int64_t)1 << 20 && N < ((int64_t)1 << 31) / 4, "size limits");
  int64_t S = 1, ss = 0;
  if (epi == 0) {
    TORCH_CHECK(C.scalar_type() == at::kFloat && C.dim() == 3 && C.is_contiguous() &&
                C.size(1) == M && C.size(2) == N, "C fp32 contiguous [S, M, N]");
    S = C.size(0);
    ss = C.stride(0);
    TORCH_CHECK(S >= 1 && S <= 32 && S <= K / bk, "1 <= S <= min(32, K / 64)");
  } else {
    TORCH_CHECK(C.scalar_type() == W.scalar_type() && C.dim() == 2 && C.is_contiguous() &&
                C.size(0) == M && C.size(1) == (epi == 2 ? N / 2 : N),
                "C [M, N] (epi 1) or [M, N/2] (epi 2), contiguous, W's dtype");
  }
  TORCH_CHECK((M + bm - 1) / bm * (N / bn) * S < ((int64_t)1 << 31), "grid too large");
  kgc::DgAux aux{};
  if (rscale.has_value()) {
    TORCH_CHECK(epi != 0 && kgc::dgemm_cfg_has_aux((int)cfg),
                "rscale: epilogues 1 / 2 of a config with the row-scale epilogue");
    TORCH_CHECK(rscale->scalar_type() == at::kFloat && rscale->is_contiguous() &&
                rscale->numel() >= M, "rscale fp32 [>= M] contiguous");
    check_same_dev(X, *rscale, "dgemm rscale");
    aux.rsc = rscale->data_ptr<float>();
  }
  if (M == 0) return;
  kgc::launch_dgemm(dt_code(W), (int)cfg, (int)epi, C.data_ptr(), X.data_ptr(), W.data_ptr(),
                    (int)M, (int)N, (int)K, X.stride(0), (int)S, ss, aux, stream());
}


// P [N/128, K/64, 8192] <- W [N, K] re-laid out for the packed K9m configs
void dgemm_pack(Tensor P, Tensor W, bool silu) {
  check_gpu(W, "W");
  c10::hip::HIPGuardMasqueradingAsCUDA g(W.device());
  TORCH_CHECK(W.dim() == 2 && W.is_contiguous(), "W [N, K] contiguous");
  TORCH_CHECK(W.scalar_type() == at::kBFloat16 || W.scalar_type() == at::kHalf, "bf16 / fp16");
  const int64_t N = W.size(0), K = W.size(1), bk = kgc::dgemm_block_k();
  TORCH_CHECK(N % 128 == 0 && K % bk == 0 && (!silu || (N / 2) % 64 == 0), "N % 128, K % 64");
  TORCH_CHECK(P.scalar_type() == W.scalar_type() && P.dim() == 3 && P.is_contiguous() &&
              P.size(0) == N / 128 && P.size(1) == K / bk && P.size(2) == 128 * bk,
              "P [N/128, K/64, 8192] contiguous, W's dtype");
  TORCH_CHECK(P.device() == W.device(), "same device");
  kgc::launch_dgemm_pack(dt_code(W), silu, P.data_ptr(), W.data_ptr(), (int)N, (int)K,
                         stream());
}

std::vector<int64_t> dgemm_cfg_info(int64_t cfg) {
  TORCH_CHECK(cfg >= 0 && cfg < kgc::dgemm_num_cfgs(), "unknown dgemm tile config");
  int bm, bn, packed;
  kgc::dgemm_cfg_info((int)cfg, &bm, &bn, &packed);
  return {bm, bn, packed};
}
int64_t dgemm_num_cfgs() { return kgc::dgemm_num_cfgs(); }
int64_t dgemm_cfg_epis(int64_t cfg) {
  TORCH_CHECK(cfg >= 0 && cfg < kgc::dgemm_num_cfgs(), "unknown dgemm tile config");
  return kgc::dgemm_cfg_epis((int)cfg);
}
bool dgemm_cfg_has_aux(int64_t cfg) {
  TORCH_CHECK(cfg >= 0 && cfg < kgc::dgemm_num_cfgs(), "unknown dgemm tile config");
  return kgc::dgemm_cfg_has_aux((int)cfg);
}

// profiling only: the packed 256 x 128 tile with its MFMAs / DMAs / one operand's DMAs removed
void dgemm_ablate(Tensor C, Tensor X, Tensor W, int64_t mode) {
  check_gpu(X, "X");
  c10::hip::HIPGuardMasqueradingAsCUDA g(X.device());
  TORCH_CHECK(W.scalar_type() == at::kBFloat16 && X.scalar_type() == at::kBFloat16, "bf16");
  int64_t N, K;
  dgemm_shape(W, true, &N, &K);
  const int64_t M = X.size(0);
  TORCH_CHECK(X.dim() == 2 && X.is_contiguous() && X.size(1) == K, "X [M, K] contiguous");
  TORCH_CHECK(C.scalar_type() == at::kFloat && C.dim() == 3 && C.is_contiguous() &&
              C.size(1) == M && C.size(2) == N && C.size(0) <= K / 64, "C fp32 [S, M, N]");
  kgc::launch_dgemm_ablate((int)mode, C.data_ptr<float>(), X.data_ptr(), W.data_ptr(), (int)M,
                           (int)N, (int)K, X.stride(0), (int)C.size(0), C.stride(0), stream());
}

void splitk_reduce(Tensor out, Tensor Cs) {
  check_gpu(Cs, "Cs");
  c10::hip::HIPGuardMasqueradingAsCUDA g(Cs.device());
  TORCH_CHECK(Cs.scalar_type() == at::kFloat && Cs.dim() == 3 && Cs.is_contiguous(), "Cs fp32 [S, M, N]");
  TORCH_CHECK(out.is_contiguous() && out.numel() == Cs.size(1) * Cs.size(2) && out.numel() % 8 == 0,
              "out [M, N] contiguous, numel % 8 == 0");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kHalf, "bf16 / fp16");
  if (out.numel() == 0) return;
  kgc::launch_splitk_reduce(dt_code(out), out.data_ptr(), Cs.data_ptr<float>(), (int)Cs.size(0),
                            out.numel(), Cs.stride(0), stream());
}

void splitk_reduce_silu(Tensor out, Tensor Cs, bool interleaved, std::optional<Tensor> rscale) {
  check_gpu(Cs, "Cs");
  c10::hip::HIPGuardMasqueradingAsCUDA g(Cs.device());
  TORCH_CHECK(Cs.scalar_type() == at::kFloat && Cs.dim() == 3 && Cs.is_contiguous(), "Cs fp32 [S, M, 2I]");
  const int64_t M = Cs.size(1), I = Cs.size(2) / 2;
  TORCH_CHECK(Cs.size(2) % 16 == 0, "2I % 16 == 0");
  TORCH_CHECK(out.dim() == 2 && out.is_contiguous() && out.size(0) == M && out.size(1) == I,
              "out [M, I] contiguous");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kHalf, "bf16 / fp16");
  if (M == 0) return;
  TORCH_CHECK(!interleaved || I % 64 == 0, "interleaved (packed SiLU tiles): I % 64 == 0");
  const float* rsc = nullptr;
  if (rscale.has_value()) {
    TORCH_CHECK(rscale->scalar_type() == at::kFloat && rscale->is_contiguous() &&
                rscale->numel() >= M, "rscale fp32 [>= M] contiguous");
    check_same_dev(Cs, *rscale, "splitk_reduce_silu rscale");
    rsc = rscale->data_ptr<float>();
  }
  kgc::launch_splitk_reduce_silu(dt_code(out), out.data_ptr(), Cs.data_ptr<float>(), (int)Cs.size(0),
                                 (int)M, (int)I, Cs.stride(0), interleaved, rsc, stream());
}

void splitk_add_rms_norm(Tensor out, Tensor Cs, Tensor residual, Tensor w, double eps) {
  check_gpu(Cs, "Cs");
  c10::hip::HIPGuardMasqueradingAsCUDA g(Cs.device());
  TORCH_CHECK(Cs.scalar_type() == at::kFloat && Cs.dim() == 3 && Cs.is_contiguous(), "Cs fp32 [S, M, H]");
  const int64_t M = Cs.size(1), H = Cs.size(2);
  TORCH_CHECK(H % 8 == 0 && H <= 8192, "H % 8 == 0, H <= 8192");
  for (const Tensor* t : {&out, &residual})
    TORCH_CHECK(t->dim() == 2 && t->is_contiguous() && t->size(0) == M && t->size(1) == H &&
                t->scalar_type() == out.scalar_type(), "out / residual [M, H] contiguous");
  TORCH_CHECK(w.is_contiguous() && w.numel() == H && w.scalar_type() == out.scalar_type(), "w [H]");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kHalf, "bf16 / fp16");
  if (M == 0) return;
  kgc::launch_splitk_add_rms_norm(dt_code(out), out.data_ptr(), Cs.data_ptr<float>(),
                                  residual.data_ptr(), w.data_ptr(), (int)M, (int)H,
                                  (int)Cs.size(0), Cs.stride(0), (float)eps, stream());
}

// ---- K12 xGMI all-reduce: IPC buffers are raw device pointers carried as int64
int64_t ar_signal_bytes() { return (int64_t)kgc::allreduce_signal_bytes(); }
int64_t ar_alloc(int64_t bytes) { return (int64_t)(intptr_t)kgc::ar_alloc(bytes); }
void ar_free(int64_t p) { kgc::ar_free((void*)(intptr_t)p); }
Tensor ar_get_handle(int64_t p) {
  Tensor h = at::zeros({64}, at::TensorOptions().dtype(at::kByte));
  kgc::ar_get_handle((void*)(intptr_t)p, h.data_ptr<uint8_t>());
  return h;
}
int64_t ar_open_handle(Tensor h) {
  TORCH_CHECK(h.device().is_cpu() && h.scalar_type() == at::kByte && h.numel() == 64,
              "IPC handle: uint8[64] CPU tensor");
  return (int64_t)(intptr_t)kgc::ar_open_handle(h.contiguous().data_ptr<uint8_t>());
}
void ar_close_handle(int64_t p) { kgc::ar_close_handle((void*)(intptr_t)p); }
int64_t ar_read_err(int64_t sig) { return (int64_t)kgc::ar_read_err((void*)(intptr_t)sig); }
// phantom TP rank: raise the never-running peers' arrival flags in this rank's signal
void ep_raise_peer_flags_op(int64_t sig, int64_t rank, int64_t nranks, int64_t value) {
  TORCH_CHECK(sig != 0 && rank >= 0 && rank < nranks &&
                  (nranks == 2 || nranks == 4 || nranks == 8) && value > 0 &&
                  value < ((int64_t)1 << 31),
              "ep_raise_peer_flags: sig, 0 <= rank < nranks in {2, 4, 8}, 0 < value < 2^31");
  kgc::ep_raise_peer_flags((void*)(intptr_t)sig, (int)rank, (int)nranks, (uint32_t)value,
                           stream());
}

void ar_raise_peer_flags(int64_t sig, int64_t rank, int64_t nranks, int64_t value) {
  TORCH_CHECK(sig != 0 && rank >= 0 && rank < nranks && (nranks == 2 || nranks == 4 ||
              nranks == 8) && value > 0 && value < (int64_t(1) << 31),
              "ar_raise_peer_flags: sig, 0 <= rank < nranks in {2, 4, 8}, 0 < value < 2^31");
  kgc::ar_raise_peer_flags((void*)(intptr_t)sig, (int)rank, (int)nranks, (uint32_t)value,
                           stream());
}
// host_out: pinned int32 [1]; valid once the current stream has passed this point
void ar_err_copy_async(int64_t sig, Tensor host_out) {
  TORCH_CHECK(host_out.device().is_cpu() && host_out.is_pinned() &&
              host_out.scalar_type() == at::kInt && host_out.numel() >= 1,
              "host_out: pinned int32 [1]");
  kgc::ar_err_copy_async((void*)(intptr_t)sig, reinterpret_cast<uint32_t*>(host_out.data_ptr()),
                         stream());
}

void xgmi_allreduce(Tensor inout, std::vector<int64_t> data, std::vector<int64_t> sig, int64_t rank,
                    int64_t cap_bytes, bool two_shot, bool wide) {
  check_gpu(inout, "inout");
  c10::hip::HIPGuardMasqueradingAsCUDA g(inout.device());
  const int64_t nr = (int64_t)data.size();
  TORCH_CHECK(nr == 2 || nr == 4 || nr == 8, "xgmi all-reduce: 2, 4 or 8 ranks");
  TORCH_CHECK((int64_t)sig.size() == nr && rank >= 0 && rank < nr, "bad rank / pointer lists");
  TORCH_CHECK(inout.is_contiguous(), "inout must be contiguous");
  TORCH_CHECK(inout.scalar_type() == at::kBFloat16 || inout.scalar_type() == at::kHalf,
              "bf16 / fp16 only");
  const int64_t bytes = inout.numel() * inout.element_size();
  TORCH_CHECK(bytes % (16 * nr) == 0, "message must be a multiple of 16 B x ranks");
  TORCH_CHECK(bytes <= cap_bytes, "message larger than the IPC buffer");
  kgc::ArPtrs P{};
  for (int64_t r = 0; r < nr; ++r) {
    P.data[r] = (void*)(intptr_t)data[r];
    P.sig[r] = (void*)(intptr_t)sig[r];
  }
  TORCH_CHECK(!wide || two_shot, "the wide grid is a two-shot form");
  kgc::launch_allreduce(dt_code(inout), P, (int)nr, (int)rank, inout.data_ptr(), bytes / 16,
                        cap_bytes / 16, two_shot, wide, stream());
}

// ---- C7 expert-parallel all-to-all over IPC peer memory
static kgc::EpPtrs ep_ptrs(const std::vector<int64_t>& data, const std::vector<int64_t>& sig,
                           int64_t rank) {
  const int64_t nr = (int64_t)data.size();
  TORCH_CHECK(nr == 2 || nr == 4 || nr == 8, "EP all-to-all: 2, 4 or 8 ranks");
  TORCH_CHECK((int64_t)sig.size() == nr && rank >= 0 && rank < nr, "bad rank / pointer lists");
  kgc::EpPtrs P{};
  for (int64_t r = 0; r < nr; ++r) {
    P.data[r] = (void*)(intptr_t)data[r];
    P.sig[r] = (void*)(intptr_t)sig[r];
  }
  return P;
}

static void ep_check_rows(const Tensor& t, const char* what) {
  check_gpu(t, what);
  TORCH_CHECK(t.dim() == 2 && t.is_contiguous() && t.size(1) % 8 == 0 &&
              (t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf),
              what, ": contiguous bf16/fp16 [rows, H], H % 8 == 0");
}

int64_t ep_signal_bytes_op() { return (int64_t)kgc::ep_signal_bytes(); }
int64_t ep_region_bytes_op(int64_t nr, int64_t C, int64_t H, int64_t esz) {
  return kgc::ep_region_bytes((int)nr, (int)C, (int)H, (int)esz);
}
int64_t ep_max_pairs_op() { return kgc::ep_max_pairs(); }

void ep_dispatch(Tensor x, Tensor topk_ids, std::vector<int64_t> data, std::vector<int64_t> sig,
                 int64_t rank, int64_t E_local, int64_t C) {
  ep_check_rows(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(topk_ids.scalar_type() == at::kInt && topk_ids.dim() == 2 && topk_ids.is_contiguous() &&
              topk_ids.size(0) == x.size(0), "topk_ids int32 [T, k]");
  const int64_t npairs = topk_ids.numel();
  TORCH_CHECK(npairs <= C && npairs <= kgc::ep_max_pairs(), "more (token, expert) pairs than the EP buffers hold");
  kgc::launch_ep_dispatch(dt_code(x), ep_ptrs(data, sig, rank), (int)data.size(), (int)rank,
                          x.data_ptr(), topk_ids.data_ptr<int>(), (int)npairs,
                          (int)topk_ids.size(1), (int)x.size(1), (int)E_local, (int)C, stream());
}

void ep_receive(Tensor x_local, Tensor ids, Tensor route, std::vector<int64_t> data,
                std::vector<int64_t> sig, int64_t rank, int64_t E_local, int64_t C) {
  ep_check_rows(x_local, "x_local");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x_local.device());
  const int64_t slots = (int64_t)data.size() * C;
  TORCH_CHECK(x_local.size(0) == slots && ids.numel() == slots && route.numel() == slots &&
              ids.scalar_type() == at::kInt && route.scalar_type() == at::kInt,
              "x_local [NR * C, H], ids / route int32 [NR * C]");
  kgc::launch_ep_receive(dt_code(x_local), ep_ptrs(data, sig, rank), (int)data.size(), (int)rank,
                         x_local.data_ptr(), ids.data_ptr<int>(), route.data_ptr<int>(),
                         (int)x_local.size(1), (int)E_local, (int)C, stream());
}

void ep_return(Tensor y, Tensor route, std::vector<int64_t> data, std::vector<int64_t> sig,
               int64_t rank, int64_t C, c10::optional<at::ScalarType> out_dtype) {
  // y: [NR * C, H] bf16 / fp16, or the down projection's fp32 split-K slices
  // [S, >= NR * C, H] (summed by the kernel, written in out_dtype)
  check_gpu(y, "y");
  c10::hip::HIPGuardMasqueradingAsCUDA g(y.device());
  const int64_t rows = (int64_t)data.size() * C;
  TORCH_CHECK(route.numel() == rows && route.scalar_type() == at::kInt && route.is_contiguous(),
              "route int32 [NR * C]");
  if (y.dim() == 3) {
    TORCH_CHECK(y.scalar_type() == at::kFloat && y.is_contiguous() && y.size(1) >= rows &&
                    y.size(2) % 8 == 0 && out_dtype.has_value() &&
                    (*out_dtype == at::kBFloat16 || *out_dtype == at::kHalf),
                "fp32 slices [S, >= NR * C, H] need out_dtype bf16 / fp16");
    kgc::launch_ep_return(*out_dtype == at::kBFloat16 ? kgc::DT_BF16 : kgc::DT_F16,
                          ep_ptrs(data, sig, rank), (int)data.size(), (int)rank, y.data_ptr(),
                          (int)y.size(0), y.stride(0), route.data_ptr<int>(), (int)y.size(2),
                          (int)C, stream());
    return;
  }
  ep_check_rows(y, "y");
  TORCH_CHECK(y.size(0) == rows && (!out_dtype.has_value() || *out_dtype == y.scalar_type()),
              "y [NR * C, H]");
  kgc::launch_ep_return(dt_code(y), ep_ptrs(data, sig, rank), (int)data.size(), (int)rank,
                        y.data_ptr(), 0, 0, route.data_ptr<int>(), (int)y.size(1), (int)C,
                        stream());
}

void ep_combine(Tensor out, Tensor topk_w, std::vector<int64_t> data, std::vector<int64_t> sig,
                int64_t rank, int64_t C) {
  ep_check_rows(out, "out");
  c10::hip::HIPGuardMasqueradingAsCUDA g(out.device());
  TORCH_CHECK(topk_w.scalar_type() == at::kFloat && topk_w.dim() == 2 && topk_w.is_contiguous() &&
              topk_w.size(0) == out.size(0) && topk_w.numel() <= C, "topk_w fp32 [T, k]");
  kgc::launch_ep_combine(dt_code(out), ep_ptrs(data, sig, rank), (int)data.size(), (int)rank,
                         out.data_ptr(), topk_w.data_ptr<float>(), (int)out.size(0),
                         (int)topk_w.size(1), (int)out.size(1), (int)C, stream());
}

int64_t ep_read_err_op(int64_t sig) { return kgc::ep_read_err((void*)(intptr_t)sig); }

void ep_err_copy_async(int64_t sig, Tensor host_out) {
  TORCH_CHECK(host_out.device().is_cpu() && host_out.is_pinned() &&
              host_out.scalar_type() == at::kInt && host_out.numel() >= 1,
              "host_out: pinned int32 [1]");
  kgc::ep_err_copy_async((void*)(intptr_t)sig, reinterpret_cast<uint32_t*>(host_out.data_ptr()),
                         stream());
}

// ---- C5 pipeline-stage handoff over IPC peer memory
int64_t pp_signal_bytes_op() { return (int64_t)kgc::pp_signal_bytes(); }
int64_t pp_read_err_op(int64_t sig) { return kgc::pp_read_err((void*)(intptr_t)sig); }

static void pp_check_pair(const Tensor& h, const Tensor& r) {
  check_gpu(h, "h");
  check_same_dev(h, r, "r");
  TORCH_CHECK(h.is_contiguous() && r.is_contiguous() && h.sizes() == r.sizes() &&
              h.scalar_type() == r.scalar_type() && (h.numel() * h.element_size()) % 16 == 0,
              "hidden / residual: contiguous, same shape and dtype, 16-byte multiple");
}

void pp_send(Tensor h, Tensor r, int64_t peer_data, int64_t peer_sig, int64_t own_sig,
             int64_t slot_bytes, int64_t R) {
  pp_check_pair(h, r);
  c10::hip::HIPGuardMasqueradingAsCUDA g(h.device());
  const int64_t bytes = h.numel() * h.element_size();
  TORCH_CHECK(bytes <= slot_bytes && R >= 1, "rows larger than a handoff slot");
  kgc::launch_pp_send((void*)(intptr_t)peer_data, (void*)(intptr_t)peer_sig,
                      (void*)(intptr_t)own_sig, h.data_ptr(), r.data_ptr(), bytes, slot_bytes,
                      (int)R, stream());
}

void pp_recv(Tensor h, Tensor r, int64_t own_data, int64_t own_sig, int64_t peer_sig,
             int64_t slot_bytes, int64_t R) {
  pp_check_pair(h, r);
  c10::hip::HIPGuardMasqueradingAsCUDA g(h.device());
  const int64_t bytes = h.numel() * h.element_size();
  TORCH_CHECK(bytes <= slot_bytes && R >= 1, "rows larger than a handoff slot");
  kgc::launch_pp_recv((void*)(intptr_t)own_data, (void*)(intptr_t)own_sig,
                      (void*)(intptr_t)peer_sig, h.data_ptr(), r.data_ptr(), bytes, slot_bytes,
                      (int)R, stream());
}

// one device word (e.g. a peer-memory collective's sticky error) -> pinned host int32,
// stream-ordered behind the step that may set it
void u32_copy_async(int64_t addr, Tensor host_out, int64_t index) {
  TORCH_CHECK(host_out.device().is_cpu() && host_out.is_pinned() &&
              host_out.scalar_type() == at::kInt && index >= 0 && index < host_out.numel(),
              "host_out: pinned int32, index in range");
  TORCH_CHECK(hipMemcpyAsync(reinterpret_cast<int*>(host_out.data_ptr()) + index,
                             (const void*)(intptr_t)addr, 4, hipMemcpyDeviceToHost,
                             stream()) == hipSuccess, "u32_copy_async");
}

// the cooperative sampler's sticky barrier-timeout word: its device address (current device)
int64_t sample_err_addr() { return (int64_t)(intptr_t)kgc::sample_err_addr(); }

// set one device word, stream-ordered (fault-injection tests of the sticky error words)
void u32_fill_async(int64_t addr, int64_t value) {
  TORCH_CHECK(hipMemsetD32Async((hipDeviceptr_t)(intptr_t)addr, (int)value, 1, stream()) ==
              hipSuccess, "u32_fill_async");
}

// zero one device word, stream-ordered (after its value was copied out)
void u32_clear_async(int64_t addr) {
  TORCH_CHECK(hipMemsetAsync((void*)(intptr_t)addr, 0, 4, stream()) == hipSuccess,
              "u32_clear_async");
}

// debug builds: OR of the K1/K2/K3 bounds-check error words (read and cleared)
int64_t debug_errors() {
  return (int64_t)(kgc::dbg_err_attention_decode() | (kgc::dbg_err_attention_prefill() << 1) |
                   (kgc::dbg_err_rope_cache() << 2));
}

bool debug_build() {
#ifdef KGC_DEBUG
  return true;
#else
  return false;
#endif
}

int64_t allreduce_rms_max_hidden_op() { return kgc::allreduce_rms_max_hidden(); }
int64_t allreduce_max_blocks_op() { return kgc::allreduce_max_blocks(); }
int64_t peer_spin_ms_op() { return kgc::peer_spin_ms(); }
int64_t coop_spin_ms_op() { return kgc::coop_spin_ms(); }
int64_t wall_clock_rate_khz_op() { return kgc::wall_clock_rate_khz(); }

void xgmi_allreduce_rms(Tensor out, Tensor in, Tensor residual, Tensor w, double eps,
                        std::vector<int64_t> data, std::vector<int64_t> sig, int64_t rank,
                        int64_t cap_bytes, bool two_shot) {
  check_gpu(in, "in");
  check_same_dev(in, out, "out");
  check_same_dev(in, residual, "residual");
  check_same_dev(in, w, "w");
  c10::hip::HIPGuardMasqueradingAsCUDA g(in.device());
  const int64_t nr = (int64_t)data.size();
  TORCH_CHECK(nr == 2 || nr == 4 || nr == 8, "xgmi all-reduce: 2, 4 or 8 ranks");
  TORCH_CHECK((int64_t)sig.size() == nr && rank >= 0 && rank < nr, "bad rank / pointer lists");
  TORCH_CHECK(in.dim() == 2 && in.is_contiguous() && out.is_contiguous() &&
              residual.is_contiguous() && w.is_contiguous(), "contiguous [M, H] rows");
  TORCH_CHECK(out.sizes() == in.sizes() && residual.sizes() == in.sizes() &&
              w.numel() == in.size(1), "out / residual [M, H], w [H]");
  TORCH_CHECK(in.scalar_type() == out.scalar_type() && in.scalar_type() == residual.scalar_type() &&
              in.scalar_type() == w.scalar_type() &&
              (in.scalar_type() == at::kBFloat16 || in.scalar_type() == at::kHalf), "bf16 / fp16 only");
  const int64_t M = in.size(0), H = in.size(1);
  TORCH_CHECK(H % 8 == 0 && H <= kgc::allreduce_rms_max_hidden(), "hidden size unsupported");
  TORCH_CHECK(M * H * in.element_size() <= cap_bytes, "rows larger than the IPC buffer");
  kgc::ArPtrs P{};
  for (int64_t r = 0; r < nr; ++r) {
    P.data[r] = (void*)(intptr_t)data[r];
    P.sig[r] = (void*)(intptr_t)sig[r];
  }
  kgc::launch_allreduce_rms(dt_code(in), P, (int)nr, (int)rank, in.data_ptr(), out.data_ptr(),
                            residual.data_ptr(), w.data_ptr(), (int)M, (int)H, (float)eps,
                            cap_bytes / 16, two_shot, stream());
}

// World emulation of the xGMI all-reduce kernels (tests): every rank's blocks in one launch
// on this device.  data / sig: each rank's region for `kind` and its signal block (plain
// device memory is enough: one device); a / b / c: per-rank operands (see launch.h).
void xgmi_allreduce_emu(int64_t kind, std::vector<Tensor> a, std::vector<Tensor> b,
                        std::vector<Tensor> c, std::optional<Tensor> w, std::vector<int64_t> data,
                        std::vector<int64_t> sig, int64_t cap_bytes, double eps) {
  const int64_t nr = (int64_t)data.size();
  TORCH_CHECK(nr == 2 || nr == 4 || nr == 8, "emulation: 2, 4 or 8 ranks");
  TORCH_CHECK((int64_t)sig.size() == nr && (int64_t)a.size() == nr, "one buffer per rank");
  TORCH_CHECK(kind >= 0 && kind <= 4, "kind 0..4");
  const Tensor& x0 = a[0];
  check_gpu(x0, "a[0]");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x0.device());
  TORCH_CHECK(x0.scalar_type() == at::kBFloat16 || x0.scalar_type() == at::kHalf, "bf16 / fp16");
  const int64_t bytes = x0.numel() * x0.element_size();
  TORCH_CHECK(bytes <= cap_bytes && bytes % (16 * nr) == 0, "message size");
  kgc::ArPtrs P{};
  kgc::ArWorld W{};
  int M = 0, H = 0;
  const void* wp = nullptr;
  if (kind == 2 || kind == 3) {
    TORCH_CHECK(x0.dim() == 2 && (int64_t)b.size() == nr && (int64_t)c.size() == nr &&
                w.has_value(), "fused: a (in), b (out), c (residual) [M, H] per rank, w [H]");
    M = (int)x0.size(0);
    H = (int)x0.size(1);
    TORCH_CHECK(H % 8 == 0 && H <= kgc::allreduce_rms_max_hidden() && w->numel() == H &&
                w->scalar_type() == x0.scalar_type() && w->is_contiguous(), "hidden / w");
    wp = w->data_ptr();
  }
  for (int64_t r = 0; r < nr; ++r) {
    P.data[r] = (void*)(intptr_t)data[r];
    P.sig[r] = (void*)(intptr_t)sig[r];
    TORCH_CHECK(a[r].is_contiguous() && a[r].sizes() == x0.sizes() &&
                a[r].scalar_type() == x0.scalar_type() && a[r].device() == x0.device(), "a[r]");
    W.a[r] = a[r].data_ptr();
    if (kind == 2 || kind == 3) {
      TORCH_CHECK(b[r].is_contiguous() && b[r].sizes() == x0.sizes() &&
                  c[r].is_contiguous() && c[r].sizes() == x0.sizes() &&
                  b[r].scalar_type() == x0.scalar_type() && c[r].scalar_type() == x0.scalar_type(),
                  "b[r] / c[r]");
      W.b[r] = b[r].data_ptr();
      W.c[r] = c[r].data_ptr();
    }
  }
  kgc::launch_allreduce_emu(dt_code(x0), (int)kind, P, W, (int)nr, bytes / 16, wp, M, H,
                            (float)eps, cap_bytes / 16, stream());
}

void skinny_gemm(Tensor C, Tensor X, Tensor W, std::optional<Tensor> bias, int64_t mt,
                 int64_t nt, int64_t nw, bool ntl, int64_t epi, std::optional<Tensor> gamma,
                 double eps, std::optional<Tensor> norm_out, std::optional<Tensor> ticket,
                 std::optional<Tensor> ssp, int64_t nss) {
  check_gpu(X, "X");
  check_same_dev(X, W, "W");
  check_same_dev(X, C, "C");
  c10::hip::HIPGuardMasqueradingAsCUDA g(X.device());
  TORCH_CHECK(X.dim() == 2 && W.dim() == 2 && C.dim() == 2, "kgc.skinny_gemm: 2-D operands");
  TORCH_CHECK(X.scalar_type() == W.scalar_type() && C.scalar_type() == X.scalar_type() &&
              (X.scalar_type() == at::kBFloat16 || X.scalar_type() == at::kHalf),
              "kgc.skinny_gemm: bf16/f16 operands of one dtype");
  TORCH_CHECK(mt == 1 || mt == 2 || mt == 4, "kgc.skinny_gemm: mt in {1,2,4}");
  TORCH_CHECK(nt == 1 || nt == 2, "kgc.skinny_gemm: nt in {1,2}");
  TORCH_CHECK(nw == 4 || nw == 8 || nw == 16, "kgc.skinny_gemm: nw in {4,8,16}");
  const int64_t M = X.size(0), K = X.size(1), N = W.size(0);
  TORCH_CHECK(M >= 1 && M <= 16 * mt, "kgc.skinny_gemm: M must be in [1, 16*mt]");
  TORCH_CHECK(W.size(1) == K && W.is_contiguous(), "kgc.skinny_gemm: W [N, K] contiguous");
  TORCH_CHECK(N % (16 * nt) == 0, "kgc.skinny_gemm: N % (16*nt) != 0");
  TORCH_CHECK(K % (32 * nw) == 0, "kgc.skinny_gemm: K % (32*nw) != 0");
  TORCH_CHECK(X.stride(1) == 1 && X.stride(0) % 8 == 0 && X.stride(0) >= K,
              "kgc.skinny_gemm: X rows dense, 16B aligned");
  if (epi == 3 || epi == 7) {   // SK_SILU: merged [gate; up] weight [2I, K] -> C [M, I]
    TORCH_CHECK(nt == 2 && !bias.has_value() && N % 32 == 0,
                "kgc.skinny_gemm: silu epilogue needs nt=2, no bias, N % 32 == 0");
    TORCH_CHECK(C.size(0) == M && C.size(1) == N / 2 && C.stride(1) == 1,
                "kgc.skinny_gemm: silu epilogue writes C [M, N/2]");
  } else {
    TORCH_CHECK(C.size(0) == M && C.size(1) == N && C.stride(1) == 1, "kgc.skinny_gemm: C [M, N]");
  }
  TORCH_CHECK(N <= INT32_MAX && K <= INT32_MAX, "kgc.skinny_gemm: dims overflow");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(W.data_ptr()) % 16 == 0, "kgc.skinny_gemm: alignment");
  const void* bp = nullptr;
  if (bias.has_value()) {
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == N &&
                bias->scalar_type() == X.scalar_type(), "kgc.skinny_gemm: bias [N]");
    check_same_dev(X, *bias, "bias");
    bp = bias->data_ptr();
  }
  TORCH_CHECK(epi >= 0 && epi <= 7, "kgc.skinny_gemm: epi in {0 plain, 1 norm, 2 accumulate, "
              "3 silu(gate) * up, 4 accumulate + rms_norm, 5 accumulate + row sums of squares, "
              "6 / 7 row-scaled plain / silu pairs}");
  float* sp = nullptr;
  if (epi >= 5) {
    TORCH_CHECK(ssp.has_value() && ssp->scalar_type() == at::kFloat && ssp->is_contiguous(),
                "kgc.skinny_gemm: epi 5-7 need ssp fp32 contiguous");
    check_same_dev(X, *ssp, "ssp");
    if (epi == 5) {
      TORCH_CHECK(ssp->numel() >= M * (N / (16 * nt)), "kgc.skinny_gemm: ssp [M, N / (16 nt)]");
    } else {
      TORCH_CHECK(nss >= 1 && nss <= 256 && ssp->numel() >= M * nss && M <= 4 * nw,
                  "kgc.skinny_gemm: row scale needs 1 <= nss <= 256 partials per row, "
                  "M <= 4 * nw, ssp [M, nss]");
    }
    sp = ssp->data_ptr<float>();
  }
  const void* gp = nullptr;
  if (epi == 1 || epi == 4) {
    const int64_t gn = epi == 1 ? K : N;
    TORCH_CHECK(gamma.has_value() && gamma->is_contiguous() && gamma->numel() == gn &&
                gamma->scalar_type() == X.scalar_type(),
                "kgc.skinny_gemm: norm needs gamma [K] (epi 1) / [N] (epi 4)");
    check_same_dev(X, *gamma, "gamma");
    gp = gamma->data_ptr();
  }
  if (epi == 2 || epi == 4 || epi == 5)   // C is read and rewritten in place: no overlap
    TORCH_CHECK(C.data_ptr() != X.data_ptr(), "kgc.skinny_gemm: accumulate target aliases X");
  void* np = nullptr;
  uint32_t* tp = nullptr;
  if (epi == 4) {
    TORCH_CHECK(N % 512 == 0 && N <= 8192,
                "kgc.skinny_gemm: accumulate + rms_norm needs N % 512 == 0, N <= 8192");
    TORCH_CHECK(norm_out.has_value() && norm_out->is_contiguous() && norm_out->size(0) == M &&
                norm_out->size(1) == N && norm_out->scalar_type() == X.scalar_type() &&
                norm_out->data_ptr() != C.data_ptr(), "kgc.skinny_gemm: norm_out [M, N]");
    TORCH_CHECK(ticket.has_value() && ticket->numel() >= 9 &&
                ticket->scalar_type() == at::kInt, "kgc.skinny_gemm: ticket int32 [>= 9] (top + 8 sub-counters)");
    check_same_dev(X, *norm_out, "norm_out");
    check_same_dev(X, *ticket, "ticket");
    np = norm_out->data_ptr();
    tp = reinterpret_cast<uint32_t*>(ticket->data_ptr());
  }
  kgc::launch_skinny_gemm(dt_code(X), (int)mt, (int)nt, (int)nw, ntl, (int)epi, C.data_ptr(),
                          X.data_ptr(), W.data_ptr(), bp, gp, (float)eps, (int)M, (int)N, (int)K,
                          X.stride(0), C.stride(0), np, tp, sp, (int)nss, stream());
}

void sample_stamps_enable(bool on) { kgc::sample_stamps_enable(on); }

std::vector<int64_t> sample_stamps() {
  uint64_t st[16] = {};
  kgc::sample_stamps_read(st);
  return std::vector<int64_t>(st, st + 16);
}

int64_t decode_wave_min_pairs() { return kgc::paged_decode_wave_min_pairs(); }
int64_t prefill_block_m() { return kgc::prefill_block_m(); }

}  // namespace

TORCH_LIBRARY(kgc, m) {
  m.def("rms_norm(Tensor(a!) out, Tensor x, Tensor(b!)? residual, Tensor weight, float eps) -> ()");
  m.def("layer_norm(Tensor(a!) out, Tensor x, Tensor weight, Tensor bias, float eps) -> ()");
  m.def("silu_mul(Tensor(a!) out, Tensor x) -> ()");
  m.def("rope_kv_write(Tensor qkv, Tensor positions, Tensor cos_sin, Tensor(a!) q_out, "
        "Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor slot_mapping, Tensor? q_norm_w, "
        "Tensor? k_norm_w, int nq, int nkv, int d, float eps, bool use_rope, float k_scale=1.0, "
        "float v_scale=1.0) -> ()");
  m.def("paged_decode(Tensor(a!) out, Tensor q, Tensor k_cache, Tensor v_cache, "
        "Tensor block_tables, Tensor ctx_lens, Tensor(b!) max_logits, Tensor(c!) exp_sums, "
        "Tensor(d!) tmp_out, int Z, float scale, float k_scale=1.0, "
        "float v_scale=1.0) -> ()");
  m.def("paged_decode_rope(Tensor(a!) out, Tensor qkv, Tensor positions, Tensor cos_sin, "
        "Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor slot_mapping, Tensor? q_norm_w, "
        "Tensor? k_norm_w, Tensor block_tables, Tensor ctx_lens, Tensor(d!) max_logits, "
        "Tensor(e!) exp_sums, Tensor(f!) tmp_out, int nq, int Z, "
        "float scale, float eps, bool use_rope, float k_scale=1.0, float v_scale=1.0, "
        "Tensor? row_scale=None) -> ()");
  m.def("prefill_attention(Tensor(a!) out, Tensor q, Tensor k_cache, Tensor v_cache, "
        "Tensor block_tables, Tensor query_start_loc, Tensor seq_lens, Tensor work_seq, "
        "Tensor work_mblk, float scale, float k_scale=1.0, float v_scale=1.0) -> ()");
  m.def("prefill_attention_rope(Tensor(a!) out, Tensor qkv, Tensor cos_sin, Tensor k_cache, "
        "Tensor v_cache, Tensor block_tables, Tensor query_start_loc, Tensor seq_lens, "
        "Tensor work_seq, Tensor work_mblk, int nq, float scale, float k_scale=1.0, "
        "float v_scale=1.0) -> ()");
  m.def("sample(Tensor(a!) out, Tensor logits, Tensor temperature, Tensor top_k, Tensor top_p, "
        "Tensor seeds, bool thresholds=True) -> ()");
  m.def("sample_vp(Tensor(a!) packed, Tensor logits, int V, Tensor temperature, Tensor seeds, "
        "int vocab_off) -> ()");
  m.def("sample_vp_unpack(Tensor(a!) out, Tensor packed) -> ()");
  m.def("decode_wave_min_pairs() -> int", &decode_wave_min_pairs);
  m.def("moe_route(Tensor(a!) topk_w, Tensor(b!) topk_ids, Tensor logits, bool renorm) -> ()");
  m.def("moe_gate_route(Tensor(a!) topk_w, Tensor(b!) topk_ids, Tensor x, Tensor wg, "
        "bool renorm) -> ()");
  m.def("moe_align(Tensor(a!) sorted_ids, Tensor(b!) block_expert, Tensor(c!) meta, "
        "Tensor topk_ids, int e0, int E_local, int bm) -> ()");
  m.def("moe_gemm(Tensor(a!) C, Tensor A, Tensor W, Tensor sorted_ids, Tensor block_expert, "
        "Tensor meta, int npairs, int topk, int bm, bool gather, bool scatter, int splitk=1) -> ()");
  m.def("moe_dgemm(Tensor(a!) C, Tensor A, Tensor Wp, Tensor sorted_ids, Tensor block_expert, "
        "Tensor meta, int npairs, int topk, int bm, int mode, int bn=256) -> ()");
  m.def("moe_combine(Tensor(a!) out, Tensor y, Tensor topk_w, Tensor? row_map=None) -> ()");
  m.def("dense_gemm_splitk(Tensor(a!) Cs, Tensor A, Tensor W, int bm) -> ()");
  m.def("splitk_reduce(Tensor(a!) out, Tensor Cs) -> ()");
  m.def("dgemm(Tensor(a!) C, Tensor X, Tensor W, int cfg, int epi, Tensor? rscale=None) -> ()");
  m.def("dgemm_cfg_info(int cfg) -> int[]", &dgemm_cfg_info);
  m.def("dgemm_num_cfgs() -> int", &dgemm_num_cfgs);
  m.def("dgemm_cfg_has_aux(int cfg) -> bool", &dgemm_cfg_has_aux);
  m.def("dgemm_cfg_epis(int cfg) -> int", &dgemm_cfg_epis);
  m.def("dgemm_ablate(Tensor(a!) C, Tensor X, Tensor W, int mode) -> ()");
  m.def("dgemm_pack(Tensor(a!) P, Tensor W, bool silu) -> ()");
  m.def("splitk_reduce_silu(Tensor(a!) out, Tensor Cs, bool interleaved=False, "
        "Tensor? rscale=None) -> ()");
  m.def("splitk_add_rms_norm(Tensor(a!) out, Tensor Cs, Tensor(b!) residual, Tensor w, float eps) -> ()");
  m.def("ar_signal_bytes() -> int", &ar_signal_bytes);
  m.def("ar_alloc(int bytes) -> int", &ar_alloc);
  m.def("ar_free(int ptr) -> ()", &ar_free);
  m.def("ar_get_handle(int ptr) -> Tensor", &ar_get_handle);
  m.def("ar_open_handle(Tensor handle) -> int", &ar_open_handle);
  m.def("ar_close_handle(int ptr) -> ()", &ar_close_handle);
  m.def("ar_read_err(int sig) -> int", &ar_read_err);
  m.def("ar_raise_peer_flags(int sig, int rank, int nranks, int value) -> ()",
        &ar_raise_peer_flags);
  m.def("ep_raise_peer_flags(int sig, int rank, int nranks, int value) -> ()",
        &ep_raise_peer_flags_op);
  m.def("ar_err_copy_async(int sig, Tensor(a!) host_out) -> ()", &ar_err_copy_async);
  m.def("xgmi_allreduce(Tensor(a!) inout, int[] data, int[] sig, int rank, int cap_bytes, "
        "bool two_shot, bool wide=False) -> ()");
  m.def("xgmi_allreduce_rms(Tensor(a!) out, Tensor inp, Tensor(b!) residual, Tensor w, float eps, "
        "int[] data, int[] sig, int rank, int cap_bytes, bool two_shot=False) -> ()");
  m.def("xgmi_allreduce_emu(int kind, Tensor(a!)[] a, Tensor(b!)[] b, Tensor(c!)[] c, Tensor? w, "
        "int[] data, int[] sig, int cap_bytes, float eps) -> ()");
  m.def("allreduce_rms_max_hidden() -> int", &allreduce_rms_max_hidden_op);
  m.def("allreduce_max_blocks() -> int", &allreduce_max_blocks_op);
  m.def("peer_spin_ms() -> int", &peer_spin_ms_op);
  m.def("coop_spin_ms() -> int", &coop_spin_ms_op);
  m.def("wall_clock_rate_khz() -> int", &wall_clock_rate_khz_op);
  m.def("debug_errors() -> int", &debug_errors);
  m.def("sample_err_addr() -> int", &sample_err_addr);
  m.def("u32_clear_async(int addr) -> ()", &u32_clear_async);
  m.def("u32_fill_async(int addr, int value) -> ()", &u32_fill_async);
  m.def("ep_signal_bytes() -> int", &ep_signal_bytes_op);
  m.def("pp_signal_bytes() -> int", &pp_signal_bytes_op);
  m.def("u32_copy_async(int addr, Tensor(a!) host_out, int index) -> ()", &u32_copy_async);
  m.def("pp_read_err(int sig) -> int", &pp_read_err_op);
  m.def("pp_send(Tensor h, Tensor r, int peer_data, int peer_sig, int own_sig, int slot_bytes, "
        "int R) -> ()");
  m.def("pp_recv(Tensor(a!) h, Tensor(b!) r, int own_data, int own_sig, int peer_sig, "
        "int slot_bytes, int R) -> ()");
  m.def("ep_region_bytes(int nr, int C, int H, int esz) -> int", &ep_region_bytes_op);
  m.def("ep_max_pairs() -> int", &ep_max_pairs_op);
  m.def("ep_read_err(int sig) -> int", &ep_read_err_op);
  m.def("ep_err_copy_async(int sig, Tensor(a!) host_out) -> ()", &ep_err_copy_async);
  m.def("ep_dispatch(Tensor x, Tensor topk_ids, int[] data, int[] sig, int rank, int E_local, "
        "int C) -> ()");
  m.def("ep_receive(Tensor(a!) x_local, Tensor(b!) ids, Tensor(c!) route, int[] data, int[] sig, "
        "int rank, int E_local, int C) -> ()");
  m.def("ep_return(Tensor y, Tensor route, int[] data, int[] sig, int rank, int C, "
        "ScalarType? out_dtype=None) -> ()");
  m.def("ep_combine(Tensor(a!) out, Tensor topk_w, int[] data, int[] sig, int rank, int C) -> ()");
  m.def("debug_build() -> bool", &debug_build);
  m.def("sample_stamps_enable(bool on) -> ()", &sample_stamps_enable);
  m.def("sample_stamps() -> int[]", &sample_stamps);
  m.def("prefill_block_m() -> int", &prefill_block_m);
  m.def("skinny_gemm(Tensor(a!) C, Tensor X, Tensor W, Tensor? bias, int mt, int nt, int nw, "
        "bool ntl, int epi=0, Tensor? gamma=None, float eps=1e-6, Tensor(b!)? norm_out=None, "
        "Tensor(c!)? ticket=None, Tensor(d!)? ssp=None, int nss=0) -> ()");
}

TORCH_LIBRARY_IMPL(kgc, CUDA, m) {
  m.impl("rms_norm", &rms_norm);
  m.impl("layer_norm", &layer_norm);
  m.impl("silu_mul", &silu_mul);
  m.impl("rope_kv_write", &rope_kv_write);
  m.impl("paged_decode", &paged_decode);
  m.impl("paged_decode_rope", &paged_decode_rope);
  m.impl("prefill_attention", &prefill_attention);
  m.impl("prefill_attention_rope", &prefill_attention_rope);
  m.impl("sample", &sample);
  m.impl("sample_vp", &sample_vp);
  m.impl("sample_vp_unpack", &sample_vp_unpack);
  m.impl("xgmi_allreduce", &xgmi_allreduce);
  m.impl("xgmi_allreduce_rms", &xgmi_allreduce_rms);
  m.impl("xgmi_allreduce_emu", &xgmi_allreduce_emu);
  m.impl("ep_dispatch", &ep_dispatch);
  m.impl("pp_send", &pp_send);
  m.impl("pp_recv", &pp_recv);
  m.impl("ep_receive", &ep_receive);
  m.impl("ep_return", &ep_return);
  m.impl("ep_combine", &ep_combine);
  m.impl("moe_route", &moe_route);
  m.impl("moe_gate_route", &moe_gate_route);
  m.impl("moe_align", &moe_align);
  m.impl("moe_gemm", &moe_gemm);
  m.impl("moe_dgemm", &moe_dgemm);
  m.impl("moe_combine", &moe_combine);
  m.impl("dense_gemm_splitk", &dense_gemm_splitk);
  m.impl("dgemm", &dgemm);
  m.impl("dgemm_ablate", &dgemm_ablate);
  m.impl("dgemm_pack", &dgemm_pack);
  m.impl("splitk_reduce", &splitk_reduce);
  m.impl("splitk_reduce_silu", &splitk_reduce_silu);
  m.impl("splitk_add_rms_norm", &splitk_add_rms_norm);
  m.impl("skinny_gemm", &skinny_gemm);
}
