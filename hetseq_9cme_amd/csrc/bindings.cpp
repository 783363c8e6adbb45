// torch <-> gfx950 kernel bindings.  Host-only TU: validates tensors, allocates
// outputs through the torch caching allocator, and launches on the CURRENT HIP
// stream of the tensor's device (so kernels order correctly with hipBLASLt GEMMs
// and RCCL, and are capturable into HIP graphs).
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "hx_launch.h"

namespace {

using torch::Tensor;
using OptT = c10::optional<Tensor>;

inline hipStream_t cur_stream(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.get_device()).stream(); }

inline void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
// Per-update dropout key: a 1-element int64 tensor on the kernel's device, read by the
// kernels themselves (ops/rng.py keeps it; graph-captured steps replay with new keys).
inline const uint64_t* seed_ptr(const Tensor& seed) {
  TORCH_CHECK(seed.is_cuda() && seed.scalar_type() == torch::kInt64 && seed.numel() >= 1,
              "dropout seed must be a 1-element int64 GPU tensor");
  return reinterpret_cast<const uint64_t*>(seed.data_ptr<int64_t>());
}
inline int act_bf16(const Tensor& t) {
  TORCH_CHECK(t.scalar_type() == torch::kFloat32 || t.scalar_type() == torch::kBFloat16, "activations must be fp32 or bf16");
  return t.scalar_type() == torch::kBFloat16 ? 1 : 0;
}
inline void check_f32(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be fp32");
}
template <typename T>
inline T* ptr_or_null(const OptT& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}
inline bool has(const OptT& t) { return t.has_value() && t->defined(); }
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// ------------------------------------------------------------------ debug mode
// ``--debug-kernels``: host-side validation that needs device reads
// (range checks on indices, finite checks on every fused op's output).  Each check
// synchronises, so it is off by default; combined with AMD_SERIALIZE_KERNEL=3 the
// first kernel producing a bad value is the one that raises.
bool g_debug = false;
void set_debug(bool on) { g_debug = on; }
bool get_debug() { return g_debug; }
inline void dbg_range(const Tensor& t, int64_t lo, int64_t hi, const char* what) {
  if (!g_debug || t.numel() == 0) return;
  const int64_t mn = t.min().item<int64_t>(), mx = t.max().item<int64_t>();
  TORCH_CHECK(mn >= lo && mx < hi, what, " out of range: [", mn, ", ", mx, "] not within [", lo, ", ", hi, ")");
}
inline void dbg_finite(const Tensor& t, const char* what) {
  if (!g_debug || !t.defined() || t.numel() == 0) return;
  TORCH_CHECK(torch::isfinite(t).all().item<bool>(), "non-finite values produced by ", what);
}

// ------------------------------------------------------------------ optimizer
void grad_norm_clip(Tensor g, Tensor gscale, Tensor out_norm, Tensor clipped, double max_norm) {
  check_f32(g, "grad");
  check_f32(gscale, "gscale");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  TORCH_CHECK(aligned16(g.data_ptr()), "flat grad must be 16-byte aligned");
  auto ws = torch::empty({hx_grad_norm_partials()}, g.options().dtype(torch::kFloat64));
  hx_grad_norm_clip(g.data_ptr<float>(), g.numel(), ws.data_ptr<double>(), gscale.data_ptr<float>(),
                    out_norm.data_ptr<float>(), clipped.data_ptr<float>(), (float)max_norm, cur_stream(g));
}

// hp (optional, device fp32 [2]): step size and wd * lr read by the kernel instead of the
// host values -- a captured training step (utils/train_graph.py) refreshes them per replay
inline const float* hp_ptr(const OptT& hp, int64_t need) {
  if (!has(hp)) return nullptr;
  TORCH_CHECK(hp->is_cuda() && hp->scalar_type() == torch::kFloat32 && hp->numel() >= need && hp->is_contiguous(),
              "optimizer hyper-parameters must be a contiguous fp32 GPU tensor");
  return hp->data_ptr<float>();
}

void adam(Tensor p, Tensor g, Tensor m, Tensor v, OptT shadow, Tensor gscale, int64_t start, int64_t end, double b1,
          double b2, double eps, double step_size, double wd_lr, OptT hp) {
  check_f32(p, "param");
  check_f32(g, "grad");
  check_f32(m, "exp_avg");
  check_f32(v, "exp_avg_sq");
  TORCH_CHECK(start >= 0 && end <= p.numel() && start <= end && start % 4 == 0, "bad param range");
  TORCH_CHECK(g.numel() == p.numel() && m.numel() == p.numel() && v.numel() == p.numel(), "flat size mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  uint16_t* sh = nullptr;
  if (has(shadow)) {
    TORCH_CHECK(shadow->scalar_type() == torch::kBFloat16 && shadow->numel() == p.numel(), "bad bf16 shadow");
    sh = reinterpret_cast<uint16_t*>(shadow->data_ptr()) + start;
  }
  hx_adam(p.data_ptr<float>() + start, g.data_ptr<float>() + start, m.data_ptr<float>() + start,
          v.data_ptr<float>() + start, sh, gscale.data_ptr<float>(), end - start, (float)b1, (float)b2, (float)eps,
          (float)step_size, (float)wd_lr, hp_ptr(hp, 2), cur_stream(p));
}

void adam_masked(Tensor p, Tensor g, Tensor m, Tensor v, OptT shadow, Tensor gscale, Tensor table, Tensor used,
                 Tensor steps, Tensor hp, double lr, double b1, double b2, double eps, double wd, OptT lr_dev) {
  check_f32(p, "param");
  check_f32(g, "grad");
  check_f32(m, "exp_avg");
  check_f32(v, "exp_avg_sq");
  TORCH_CHECK(g.numel() == p.numel() && m.numel() == p.numel() && v.numel() == p.numel(), "flat size mismatch");
  const int64_t nparam = steps.numel();
  TORCH_CHECK(steps.is_cuda() && steps.scalar_type() == torch::kInt32 && steps.is_contiguous(), "steps: int32 GPU");
  TORCH_CHECK(used.is_cuda() && used.scalar_type() == torch::kFloat64 && used.is_contiguous() &&
                  used.numel() == nparam, "used flags: contiguous f64 GPU tensor, one per parameter");
  TORCH_CHECK(hp.is_cuda() && hp.scalar_type() == torch::kFloat32 && hp.numel() >= 2 * nparam, "hp: f32 [2*nparam]");
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == torch::kInt64 && table.dim() == 2 && table.size(1) == 3 &&
                  table.is_contiguous(), "table: int64 [nblocks, 3]");
  uint16_t* sh = nullptr;
  if (has(shadow)) {
    TORCH_CHECK(shadow->scalar_type() == torch::kBFloat16 && shadow->numel() == p.numel(), "bad bf16 shadow");
    sh = reinterpret_cast<uint16_t*>(shadow->data_ptr());
  }
  if (has(lr_dev))
    TORCH_CHECK(lr_dev->is_cuda() && lr_dev->scalar_type() == torch::kFloat64 && lr_dev->numel() == 1, "lr_dev: f64 [1]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  hx_adam_masked(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), sh,
                 gscale.data_ptr<float>(), table.data_ptr<int64_t>(), (int)table.size(0), used.data_ptr<double>(),
                 steps.data_ptr<int>(), hp.data_ptr<float>(), (int)nparam, lr, b1, b2, (float)eps, wd,
                 has(lr_dev) ? lr_dev->data_ptr<double>() : nullptr, cur_stream(p));
}

void adadelta(Tensor p, Tensor g, Tensor sq, Tensor acc, Tensor gscale, int64_t start, int64_t end, double lr,
              double rho, double eps, double wd, OptT hp) {
  check_f32(p, "param");
  TORCH_CHECK(start >= 0 && end <= p.numel() && start <= end, "bad param range");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  hx_adadelta(p.data_ptr<float>() + start, g.data_ptr<float>() + start, sq.data_ptr<float>() + start,
              acc.data_ptr<float>() + start, gscale.data_ptr<float>(), end - start, (float)lr, (float)rho,
              (float)eps, (float)wd, hp_ptr(hp, 1), cur_stream(p));
}

// ------------------------------------------------------------------ layernorm
// amax_out (fp32 runs only): receives max |out| of every row, [rows] (the fp16x3 GEMMs' per-row
// operand scale, ops/gemm16.py)
inline float* amax_ptr(const OptT& a, int64_t need, const char* what) {
  if (!has(a)) return nullptr;
  check_f32(*a, what);
  TORCH_CHECK(a->is_contiguous() && a->numel() >= need, what, ": needs ", need, " fp32 partials");
  return a->data_ptr<float>();
}
// pieces_out (fp32 runs, with amax_out): fp16 P2 pieces [rows, 2H] of the output at its row scales,
// the consumer GEMM's A operand already split (gemm_f16 with fp16 A)
inline uint16_t* pieces_ptr(const OptT& p, int64_t rows, int H, const OptT& amax, const char* what) {
  if (!has(p)) return nullptr;
  TORCH_CHECK(has(amax), what, ": pieces need the row maxima output too");
  TORCH_CHECK(p->is_cuda() && p->scalar_type() == torch::kHalf && p->is_contiguous() && p->numel() == rows * 2 * H &&
                  H % 16 == 0 && aligned16(p->data_ptr()), what, ": fp16 [rows, 2H] (H % 16 == 0)");
  return reinterpret_cast<uint16_t*>(p->data_ptr());
}
std::vector<Tensor> ln_fwd(Tensor y, OptT bias, OptT res, Tensor gamma, Tensor beta, double eps, double keep_prob,
                           const Tensor& seed, int64_t stream, bool drop_after, bool save_z, OptT amax_out,
                           OptT pieces_out) {
  check_cuda(y, "input");
  const int H = (int)y.size(-1);
  const int64_t rows = y.numel() / H;
  TORCH_CHECK(H % 4 == 0 && H <= 2048, "LayerNorm hidden size must be a multiple of 4 and <= 2048");
  check_f32(gamma, "gamma");
  check_f32(beta, "beta");
  if (has(res)) {
    check_cuda(*res, "residual");
    TORCH_CHECK(res->scalar_type() == y.scalar_type() && res->numel() == y.numel(), "residual mismatch");
  }
  if (has(bias)) check_f32(*bias, "bias");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(y.device());
  auto out = torch::empty_like(y);
  Tensor z = save_z ? torch::empty_like(y) : Tensor();
  auto st = y.options().dtype(torch::kFloat32);
  auto mean = torch::empty({rows}, st), rstd = torch::empty({rows}, st);
  hx_ln_fwd(act_bf16(y), y.data_ptr(), ptr_or_null<float>(bias), has(res) ? res->data_ptr() : nullptr,
            gamma.data_ptr<float>(), beta.data_ptr<float>(), out.data_ptr(), save_z ? z.data_ptr() : nullptr,
            mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, H, (float)eps, (float)keep_prob, seed_ptr(seed),
            (uint64_t)stream, drop_after ? 1 : 0, cur_stream(y),
            act_bf16(y) ? nullptr : amax_ptr(amax_out, rows, "ln_fwd amax"),
            act_bf16(y) ? nullptr : pieces_ptr(pieces_out, rows, H, amax_out, "ln_fwd pieces"));
  dbg_finite(out, "ln_fwd");
  return {out, z, mean, rstd};
}

std::vector<Tensor> ln_bwd(Tensor dout, Tensor z, Tensor mean, Tensor rstd, Tensor gamma, double keep_prob,
                           const Tensor& seed, int64_t stream, bool drop_after, bool want_dy, bool want_dbias,
                           OptT dgamma_out, OptT dbeta_out, OptT dbias_out, OptT amax_out, OptT colmax_out,
                           OptT pieces_out) {
  check_cuda(dout, "grad_output");
  check_cuda(z, "saved input");
  const int H = (int)z.size(-1);
  const int64_t rows = z.numel() / H;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(z.device());
  auto dz = torch::empty_like(z);
  Tensor dy = want_dy ? torch::empty_like(z) : Tensor();
  auto f32 = z.options().dtype(torch::kFloat32);
  auto dgamma = has(dgamma_out) ? *dgamma_out : torch::empty({H}, f32);
  auto dbeta = has(dbeta_out) ? *dbeta_out : torch::empty({H}, f32);
  Tensor dbias = want_dbias ? (has(dbias_out) ? *dbias_out : torch::empty({H}, f32)) : Tensor();
  TORCH_CHECK(dgamma.numel() == H && dbeta.numel() == H && dgamma.is_contiguous() && dbeta.is_contiguous(),
              "bad dgamma/dbeta outputs");
  const int nblk = hx_ln_bwd_blocks(rows);
  auto partial = torch::empty({(int64_t)nblk * 4 * H}, f32);
  hx_ln_bwd(act_bf16(z), dout.data_ptr(), z.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
            gamma.data_ptr<float>(), dz.data_ptr(), want_dy ? dy.data_ptr() : nullptr, partial.data_ptr<float>(), nblk,
            rows, H, (float)keep_prob, seed_ptr(seed), (uint64_t)stream, drop_after ? 1 : 0,
            (want_dy && want_dbias) ? 1 : 0, dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
            want_dbias ? dbias.data_ptr<float>() : nullptr, 0, cur_stream(z),
            act_bf16(z) ? nullptr : amax_ptr(amax_out, rows, "ln_bwd amax"),
            act_bf16(z) ? nullptr : amax_ptr(colmax_out, H, "ln_bwd colmax"),
            act_bf16(z) ? nullptr : pieces_ptr(pieces_out, rows, H, amax_out, "ln_bwd pieces"));
  dbg_finite(dz, "ln_bwd (dz)");
  return {dz, dy, dgamma, dbeta, dbias};
}

std::vector<Tensor> embed_ln_fwd(Tensor ids, OptT tt, Tensor wte, Tensor wpe, Tensor wtt, Tensor gamma, Tensor beta,
                                 double eps, double keep_prob, const Tensor& seed, int64_t stream, bool bf16_out,
                                 OptT amax_out, OptT pieces_out) {
  dbg_range(ids, 0, wte.size(0), "token ids");
  if (has(tt)) dbg_range(*tt, 0, wtt.size(0), "token type ids");
  check_cuda(ids, "input_ids");
  TORCH_CHECK(ids.scalar_type() == torch::kInt64 && ids.dim() == 2, "input_ids must be int64 [B, S]");
  check_f32(wte, "word_embeddings");
  check_f32(wpe, "position_embeddings");
  check_f32(wtt, "token_type_embeddings");
  const int64_t B = ids.size(0), S = ids.size(1);
  const int H = (int)wte.size(1);
  TORCH_CHECK(H % 4 == 0 && H <= 2048, "hidden size must be a multiple of 4 and <= 2048");
  TORCH_CHECK(S <= wpe.size(0), "sequence longer than max_position_embeddings");
  if (has(tt)) TORCH_CHECK(tt->scalar_type() == torch::kInt64 && tt->numel() == ids.numel(), "token_type_ids mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(ids.device());
  auto opt = wte.options().dtype(bf16_out ? torch::kBFloat16 : torch::kFloat32);
  auto out = torch::empty({B, S, H}, opt), z = torch::empty({B, S, H}, opt);
  auto f32 = wte.options();
  auto mean = torch::empty({B * S}, f32), rstd = torch::empty({B * S}, f32);
  hx_embed_ln_fwd(bf16_out ? 1 : 0, ids.data_ptr<int64_t>(), has(tt) ? tt->data_ptr<int64_t>() : nullptr,
                  wte.data_ptr<float>(), wpe.data_ptr<float>(), wtt.data_ptr<float>(), gamma.data_ptr<float>(),
                  beta.data_ptr<float>(), out.data_ptr(), z.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                  B * S, (int)S, H, (float)eps, (float)keep_prob, seed_ptr(seed), (uint64_t)stream, cur_stream(ids),
                  bf16_out ? nullptr : amax_ptr(amax_out, B * S, "embed_ln_fwd amax"),
                  bf16_out ? nullptr : pieces_ptr(pieces_out, B * S, H, amax_out, "embed_ln_fwd pieces"));
  dbg_finite(out, "embed_ln_fwd");
  return {out, z, mean, rstd};
}

// Scatter-ACCUMULATES the embedding gradients into dwte / dwpe / dwtt (caller zeroes them
// when they are fresh).
// word-embedding gradient, accumulated into dwte: rows visited in id-sorted order
void embed_word_grad(Tensor dz, Tensor ids, Tensor order, Tensor dwte) {
  check_cuda(dz, "grad");
  check_cuda(ids, "ids");
  check_cuda(order, "order");
  check_f32(dwte, "dwte");
  TORCH_CHECK(ids.scalar_type() == torch::kLong && order.scalar_type() == torch::kLong, "ids/order must be int64");
  const int H = (int)dz.size(-1);
  const int64_t rows = dz.numel() / H;
  TORCH_CHECK(ids.numel() == rows && order.numel() == rows, "ids/order/grad row mismatch");
  TORCH_CHECK(dwte.size(-1) == H && H % 4 == 0 && H <= 2048, "bad embedding width");
  dbg_range(ids, 0, dwte.size(0), "token ids");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dz.device());
  hx_embed_word_grad_sorted(act_bf16(dz), dz.data_ptr(), ids.data_ptr<int64_t>(), order.data_ptr<int64_t>(),
                            dwte.data_ptr<float>(), rows, H, cur_stream(dz));
}

// token-type embedding gradient (ntypes <= 3) into dwtt [ntypes, H] (overwritten)
void embed_type_grad(Tensor dz, Tensor tt, Tensor dwtt) {
  check_cuda(dz, "grad");
  check_f32(dwtt, "dwtt");
  TORCH_CHECK(tt.scalar_type() == torch::kLong && tt.is_contiguous() && tt.device() == dz.device(), "tt: int64");
  const int H = (int)dz.size(-1);
  const int64_t rows = dz.numel() / H;
  const int ntypes = (int)dwtt.size(0);
  TORCH_CHECK(dz.is_contiguous() && tt.numel() == rows && dwtt.dim() == 2 && dwtt.size(1) == H &&
                  dwtt.is_contiguous() && ntypes >= 1 && ntypes <= 3 && H % 4 == 0 && H <= 2048,
              "embed_type_grad: contiguous dz [rows, H], tt [rows], dwtt [ntypes <= 3, H]");
  dbg_range(tt, 0, ntypes, "token type ids");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dz.device());
  Tensor part = torch::empty({(int64_t)hx_type_grad_blocks(rows) * ntypes * H}, dz.options().dtype(torch::kFloat32));
  hx_type_grad(act_bf16(dz), dz.data_ptr(), tt.data_ptr<int64_t>(), part.data_ptr<float>(), dwtt.data_ptr<float>(),
               rows, H, ntypes, cur_stream(dz));
}

// ------------------------------------------------------------------ elementwise
Tensor bias_act_fwd(Tensor y, OptT b, int64_t act) {
  check_cuda(y, "input");
  const int N = (int)y.size(-1);
  TORCH_CHECK(N % 4 == 0, "bias_act: last dim must be a multiple of 4");
  if (has(b)) check_f32(*b, "bias");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(y.device());
  auto out = torch::empty_like(y);
  hx_bias_act_fwd(act_bf16(y), (int)act, y.data_ptr(), ptr_or_null<float>(b), out.data_ptr(), y.numel() / N, N,
                  cur_stream(y));
  dbg_finite(out, "bias_act_fwd");
  return out;
}

std::vector<Tensor> bias_act_bwd(Tensor dout, OptT y, OptT b, OptT saved_out, int64_t act, bool want_dbias,
                                 OptT dbias_out) {
  check_cuda(dout, "grad_output");
  const int N = (int)dout.size(-1);
  const int64_t rows = dout.numel() / N;
  TORCH_CHECK(N % 4 == 0, "bias_act: last dim must be a multiple of 4");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dout.device());
  auto dy = torch::empty_like(dout);
  auto f32 = dout.options().dtype(torch::kFloat32);
  Tensor dbias, ws;
  if (want_dbias) {
    dbias = has(dbias_out) ? *dbias_out : torch::empty({N}, f32);
    ws = torch::empty({(int64_t)hx_colsum_ws_floats(rows, N)}, f32);
  }
  hx_bias_act_bwd(act_bf16(dout), (int)act, dout.data_ptr(), has(y) ? y->data_ptr() : nullptr, ptr_or_null<float>(b),
                  has(saved_out) ? saved_out->data_ptr() : nullptr, dy.data_ptr(),
                  want_dbias ? ws.data_ptr<float>() : nullptr, want_dbias ? dbias.data_ptr<float>() : nullptr, rows, N,
                  0, cur_stream(dout));
  dbg_finite(dy, "bias_act_bwd");
  return {dy, dbias};
}

Tensor colsum(Tensor x, OptT scale, OptT out_) {
  TORCH_CHECK(x.is_cuda(), "input must be a GPU tensor");
  const int N = (int)x.size(-1);
  // 2-D with unit column stride: any row stride (e.g. the valid columns of a padded buffer)
  const bool strided2d = x.dim() == 2 && x.stride(1) == 1;
  TORCH_CHECK(strided2d || x.is_contiguous(), "colsum: contiguous input or 2-D rows with unit column stride");
  const int64_t rows = strided2d ? x.size(0) : x.numel() / N;
  const int64_t ld = strided2d ? x.stride(0) : N;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto f32 = x.options().dtype(torch::kFloat32);
  auto out = has(out_) ? *out_ : torch::empty({N}, f32);
  TORCH_CHECK(out.numel() == N && out.is_contiguous(), "bad colsum output");
  auto ws = torch::empty({(int64_t)hx_colsum_ws_floats(rows, N)}, f32);
  hx_colsum(act_bf16(x), x.data_ptr(), ptr_or_null<float>(scale), ws.data_ptr<float>(), out.data_ptr<float>(), rows,
            N, 0, cur_stream(x), ld);
  return out;
}

Tensor dropout(Tensor x, double keep_prob, const Tensor& seed, int64_t stream) {
  check_cuda(x, "input");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto out = torch::empty_like(x);
  hx_dropout(act_bf16(x), x.data_ptr(), out.data_ptr(), x.numel(), (float)keep_prob, seed_ptr(seed),
             (uint64_t)stream, cur_stream(x));
  return out;
}

Tensor softmax_xent_(Tensor logits, OptT bias, Tensor labels, int64_t ignore_index) {
  dbg_range(labels, std::min<int64_t>(ignore_index, 0), logits.size(-1), "MLM labels");
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1, "logits must be a 2-D row-major GPU tensor");
  check_cuda(labels, "labels");
  TORCH_CHECK(labels.scalar_type() == torch::kInt64 && labels.numel() == logits.size(0), "labels must be int64 [rows]");
  if (has(bias)) {
    check_f32(*bias, "bias");
    TORCH_CHECK(bias->numel() >= logits.size(1), "bias too small");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  auto loss = torch::empty({logits.size(0)}, logits.options().dtype(torch::kFloat32));
  hx_softmax_xent(act_bf16(logits), logits.data_ptr(), ptr_or_null<float>(bias), labels.data_ptr<int64_t>(),
                  loss.data_ptr<float>(), logits.size(0), (int)logits.size(1), logits.stride(0), ignore_index,
                  cur_stream(logits));
  dbg_finite(loss, "softmax_xent");
  return loss;
}

// ------------------------------------------------------------------ attention
std::vector<Tensor> attn_fwd(Tensor qkv, Tensor mask_bias, int64_t nh, double keep, const Tensor& seed, int64_t stream,
                             OptT bias, int split = 0, OptT amax_out = OptT(), OptT colmax_out = OptT()) {
  // split: 0 none (fp32 / bf16 MFMA), 2 fp16x3 (attention_f16.hip)
  check_cuda(qkv, "qkv");
  const int bf = act_bf16(qkv);
  check_f32(mask_bias, "mask_bias");
  TORCH_CHECK(qkv.dim() == 3, "qkv must be [B, S, 3H]");
  const int64_t B = qkv.size(0), S = qkv.size(1), H = qkv.size(2) / 3;
  TORCH_CHECK(H == nh * 64, "fused attention needs head_dim == 64");
  TORCH_CHECK(mask_bias.numel() == B * S, "mask_bias must be [B, S]");
  if (has(bias)) {
    check_f32(*bias, "qkv bias");
    TORCH_CHECK(bias->numel() == 3 * H, "qkv bias must have 3H elements");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  auto out = torch::empty({B, S, H}, qkv.options());
  auto lse = torch::empty({B, nh, S}, qkv.options().dtype(torch::kFloat32));
  Tensor dmask;
  // 1 bit per (key, query), stored [key][query word] with both padded to 128
  const int64_t Sp = (S + 127) / 128 * 128;
  if (keep < 1.0) dmask = torch::empty({B, nh, Sp, Sp / 32}, qkv.options().dtype(torch::kInt32));
  else dmask = torch::empty({0}, qkv.options().dtype(torch::kInt32));
  uint32_t* dm = keep < 1.0 ? reinterpret_cast<uint32_t*>(dmask.data_ptr<int32_t>()) : nullptr;
  if (split) {
    TORCH_CHECK(!bf, "attn_fwd_f16: fp32 activations only");
    float* am = amax_ptr(amax_out, B * S * nh, "attn_fwd amax");   // [B * S rows][nh heads]
    float* cm = amax_ptr(colmax_out, B * ((S + 127) / 128) * H, "attn_fwd colmax");   // [B * qblocks][H]
    hx_attn_fwd_f16(qkv.data_ptr<float>(), ptr_or_null<float>(bias), mask_bias.data_ptr<float>(),
                    out.data_ptr<float>(), lse.data_ptr<float>(), dm, (int)B, (int)S, (int)nh, (float)keep,
                    seed_ptr(seed), (uint64_t)stream, cur_stream(qkv), am, cm);
  } else {
    hx_attn_fwd(bf, qkv.data_ptr(), ptr_or_null<float>(bias), mask_bias.data_ptr<float>(), out.data_ptr(),
                lse.data_ptr<float>(), dm, (int)B, (int)S, (int)nh, (float)keep, seed_ptr(seed), (uint64_t)stream,
                cur_stream(qkv));
  }
  dbg_finite(out, "attn_fwd");
  return {out, lse, dmask};
}
// fp32 attention forward on the fp16 matrix cores (fp16x3, attention_f16.hip): {out, lse, dmask}
std::vector<Tensor> attn_fwd_f16(Tensor qkv, Tensor mask_bias, int64_t nh, double keep, const Tensor& seed,
                                 int64_t stream, OptT bias, OptT amax_out, OptT colmax_out) {
  return attn_fwd(qkv, mask_bias, nh, keep, seed, stream, bias, 2, amax_out, colmax_out);
}

// returns {dqkv, dbias} (dbias: [3H] fp32 when bias is given or want_dbias -- written into
// dbq/dbk/dbv when those slots are given -- else an empty tensor)
std::vector<Tensor> attn_bwd(Tensor dout, Tensor qkv, Tensor mask_bias, Tensor out, Tensor lse, Tensor dmask,
                             int64_t nh, double keep, OptT bias, OptT dbq, OptT dbk, OptT dbv, int split = 0,
                             OptT amax_out = OptT(), OptT colmax_out = OptT(), bool want_dbias = false) {
  // split: 0 none (fp32 / bf16 MFMA), 2 fp16x3 (attention_f16.hip)
  check_cuda(dout, "grad_output");
  check_cuda(qkv, "qkv");
  const int bf = act_bf16(qkv);
  TORCH_CHECK(!(split && bf), "attn_bwd_f16: fp32 activations only");
  TORCH_CHECK(dout.scalar_type() == qkv.scalar_type() && out.scalar_type() == qkv.scalar_type(),
              "attention activations must share one dtype");
  const int64_t B = qkv.size(0), S = qkv.size(1), H = qkv.size(2) / 3;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  // one key block per head (S <= 128): every dQKV element is written exactly once (no
  // memset).  Otherwise dQ partials from the S/128 key blocks are added atomically in
  // fp32: into dqkv itself (fp32, its dQ third zero-filled) or a [B, S, H] fp32 scratch (bf16).
  const bool multi = S > 128;
  Tensor dqkv = torch::empty_like(qkv);
  if (multi && !bf) dqkv.narrow(-1, 0, H).zero_();   // only the dQ third is accumulated into
  Tensor dq32;
  float* dq_acc = nullptr;
  int dq_ld = 0;
  if (multi && bf) {
    dq32 = torch::zeros({B, S, H}, qkv.options().dtype(torch::kFloat32));
    dq_acc = dq32.data_ptr<float>();
    dq_ld = (int)H;
  } else if (multi) {
    dq_acc = dqkv.data_ptr<float>();
    dq_ld = (int)(3 * H);
  }
  Tensor dbias, part;
  float *pq = nullptr, *pk = nullptr, *pv = nullptr;
  // the QKV-bias gradient: when the bias is added here, or (want_dbias) when the projection
  // already added it and only its gradient -- the column sums of dQKV -- is wanted
  if (has(bias) || want_dbias) {
    const bool slots = has(dbq) && has(dbk) && has(dbv);
    if (slots) {
      for (const auto* t : {&dbq, &dbk, &dbv}) {
        check_f32(**t, "qkv bias grad");
        TORCH_CHECK((*t)->numel() == H, "qkv bias grad must have H elements");
      }
      pq = dbq->data_ptr<float>(); pk = dbk->data_ptr<float>(); pv = dbv->data_ptr<float>();
    } else {
      dbias = torch::empty({3 * H}, qkv.options().dtype(torch::kFloat32));
      pq = dbias.data_ptr<float>(); pk = pq + H; pv = pq + 2 * H;
    }
    part = torch::empty({B * ((S + 127) / 128), 3 * H}, qkv.options().dtype(torch::kFloat32));
  }
  hx_attn_bwd(split ? 3 : bf, qkv.data_ptr(), ptr_or_null<float>(bias), pq, pk, pv, part.defined() ? part.data_ptr<float>() : nullptr,
              mask_bias.data_ptr<float>(), dout.data_ptr(), out.data_ptr(), lse.data_ptr<float>(),
              keep < 1.0 ? reinterpret_cast<const uint32_t*>(dmask.data_ptr<int32_t>()) : nullptr,
              dqkv.data_ptr(), dq_acc, dq_ld, (int)B, (int)S, (int)nh, (float)keep, cur_stream(qkv),
              split ? amax_ptr(amax_out, B * S * nh, "attn_bwd amax") : nullptr,   // [B * S][nh]
              split ? amax_ptr(colmax_out, B * ((S + 127) / 128) * 3 * H, "attn_bwd colmax") : nullptr);   // [B * kb][3H]
  if (multi && bf) dqkv.narrow(-1, 0, H).copy_(dq32);
  dbg_finite(dqkv, "attn_bwd");
  return {dqkv, dbias};
}

// ------------------------------------------------------------------ bf16 weight gradient
// out[M, N] (fp32, overwritten) = dy[T, M]^T . x[T, N] (bf16, unit column stride, 16-B rows)
bool wgrad_bf16_ok(const Tensor& dy, const Tensor& x) {
  if (!dy.is_cuda() || dy.scalar_type() != torch::kBFloat16 || x.scalar_type() != torch::kBFloat16) return false;
  if (dy.dim() != 2 || x.dim() != 2 || dy.size(0) != x.size(0) || dy.size(0) < 1) return false;
  if (dy.stride(1) != 1 || x.stride(1) != 1 || dy.stride(0) % 8 || x.stride(0) % 8) return false;
  if (!aligned16(dy.data_ptr()) || !aligned16(x.data_ptr())) return false;
  return dy.size(1) % 128 == 0 && x.size(1) % 128 == 0 && dy.size(0) < (1LL << 31);
}
Tensor wgrad_bf16(Tensor dy, Tensor x, Tensor out) {
  TORCH_CHECK(wgrad_bf16_ok(dy, x), "wgrad_bf16: unsupported operands (need bf16 [T, M] / [T, N] row-major "
              "with M, N multiples of 128 and 16-byte rows)");
  check_f32(out, "wgrad out");
  const int64_t T = dy.size(0), M = dy.size(1), N = x.size(1);
  // out may hold fewer rows than the (tile-padded) M: rows past out.size(0) are not stored
  TORCH_CHECK(out.size(0) <= M && out.size(0) > 0 && out.size(1) == N && out.is_contiguous(),
              "wgrad out must be [<= M, N]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  int cfg = 0, nsplit = 1;
  hx_wgrad_bf16_plan((int)M, (int)N, (int)T, &cfg, &nsplit);
  Tensor ws;
  if (nsplit > 1) ws = torch::empty({nsplit * M * N}, out.options());
  hx_wgrad_bf16(dy.data_ptr(), (int)dy.stride(0), x.data_ptr(), (int)x.stride(0), out.data_ptr<float>(),
                nsplit > 1 ? ws.data_ptr<float>() : nullptr, (int)M, (int)N, (int)T, cfg, nsplit, (int)out.size(0),
                cur_stream(dy));
  dbg_finite(out, "wgrad_bf16");
  return out;
}

// ------------------------------------------------------------------ fp16x3 GEMMs (gemm_f16.hip)
// fp32 operands travel with max |x| partials (any 1-D fp32 tensor whose max is max |x|): the
// kernels turn them into the power-of-two scale of the fp16 split
inline void check_af32(const Tensor& a, const char* what) {
  check_f32(a, what);
  TORCH_CHECK(a.dim() == 2 && a.stride(1) == 1 && a.stride(0) % 4 == 0 && aligned16(a.data_ptr()) &&
                  a.size(1) % 16 == 0 && a.size(0) < (1LL << 31),
              what, ": fp32 [rows, K] with unit column stride, 16-B aligned rows and K % 16 == 0");
}
// max |x| partials of an fp32 operand: 1-D = partials of the whole tensor (any number; their max
// is a per-tensor bound), 2-D [rows, P] = P partials per operand row (the row's own scale)
struct ScaleSrc {
  const float* p;
  int np, rs;
};
inline ScaleSrc scale_src(const Tensor& t, const Tensor& ref, int64_t rows, const char* what) {
  check_f32(t, what);
  TORCH_CHECK(t.is_contiguous() && t.numel() >= 1 && t.numel() < (1LL << 31) && t.device() == ref.device(), what,
              ": max |x| partials on the operand's device");
  if (t.dim() == 1) return {t.data_ptr<float>(), (int)t.numel(), 0};
  TORCH_CHECK(t.dim() == 2 && t.size(0) == rows && t.size(1) >= 1 && t.size(1) <= 64, what,
              ": per-row max |x| partials must be [rows, P <= 64] (rows = ", rows, ")");
  return {t.data_ptr<float>(), (int)t.size(1), (int)t.size(1)};
}
inline void check_amax(const Tensor& t, const Tensor& ref, const char* what) {
  check_f32(t, what);
  TORCH_CHECK(t.is_contiguous() && t.numel() >= 1 && t.numel() < (1LL << 31) && t.device() == ref.device(), what,
              ": max |x| partials on the operand's device");
}
inline void check_p2(const Tensor& b, int64_t K, const char* what) {
  TORCH_CHECK(b.is_cuda() && b.scalar_type() == torch::kHalf && b.dim() == 2 && b.is_contiguous() &&
                  b.size(1) == 2 * K && aligned16(b.data_ptr()), what, ": fp16 P2 pieces [N, 2K]");
}

// max |x| of every row: [rows, 1]
Tensor amax_rows(Tensor x) {
  check_f32(x, "amax_rows");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 4 == 0 && x.size(1) % 4 == 0 &&
                  aligned16(x.data_ptr()), "amax_rows: fp32 [rows, cols] with 16-B rows, cols % 4 == 0");
  Tensor out = torch::empty({x.size(0), 1}, x.options());
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  hx_amax_rows(x.data_ptr<float>(), x.size(0), (int)x.size(1), x.stride(0), out.data_ptr<float>(), cur_stream(x));
  return out;
}

// fp32 rows [rows, K] -> fp16 P2 pieces [rows, 2K] at each row's scale (the max of its partials
// amax [rows, P]): the pre-split A operand of gemm_f16*
Tensor split_rows_f16(Tensor x, Tensor amax) {
  check_af32(x, "split_rows_f16");
  const ScaleSrc sa = scale_src(amax, x, x.size(0), "split_rows_f16");
  TORCH_CHECK(sa.rs == sa.np, "split_rows_f16: per-row partials [rows, P]");
  Tensor out = torch::empty({x.size(0), 2 * x.size(1)}, x.options().dtype(torch::kHalf));
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  hx_split_rows_f16(x.data_ptr<float>(), x.stride(0), sa.p, sa.np, x.size(0), (int)x.size(1),
                    reinterpret_cast<uint16_t*>(out.data_ptr()), cur_stream(x));
  return out;
}

// [(wf, wt, rmax, cmax)] per weight W [N, K]: P2 fp16 pieces of W (rows scaled by their own
// maxima) and of W^T (rows = columns of W, scaled by the column maxima); rmax [N, 1] / cmax [K, 1]
// are the per-row scale sources of the forward / data-gradient products
// rows: optional padded row count per weight (>= its rows, a multiple of 64): the pieces cover the
// padded rows, read as zero past W's own (the MLM decoder's vocabulary, without a padded copy)
std::vector<std::vector<Tensor>> split_weight_f16(std::vector<Tensor> Ws, std::vector<int64_t> rows) {
  TORCH_CHECK(!Ws.empty() && Ws.size() <= HX_WBATCH, "split_weight_f16: 1..64 weights");
  TORCH_CHECK(rows.empty() || rows.size() == Ws.size(), "split_weight_f16: one padded row count per weight");
  HxWeightBatch d{};
  d.n = (int)Ws.size();
  int64_t rc_floats = 0;
  for (size_t i = 0; i < Ws.size(); ++i) rc_floats += (rows.empty() ? Ws[i].size(0) : rows[i]) + Ws[i].size(1);
  Tensor rc = torch::empty({rc_floats}, Ws[0].options());
  std::vector<std::vector<Tensor>> out;
  int tiles = 0;
  int64_t off = 0;
  for (int i = 0; i < d.n; ++i) {
    const Tensor& W = Ws[i];
    check_f32(W, "split_weight_f16 input");
    const int64_t N = rows.empty() ? W.size(0) : rows[i], K = W.size(1);
    TORCH_CHECK(W.dim() == 2 && W.is_contiguous() && N % 64 == 0 && N >= W.size(0) && W.size(0) >= 1 &&
                    K % 64 == 0 && aligned16(W.data_ptr()) && W.device() == Ws[0].device(),
                "split_weight_f16: every W contiguous [N, K] (N padded to a multiple of 64 >= its rows), K a "
                "multiple of 64, one device");
    auto hf = W.options().dtype(torch::kHalf);
    Tensor wf = torch::empty({N, 2 * K}, hf), wt = torch::empty({K, 2 * N}, hf);
    d.W[i] = W.data_ptr<float>();
    d.wf[i] = reinterpret_cast<uint16_t*>(wf.data_ptr());
    d.wt[i] = reinterpret_cast<uint16_t*>(wt.data_ptr());
    d.N[i] = (int)N;
    d.K[i] = (int)K;
    d.nv[i] = N > W.size(0) ? (int)W.size(0) : 0;
    d.start[i] = tiles;
    d.roff[i] = off;
    tiles += (int)((N / 64) * (K / 64));
    out.push_back({wf, wt, rc.narrow(0, off, N).view({N, 1}), rc.narrow(0, off + N, K).view({K, 1})});
    off += N + K;
  }
  d.start[d.n] = tiles;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(Ws[0].device());
  hx_split_weight_f16(d, rc.data_ptr<float>(), rc_floats, cur_stream(Ws[0]));
  return out;
}

// A is fp32 [M, K], or its fp16 P2 pieces [M, 2K] split at the row scales of aa (split_rows_f16,
// or a fused producer): then the kernel reads them as they are (no split in the k loop)
static HxGemmF16 f16_args(const Tensor& a, const Tensor& aa, const Tensor& b, const Tensor& ba, const char* what) {
  const bool pieces = a.scalar_type() == torch::kHalf;
  if (pieces) {
    TORCH_CHECK(a.is_cuda() && a.dim() == 2 && a.stride(1) == 1 && a.size(1) % 32 == 0 && a.stride(0) % 8 == 0 &&
                    aligned16(a.data_ptr()) && a.size(0) < (1LL << 31) && aa.dim() == 2,
                what, ": fp16 A pieces [M, 2K] (K % 16 == 0, 16-B rows) with per-row max |x| partials");
  } else {
    check_af32(a, what);
  }
  const int64_t K = pieces ? a.size(1) / 2 : a.size(1);
  check_p2(b, K, what);
  TORCH_CHECK(b.device() == a.device() && b.size(0) < (1LL << 31), what, ": operands on one device");
  const ScaleSrc sa = scale_src(aa, b, a.size(0), what), sb = scale_src(ba, b, b.size(0), what);
  HxGemmF16 p{};
  p.A = a.data_ptr();
  p.lda = pieces ? a.stride(0) / 2 : a.stride(0);
  p.apieces = pieces ? 1 : 0;
  p.a_amax = sa.p;
  p.na = sa.np;
  p.a_rs = sa.rs;
  p.B = reinterpret_cast<const uint16_t*>(b.data_ptr());
  p.ldb = b.size(1);
  p.b_amax = sb.p;
  p.nb = sb.np;
  p.b_rs = sb.rs;
  p.M = (int)a.size(0);
  p.N = (int)b.size(0);
  p.K = (int)K;
  p.ks = 1;
  return p;
}
inline void check_vec(const OptT& v, int64_t n, const char* what) {
  if (!has(v)) return;
  check_f32(*v, what);
  TORCH_CHECK(v->numel() == n && v->is_contiguous() && aligned16(v->data_ptr()), what, ": fp32 [N], 16-B aligned");
}

// C (+)= a . b^T (+ bias); ks split-K slabs (0 = plan: deep reductions with few output tiles),
// combined (with the beta / bias epilogue) by one pass over the slabs
Tensor gemm_f16(Tensor a, Tensor a_amax, Tensor b, Tensor b_amax, OptT out_, bool beta, OptT bias, int64_t ks) {
  HxGemmF16 p = f16_args(a, a_amax, b, b_amax, "gemm_f16");
  check_vec(bias, p.N, "gemm_f16 bias");
  const int cfg = hx_gemm_f16_plan(p.M, p.N, p.K);
  TORCH_CHECK(cfg >= 0, "gemm_f16: no tile for N = ", p.N);
  TORCH_CHECK(!beta || has(out_), "gemm_f16: beta needs an output to accumulate into");
  if (ks <= 0) ks = hx_gemm_f16_ks(p.M, p.N, p.K, cfg);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  auto f32 = a.options().dtype(torch::kFloat32);
  Tensor out = has(out_) ? *out_ : torch::empty({p.M, p.N}, f32);
  TORCH_CHECK(out.scalar_type() == torch::kFloat32 && out.dim() == 2 && out.size(0) == p.M && out.size(1) == p.N &&
                  out.stride(1) == 1 && out.stride(0) % 4 == 0 && aligned16(out.data_ptr()),
              "gemm_f16: out must be fp32 [M, N] with unit column stride and 16-B rows");
  if (ks > 1) {
    Tensor part = torch::empty({ks, p.M, p.N}, f32);
    p.C = part.data_ptr<float>();
    p.ldc = p.N;
    p.ks = (int)ks;
    p.c_zs = (int64_t)p.M * p.N;
    TORCH_CHECK(hx_gemm_f16(p, cfg, cur_stream(a)) == 0, "gemm_f16: split-K launch failed (ks must divide K / 16)");
    hx_gemm_f16_slab_combine(part.data_ptr<float>(), out.data_ptr<float>(), out.stride(0), p.M, p.N, (int)ks,
                             beta ? 1 : 0, ptr_or_null<float>(bias), cur_stream(a));
    dbg_finite(out, "gemm_f16");
    return out;
  }
  p.C = out.data_ptr<float>();
  p.ldc = out.stride(0);
  p.beta = beta ? 1 : 0;
  p.bias = ptr_or_null<float>(bias);
  TORCH_CHECK(hx_gemm_f16(p, cfg, cur_stream(a)) == 0, "gemm_f16: launch failed");
  dbg_finite(out, "gemm_f16");
  return out;
}

// FFN up: u = a . b^T + bias -> (gelu'(u) if dmode else u, h = gelu(u) fp32, max |h| per (row, N
// tile) [M, TN] -- h's per-row scale source for the FFN-down GEMM --, max |h| per (M tile, column)
// [TM, N] -- h's column maxima for the FFN-down weight gradient)
std::vector<Tensor> gemm_f16_gelu(Tensor a, Tensor a_amax, Tensor b, Tensor b_amax, OptT bias, int64_t dmode) {
  HxGemmF16 p = f16_args(a, a_amax, b, b_amax, "gemm_f16_gelu");
  check_vec(bias, p.N, "gemm_f16_gelu bias");
  const int cfg = hx_gemm_f16_plan(p.M, p.N, p.K);
  TORCH_CHECK(cfg >= 0, "gemm_f16_gelu: no tile for N = ", p.N);
  auto f32 = a.options().dtype(torch::kFloat32);
  Tensor c = torch::empty({p.M, p.N}, f32), h = torch::empty({p.M, p.N}, f32);
  Tensor rm = torch::empty({p.M, hx_gemm_f16_tn(p.N, cfg)}, f32), cm = torch::empty({hx_gemm_f16_tm(p.M, cfg), p.N}, f32);
  p.kind = 1;
  p.C = c.data_ptr<float>();
  p.ldc = p.N;
  p.bias = ptr_or_null<float>(bias);
  p.P = h.data_ptr<float>();
  p.ldp = p.N;
  p.rowmax = rm.data_ptr<float>();
  p.colmax = cm.data_ptr<float>();
  p.dmode = dmode ? 1 : 0;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  TORCH_CHECK(hx_gemm_f16(p, cfg, cur_stream(a)) == 0, "gemm_f16_gelu: launch failed");
  dbg_finite(h, "gemm_f16_gelu");
  return {c, h, rm, cm};
}

// FFN down data gradient + GELU backward: t = (a . b^T) * (dmode ? u : gelu'(u + bias)) ->
// (t fp32, max |t| per (row, N tile) [M, TN], max |t| per (M tile, column) [TM, N], dbias =
// column sums of t (into dbias_out when given))
std::vector<Tensor> gemm_f16_dgelu(Tensor a, Tensor a_amax, Tensor b, Tensor b_amax, Tensor u, OptT bias,
                                   OptT dbias_out, int64_t dmode) {
  TORCH_CHECK(!dmode || !has(bias), "gemm_f16_dgelu: dmode 1 takes gelu'(u), which has the bias in it");
  HxGemmF16 p = f16_args(a, a_amax, b, b_amax, "gemm_f16_dgelu");
  check_vec(bias, p.N, "gemm_f16_dgelu bias");
  check_f32(u, "gemm_f16_dgelu u");
  TORCH_CHECK(u.dim() == 2 && u.size(0) == p.M && u.size(1) == p.N && u.is_contiguous() && aligned16(u.data_ptr()),
              "gemm_f16_dgelu: u must be fp32 [M, N]");
  const int cfg = hx_gemm_f16_plan(p.M, p.N, p.K);
  TORCH_CHECK(cfg >= 0, "gemm_f16_dgelu: no tile for N = ", p.N);
  const int prow = hx_gemm_f16_colpart_rows(p.M, cfg);
  auto f32 = a.options().dtype(torch::kFloat32);
  Tensor t = torch::empty({p.M, p.N}, f32);
  Tensor rm = torch::empty({p.M, hx_gemm_f16_tn(p.N, cfg)}, f32), cm = torch::empty({hx_gemm_f16_tm(p.M, cfg), p.N}, f32);
  Tensor part = torch::empty({prow, p.N}, f32);
  Tensor db = has(dbias_out) ? *dbias_out : torch::empty({p.N}, f32);
  TORCH_CHECK(db.numel() == p.N && db.scalar_type() == torch::kFloat32 && db.is_contiguous(), "gemm_f16_dgelu: dbias");
  p.kind = 2;
  p.bias = ptr_or_null<float>(bias);
  p.aux = u.data_ptr<float>();
  p.ldaux = p.N;
  p.P = t.data_ptr<float>();
  p.ldp = p.N;
  p.colpart = part.data_ptr<float>();
  p.rowmax = rm.data_ptr<float>();
  p.colmax = cm.data_ptr<float>();
  p.dmode = dmode ? 1 : 0;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  TORCH_CHECK(hx_gemm_f16(p, cfg, cur_stream(a)) == 0, "gemm_f16_dgelu: launch failed");
  hx_fold_cols(part.data_ptr<float>(), prow, p.N, db.data_ptr<float>(), 0, cur_stream(a));
  dbg_finite(t, "gemm_f16_dgelu");
  return {t, rm, cm, db};
}

// the per-column scale source of a weight-gradient operand: 1-D = partials of the whole tensor (a
// per-tensor bound), 2-D [P, cols] = P partials per column; with aff = (gamma, beta) the
// LayerNorm-output bound (|gamma| z + |beta|) mul instead (t unused)
inline HxColScale col_scale_src(const Tensor& t, const Tensor& ref, int64_t cols, const char* what, const OptT& g,
                                const OptT& b, double z, double mul) {
  HxColScale c{};
  if (has(g)) {
    TORCH_CHECK(has(b), what, ": the affine bound needs gamma and beta");
    check_f32(*g, what);
    check_f32(*b, what);
    TORCH_CHECK(g->numel() == cols && b->numel() == cols && g->is_contiguous() && b->is_contiguous() &&
                    g->device() == ref.device() && b->device() == ref.device(), what, ": gamma / beta [cols]");
    c.g = g->data_ptr<float>();
    c.b = b->data_ptr<float>();
    c.z = (float)z;
    c.mul = (float)mul;
    return c;
  }
  check_f32(t, what);
  TORCH_CHECK(t.is_contiguous() && t.numel() >= 1 && t.numel() < (1LL << 31) && t.device() == ref.device(), what,
              ": max |x| partials on the operand's device");
  c.p = t.data_ptr<float>();
  if (t.dim() == 1) {
    c.np = (int)t.numel();
    return c;
  }
  TORCH_CHECK(t.dim() == 2 && t.size(1) == cols && t.size(0) >= 1 && t.size(0) <= 256, what,
              ": per-column max |x| partials must be [P <= 256, cols] (cols = ", cols, ")");
  c.np = (int)t.size(0);
  c.cs = (int)cols;
  return c;
}

// max |x| of every row and every column in one read: ([rows, 1], [1, cols]); cols <= 4096
std::vector<Tensor> amax_rows_cols(Tensor x) {
  // rows may be strided (the dQ third of a [rows, 3H] gradient)
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kFloat32, "amax_rows_cols: fp32 GPU tensor");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 4 == 0 && x.size(1) % 4 == 0 &&
                  x.size(1) <= 4096 && aligned16(x.data_ptr()),
              "amax_rows_cols: fp32 [rows, cols <= 4096] with 16-B rows, cols % 4 == 0");
  Tensor r = torch::empty({x.size(0), 1}, x.options());
  Tensor c = torch::empty({1, x.size(1)}, x.options());
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(hx_amax_rows_cols(x.data_ptr<float>(), x.size(0), (int)x.size(1), x.stride(0), r.data_ptr<float>(),
                                c.data_ptr<float>(), cur_stream(x)) == 0, "amax_rows_cols: launch");
  return {r, c};
}

// max |x| of every column: [1, cols]
Tensor amax_cols(Tensor x) {
  check_f32(x, "amax_cols");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 4 == 0 && x.size(1) % 4 == 0 &&
                  aligned16(x.data_ptr()), "amax_cols: fp32 [rows, cols] with 16-B rows, cols % 4 == 0");
  Tensor out = torch::empty({1, x.size(1)}, x.options());
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  hx_amax_cols(x.data_ptr<float>(), x.size(0), (int)x.size(1), x.stride(0), out.data_ptr<float>(), cur_stream(x));
  return out;
}

// dW = dy^T x over the token rows: dy [T, M], x [T, N] fp32 (M, N multiples of 128); out [<= M, N]
// (rows of dy's padding columns past out.size(0) are not stored); dy_amax / x_amax: per-column
// max |x| partials of each operand ([P, M] / [P, N]) or per-tensor partials (1-D)
Tensor wgrad_f16(Tensor dy, Tensor dy_amax, Tensor x, Tensor x_amax, Tensor out, OptT x_gamma, OptT x_beta, double x_z,
                 double x_mul) {
  check_f32(dy, "wgrad_f16 dy");
  check_f32(x, "wgrad_f16 x");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0) && dy.stride(1) == 1 && x.stride(1) == 1 &&
                  dy.stride(0) % 4 == 0 && x.stride(0) % 4 == 0 && aligned16(dy.data_ptr()) &&
                  aligned16(x.data_ptr()) && dy.size(1) % 128 == 0 && x.size(1) % 128 == 0 &&
                  dy.size(0) < (1 << 30) && x.device() == dy.device(),
              "wgrad_f16: dy [T, M], x [T, N] fp32 with 16-B rows, M and N multiples of 128");
  const int64_t T = dy.size(0), M = dy.size(1), N = x.size(1);
  const HxColScale sa = col_scale_src(dy_amax, dy, M, "wgrad_f16 dy partials", OptT(), OptT(), 0, 0);
  const HxColScale sb = col_scale_src(x_amax, dy, N, "wgrad_f16 x partials", x_gamma, x_beta, x_z, x_mul);
  check_f32(out, "wgrad_f16 out");
  TORCH_CHECK(out.dim() == 2 && out.size(0) <= M && out.size(1) == N && out.is_contiguous(),
              "wgrad_f16: out must be contiguous fp32 [<= M, N]");
  int cfg = 0, nsplit = 1;
  hx_wgrad_f16_plan((int)M, (int)N, (int)T, &cfg, &nsplit);
  Tensor ws;
  if (nsplit > 1) ws = torch::empty({nsplit, M, N}, dy.options());
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  TORCH_CHECK(hx_wgrad_f16(dy.data_ptr<float>(), (int)dy.stride(0), sa, x.data_ptr<float>(), (int)x.stride(0), sb,
                           out.data_ptr<float>(), nsplit > 1 ? ws.data_ptr<float>() : nullptr, (int)M, (int)N, (int)T,
                           cfg, nsplit, (int)out.size(0), cur_stream(dy)) == 0,
              "wgrad_f16: launch failed");
  dbg_finite(out, "wgrad_f16");
  return out;
}

// --precision bf16 on the same kernel: out (+)= a . b^T (+ bias), a bf16 [M, K], b bf16 [N, K]
// (contiguous); the output is bf16 (out_bf16) or fp32
Tensor gemm_bf16(Tensor a, Tensor b, OptT out_, bool beta, OptT bias, bool out_bf16) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16 &&
                  a.dim() == 2 && b.dim() == 2 && a.stride(1) == 1 && a.stride(0) % 8 == 0 &&
                  aligned16(a.data_ptr()) && b.is_contiguous() && aligned16(b.data_ptr()) && a.size(1) == b.size(1) &&
                  a.size(1) % 32 == 0 && a.device() == b.device(),
              "gemm_bf16: a [M, K] / b [N, K] bf16 with 16-B rows, K % 32 == 0");
  HxGemmF16 p{};
  p.A = a.data_ptr();
  p.lda = a.stride(0);
  p.B = reinterpret_cast<const uint16_t*>(b.data_ptr());
  p.ldb = b.size(1);
  p.M = (int)a.size(0);
  p.N = (int)b.size(0);
  p.K = (int)a.size(1);
  p.ks = 1;
  p.abf16 = 1;
  p.obf16 = out_bf16 ? 1 : 0;
  check_vec(bias, p.N, "gemm_bf16 bias");
  const int cfg = hx_gemm_bf16_plan(p.M, p.N, p.K);
  TORCH_CHECK(cfg >= 0, "gemm_bf16: no tile for N = ", p.N);
  TORCH_CHECK(!beta || has(out_), "gemm_bf16: beta needs an output to accumulate into");
  Tensor out = has(out_) ? *out_ : torch::empty({p.M, p.N}, a.options().dtype(out_bf16 ? torch::kBFloat16
                                                                                       : torch::kFloat32));
  TORCH_CHECK(out.scalar_type() == (out_bf16 ? torch::kBFloat16 : torch::kFloat32) && out.dim() == 2 &&
                  out.size(0) == p.M && out.size(1) == p.N && out.stride(1) == 1 && out.stride(0) % 8 == 0 &&
                  aligned16(out.data_ptr()),
              "gemm_bf16: out [M, N] of the output dtype with 16-B rows");
  p.C = reinterpret_cast<float*>(out.data_ptr());
  p.ldc = out.stride(0);
  p.beta = beta ? 1 : 0;
  p.bias = ptr_or_null<float>(bias);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  TORCH_CHECK(hx_gemm_f16(p, cfg, cur_stream(a)) == 0, "gemm_bf16: launch failed");
  dbg_finite(out, "gemm_bf16");
  return out;
}

static HxGemmF16 bf16_args(const Tensor& a, const Tensor& b, const char* what) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16 &&
                  a.dim() == 2 && b.dim() == 2 && a.stride(1) == 1 && a.stride(0) % 8 == 0 &&
                  aligned16(a.data_ptr()) && b.is_contiguous() && aligned16(b.data_ptr()) && a.size(1) == b.size(1) &&
                  a.size(1) % 32 == 0 && a.device() == b.device(),
              what, ": a [M, K] / b [N, K] bf16 with 16-B rows, K % 32 == 0");
  HxGemmF16 p{};
  p.A = a.data_ptr();
  p.lda = a.stride(0);
  p.B = reinterpret_cast<const uint16_t*>(b.data_ptr());
  p.ldb = b.size(1);
  p.M = (int)a.size(0);
  p.N = (int)b.size(0);
  p.K = (int)a.size(1);
  p.ks = 1;
  p.abf16 = 1;
  p.obf16 = 1;
  return p;
}

// --precision bf16 FFN up: u = a . b^T + bias -> (gelu'(u), gelu(u)), both bf16 [M, N]
std::vector<Tensor> gemm_bf16_gelu(Tensor a, Tensor b, Tensor bias) {
  HxGemmF16 p = bf16_args(a, b, "gemm_bf16_gelu");
  check_vec(bias, p.N, "gemm_bf16_gelu bias");
  const int cfg = hx_gemm_bf16_plan(p.M, p.N, p.K);
  TORCH_CHECK(cfg >= 0, "gemm_bf16_gelu: no tile for N = ", p.N);
  Tensor d = torch::empty({p.M, p.N}, a.options()), h = torch::empty({p.M, p.N}, a.options());
  p.kind = 1;
  p.C = reinterpret_cast<float*>(d.data_ptr());
  p.ldc = p.N;
  p.bias = bias.data_ptr<float>();
  p.P = reinterpret_cast<float*>(h.data_ptr());
  p.ldp = p.N;
  p.dmode = 1;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  TORCH_CHECK(hx_gemm_f16(p, cfg, cur_stream(a)) == 0, "gemm_bf16_gelu: launch failed");
  dbg_finite(h, "gemm_bf16_gelu");
  return {d, h};
}

// --precision bf16 FFN-down data gradient + GELU backward: t = (a . b^T) * (dmode ? d : gelu'(d + bias))
// (d: bf16 gelu'(u) from gemm_bf16_gelu, or the pre-bias u) -> (t bf16, dbias = column sums of t
// into dbias_out when given)
std::vector<Tensor> gemm_bf16_dgelu(Tensor a, Tensor b, Tensor d, OptT dbias_out, OptT bias, int64_t dmode) {
  TORCH_CHECK(!dmode || !has(bias), "gemm_bf16_dgelu: dmode 1 takes gelu'(u), which has the bias in it");
  HxGemmF16 p = bf16_args(a, b, "gemm_bf16_dgelu");
  check_vec(bias, p.N, "gemm_bf16_dgelu bias");
  TORCH_CHECK(d.scalar_type() == torch::kBFloat16 && d.dim() == 2 && d.size(0) == p.M && d.size(1) == p.N &&
                  d.is_contiguous() && aligned16(d.data_ptr()) && d.device() == a.device(),
              "gemm_bf16_dgelu: d must be bf16 [M, N]");
  const int cfg = hx_gemm_bf16_plan(p.M, p.N, p.K);
  TORCH_CHECK(cfg >= 0, "gemm_bf16_dgelu: no tile for N = ", p.N);
  const int prow = hx_gemm_f16_colpart_rows(p.M, cfg);
  auto f32 = a.options().dtype(torch::kFloat32);
  Tensor t = torch::empty({p.M, p.N}, a.options());
  Tensor part = torch::empty({prow, p.N}, f32);
  Tensor db = has(dbias_out) ? *dbias_out : torch::empty({p.N}, f32);
  TORCH_CHECK(db.numel() == p.N && db.scalar_type() == torch::kFloat32 && db.is_contiguous() && db.device() == a.device(),
              "gemm_bf16_dgelu: dbias");
  p.kind = 2;
  p.bias = ptr_or_null<float>(bias);
  p.aux = reinterpret_cast<const float*>(d.data_ptr());
  p.ldaux = p.N;
  p.P = reinterpret_cast<float*>(t.data_ptr());
  p.ldp = p.N;
  p.colpart = part.data_ptr<float>();
  p.dmode = dmode ? 1 : 0;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  TORCH_CHECK(hx_gemm_f16(p, cfg, cur_stream(a)) == 0, "gemm_bf16_dgelu: launch failed");
  hx_fold_cols(part.data_ptr<float>(), prow, p.N, db.data_ptr<float>(), 0, cur_stream(a));
  dbg_finite(t, "gemm_bf16_dgelu");
  return {t, db};
}

// W^T in bf16 ([K, N]) of every fp32 weight W [N, K] in the list, one launch
std::vector<Tensor> weight_bf16_t(std::vector<Tensor> Ws) {
  TORCH_CHECK(!Ws.empty() && Ws.size() <= HX_WBATCH, "weight_bf16_t: 1..64 weights");
  HxWeightBatch d{};
  d.n = (int)Ws.size();
  std::vector<Tensor> out;
  int tiles = 0;
  for (int i = 0; i < d.n; ++i) {
    const Tensor& W = Ws[i];
    check_f32(W, "weight_bf16_t input");
    TORCH_CHECK(W.dim() == 2 && W.is_contiguous() && W.size(0) % 64 == 0 && W.size(1) % 64 == 0 &&
                    aligned16(W.data_ptr()) && W.device() == Ws[0].device(),
                "weight_bf16_t: every W contiguous [N, K], N and K multiples of 64, one device");
    Tensor wt = torch::empty({W.size(1), W.size(0)}, W.options().dtype(torch::kBFloat16));
    d.W[i] = W.data_ptr<float>();
    d.wt[i] = reinterpret_cast<uint16_t*>(wt.data_ptr());
    d.wf[i] = nullptr;
    d.N[i] = (int)W.size(0);
    d.K[i] = (int)W.size(1);
    d.start[i] = tiles;
    tiles += (int)((W.size(0) / 64) * (W.size(1) / 64));
    out.push_back(wt);
  }
  d.start[d.n] = tiles;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(Ws[0].device());
  hx_weight_bf16_t(d, cur_stream(Ws[0]));
  return out;
}

// ------------------------------------------------------------------ xGMI all-reduce
// Contexts travel to Python as integers (owned by parallel/xgmi.py).
inline void xar_check(int rc) { TORCH_CHECK(rc == 0, hx_xar_last_error()); }
inline void* as_ctx(int64_t h) { return reinterpret_cast<void*>(static_cast<uintptr_t>(h)); }
int64_t xar_create(int64_t rank, int64_t world, int64_t nblocks, double timeout_s, int64_t oneshot_max_bytes) {
  void* c = nullptr;
  xar_check(hx_xar_create((int)rank, (int)world, (int)nblocks, timeout_s, oneshot_max_bytes, &c));
  return static_cast<int64_t>(reinterpret_cast<uintptr_t>(c));
}
void xar_register(int64_t h, Tensor buf) {
  check_f32(buf, "xGMI registered buffer");
  TORCH_CHECK(buf.is_contiguous() && aligned16(buf.data_ptr()), "xGMI registered buffer: contiguous, 16-B aligned");
  xar_check(hx_xar_register(as_ctx(h), buf.data_ptr<float>(), buf.numel()));
}
py::bytes xar_export(int64_t h) {
  char buf[kXarRecord];
  xar_check(hx_xar_export(as_ctx(h), buf));
  return py::bytes(buf, kXarRecord);
}
void xar_open(int64_t h, py::bytes recs) {
  const std::string s = recs;
  xar_check(hx_xar_open(as_ctx(h), s.data()));
}
void xar_allreduce(int64_t h, Tensor buf) {
  check_f32(buf, "all-reduce bucket");
  TORCH_CHECK(aligned16(buf.data_ptr()), "all-reduce bucket must be 16-byte aligned");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(buf.device());
  xar_check(hx_xar_allreduce(as_ctx(h), buf.data_ptr<float>(), buf.numel(), cur_stream(buf)));
}
void xar_allreduce_sim(std::vector<int64_t> hs, std::vector<Tensor> bufs, int64_t mute) {
  TORCH_CHECK(hs.size() == bufs.size() && hs.size() >= 2 && hs.size() <= 8, "1 context per simulated rank (2..8)");
  std::vector<void*> cs;
  std::vector<float*> ps;
  for (size_t i = 0; i < hs.size(); ++i) {
    check_f32(bufs[i], "bucket");
    TORCH_CHECK(bufs[i].numel() == bufs[0].numel() && aligned16(bufs[i].data_ptr()), "equal, aligned buckets");
    cs.push_back(as_ctx(hs[i]));
    ps.push_back(bufs[i].data_ptr<float>());
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(bufs[0].device());
  TORCH_CHECK(mute >= -1 && mute < (int64_t)hs.size(), "mute must be -1 or a simulated rank");
  xar_check(hx_xar_allreduce_sim(cs.data(), ps.data(), (int)hs.size(), bufs[0].numel(), (int)mute,
                                 cur_stream(bufs[0])));
}
int64_t xar_error(int64_t h) { return hx_xar_error(as_ctx(h)); }
void xar_error_async(int64_t h, Tensor out) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kInt && out.numel() >= 1 && out.is_contiguous(),
              "error word target: contiguous int32 GPU tensor");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(out.device());
  xar_check(hx_xar_error_async(as_ctx(h), out.data_ptr<int32_t>(), cur_stream(out)));
}
// PCI bus id ("dddd:bb:dd.f") of a device visible to this process: the process-independent
// identity of a GPU (local ordinals differ between processes with different visible sets)
std::string device_pci_bus_id(int64_t dev) {
  char id[64] = {0};
  TORCH_CHECK(hipDeviceGetPCIBusId(id, (int)sizeof(id), (int)dev) == hipSuccess, "hipDeviceGetPCIBusId failed");
  return std::string(id);
}
int64_t xar_oneshot_max(int64_t h) { return hx_xar_oneshot_max(as_ctx(h)); }
void xar_destroy(int64_t h) { hx_xar_destroy(as_ctx(h)); }

}  // namespace

namespace hx {
void register_reducer(py::module& m);   // csrc/native/reducer.cpp
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  hx::register_reducer(m);
  m.doc() = "hetseq_9cme_amd gfx950 (MI355X) kernels";
  m.def("grad_norm_clip", &grad_norm_clip);
  m.def("adam", &adam);
  m.def("adam_masked", &adam_masked, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("shadow"),
        py::arg("gscale"), py::arg("table"), py::arg("used"), py::arg("steps"), py::arg("hp"), py::arg("lr"),
        py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("lr_dev") = py::none());
  m.def("adam_mask_chunk", &hx_adam_mask_chunk);
  m.def("adadelta", &adadelta);
  m.def("ln_fwd", &ln_fwd, py::arg("y"), py::arg("bias"), py::arg("res"), py::arg("gamma"), py::arg("beta"),
        py::arg("eps"), py::arg("keep_prob"), py::arg("seed"), py::arg("stream"), py::arg("drop_after"),
        py::arg("save_z"), py::arg("amax_out") = py::none(), py::arg("pieces_out") = py::none());
  m.def("ln_bwd", &ln_bwd, py::arg("dout"), py::arg("z"), py::arg("mean"), py::arg("rstd"), py::arg("gamma"),
        py::arg("keep_prob"), py::arg("seed"), py::arg("stream"), py::arg("drop_after"), py::arg("want_dy"),
        py::arg("want_dbias"), py::arg("dgamma_out"), py::arg("dbeta_out"), py::arg("dbias_out"),
        py::arg("amax_out") = py::none(), py::arg("colmax_out") = py::none(), py::arg("pieces_out") = py::none());
  m.def("ln_fwd_blocks", &hx_ln_fwd_blocks);
  m.def("ln_bwd_blocks", &hx_ln_bwd_blocks);
  m.def("embed_ln_fwd", &embed_ln_fwd, py::arg("ids"), py::arg("tt"), py::arg("wte"), py::arg("wpe"), py::arg("wtt"),
        py::arg("gamma"), py::arg("beta"), py::arg("eps"), py::arg("keep_prob"), py::arg("seed"), py::arg("stream"),
        py::arg("bf16_out"), py::arg("amax_out") = py::none(), py::arg("pieces_out") = py::none());
  m.def("embed_word_grad", &embed_word_grad);
  m.def("embed_type_grad", &embed_type_grad);
  m.def("bias_act_fwd", &bias_act_fwd);
  m.def("bias_act_bwd", &bias_act_bwd);
  m.def("colsum", &colsum);
  m.def("dropout", &dropout);
  m.def("softmax_xent_", &softmax_xent_);
  m.def("attn_fwd", [](Tensor qkv, Tensor mask_bias, int64_t nh, double keep, const Tensor& seed, int64_t stream,
                        OptT bias) { return attn_fwd(qkv, mask_bias, nh, keep, seed, stream, bias, false); });
  m.def("attn_fwd_f16", &attn_fwd_f16, py::arg("qkv"), py::arg("mask_bias"), py::arg("nh"), py::arg("keep"),
        py::arg("seed"), py::arg("stream"), py::arg("bias"), py::arg("amax_out") = py::none(),
        py::arg("colmax_out") = py::none());
  m.def("attn_bwd", [](Tensor dout, Tensor qkv, Tensor mask_bias, Tensor out, Tensor lse, Tensor dmask, int64_t nh,
                       double keep, OptT bias, OptT dbq, OptT dbk, OptT dbv, bool want_dbias) {
    return attn_bwd(dout, qkv, mask_bias, out, lse, dmask, nh, keep, bias, dbq, dbk, dbv, 0, OptT(), OptT(), want_dbias);
  }, py::arg("dout"), py::arg("qkv"), py::arg("mask_bias"), py::arg("out"), py::arg("lse"), py::arg("dmask"),
     py::arg("nh"), py::arg("keep"), py::arg("bias"), py::arg("dbq"), py::arg("dbk"), py::arg("dbv"),
     py::arg("want_dbias") = false);
  // fp32 attention backward on the fp16 matrix cores (fp16x3, attention_f16.hip)
  m.def("attn_bwd_f16", [](Tensor dout, Tensor qkv, Tensor mask_bias, Tensor out, Tensor lse, Tensor dmask, int64_t nh,
                           double keep, OptT bias, OptT dbq, OptT dbk, OptT dbv, OptT amax_out, OptT colmax_out,
                           bool want_dbias) {
    return attn_bwd(dout, qkv, mask_bias, out, lse, dmask, nh, keep, bias, dbq, dbk, dbv, 2, amax_out, colmax_out,
                    want_dbias);
  }, py::arg("dout"), py::arg("qkv"), py::arg("mask_bias"), py::arg("out"), py::arg("lse"), py::arg("dmask"),
     py::arg("nh"), py::arg("keep"), py::arg("bias"), py::arg("dbq"), py::arg("dbk"), py::arg("dbv"),
     py::arg("amax_out") = py::none(), py::arg("colmax_out") = py::none(), py::arg("want_dbias") = false);
  m.def("wgrad_bf16", &wgrad_bf16);
  m.def("wgrad_bf16_ok", &wgrad_bf16_ok);
  m.def("amax_rows", &amax_rows);
  m.def("split_rows_f16", &split_rows_f16);
  m.def("amax_cols", &amax_cols);
  m.def("amax_rows_cols", &amax_rows_cols);
  m.def("split_weight_f16", &split_weight_f16, py::arg("Ws"), py::arg("rows") = std::vector<int64_t>());
  m.def("gemm_f16", &gemm_f16, py::arg("a"), py::arg("a_amax"), py::arg("b"), py::arg("b_amax"),
        py::arg("out") = py::none(), py::arg("beta") = false, py::arg("bias") = py::none(), py::arg("ks") = 0);
  m.def("gemm_f16_gelu", &gemm_f16_gelu, py::arg("a"), py::arg("a_amax"), py::arg("b"), py::arg("b_amax"),
        py::arg("bias"), py::arg("dmode") = 1);
  m.def("gemm_f16_dgelu", &gemm_f16_dgelu, py::arg("a"), py::arg("a_amax"), py::arg("b"), py::arg("b_amax"),
        py::arg("u"), py::arg("bias") = py::none(), py::arg("dbias_out") = py::none(), py::arg("dmode") = 1);
  m.def("wgrad_f16", &wgrad_f16, py::arg("dy"), py::arg("dy_amax"), py::arg("x"), py::arg("x_amax"), py::arg("out"),
        py::arg("x_gamma") = py::none(), py::arg("x_beta") = py::none(), py::arg("x_z") = 0.0,
        py::arg("x_mul") = 1.0);
  m.def("gemm_bf16_gelu", &gemm_bf16_gelu, py::arg("a"), py::arg("b"), py::arg("bias"));
  m.def("gemm_bf16_dgelu", &gemm_bf16_dgelu, py::arg("a"), py::arg("b"), py::arg("d"),
        py::arg("dbias_out") = py::none(), py::arg("bias") = py::none(), py::arg("dmode") = 1);
  m.def("gemm_bf16", &gemm_bf16, py::arg("a"), py::arg("b"), py::arg("out") = py::none(), py::arg("beta") = false,
        py::arg("bias") = py::none(), py::arg("out_bf16") = true);
  m.def("weight_bf16_t", &weight_bf16_t);

  m.def("gemm_f16_plan", &hx_gemm_f16_plan);
  m.def("gemm_f16_ks", &hx_gemm_f16_ks);
  m.def("gemm_f16_tiles", &hx_gemm_f16_tiles);
  m.def("wgrad_f16_plan", [](int64_t M, int64_t N, int64_t T) {
    int c = 0, s = 1;
    hx_wgrad_f16_plan((int)M, (int)N, (int)T, &c, &s);
    return std::make_tuple(c, s);
  });

  m.def("xar_create", &xar_create);
  m.def("xar_register", &xar_register);
  m.def("device_pci_bus_id", &device_pci_bus_id);
  m.def("xar_export", &xar_export);
  m.def("xar_open", &xar_open);
  m.def("xar_allreduce", &xar_allreduce);
  m.def("xar_allreduce_sim", &xar_allreduce_sim);
  m.def("xar_error", &xar_error);
  m.def("xar_error_async", &xar_error_async);
  m.def("xar_oneshot_max", &xar_oneshot_max);
  m.def("xar_destroy", &xar_destroy);
  m.def("set_debug", &set_debug);
  m.def("get_debug", &get_debug);
  // CUs reserved for a concurrent comm kernel (cu_reserve.hip)
  m.def("num_cus", &hx_num_cus);
  m.def("set_reserved_cus", &hx_set_reserved_cus);
  m.def("reserved_cus", &hx_reserved_cus);
  m.def("cu_slots", &hx_cu_slots);
  m.def("cu_masked_stream", [](int64_t first_cu, int64_t count) {
    hipStream_t st = hx_cu_masked_stream((int)first_cu, (int)count);
    TORCH_CHECK(st != nullptr, "hipExtStreamCreateWithCUMask failed");
    return (int64_t)(uintptr_t)st;
  });
  m.def("priority_stream", [](int64_t prio) {
    hipStream_t st = hx_priority_stream((int)prio);
    TORCH_CHECK(st != nullptr, "hipStreamCreateWithPriority failed");
    return (int64_t)(uintptr_t)st;
  });
  m.def("stream_priority_range", []() {
    int least = 0, greatest = 0;
    hx_stream_priority_range(&least, &greatest);
    return std::vector<int64_t>{least, greatest};
  });
  m.def("destroy_stream", [](int64_t h) { hx_destroy_stream(reinterpret_cast<hipStream_t>((uintptr_t)h)); });
  m.def("spin", [](int64_t blocks, double us, int64_t lds_bytes, Tensor sink, int64_t stream) {
    TORCH_CHECK(sink.is_cuda() && sink.scalar_type() == torch::kInt32 && sink.numel() >= 256, "spin: int32 sink[256]");
    TORCH_CHECK(lds_bytes >= 0 && lds_bytes <= 160 * 1024 && us >= 0 && us < 1e7, "spin: bad arguments");
    hipStream_t st = stream ? reinterpret_cast<hipStream_t>((uintptr_t)stream) : cur_stream(sink);
    hx_spin((int)blocks, us, (int)lds_bytes, reinterpret_cast<uint32_t*>(sink.data_ptr<int>()), st);
  });
}
