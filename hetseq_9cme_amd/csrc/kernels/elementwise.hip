// Bias + activation epilogues, dropout and column reductions.
//
// Reference: TorchScript-fused ``bias_gelu`` / ``bias_tanh`` (bert_modeling.py:104-116,
// used by LinearActivation :166-168) plus autograd's separate bias-grad reductions.
// Here:
//   * bias_act_fwd : out = act(y + b) in one streaming pass (float4, 16 B / lane)
//   * bias_act_bwd : dy = dout * act'(.) AND the per-row-chunk column partials of dy
//                    (-> dbias) in the same pass; a tiny second kernel folds them.
//                    GELU backward recomputes act' from y (nothing extra stored);
//                    tanh backward uses the saved output (1 - out^2).
//   * dropout fwd/bwd with the Philox stream (mask regenerated, never stored)
//   * colsum      : generic [rows, N] -> [N] column sum (bias grads of plain linears)
#include <stdlib.h>

#include "hx_launch.h"
#include "hx_vec.h"
#include "hx_reduce.h"

namespace {

constexpr int NT = 256;
constexpr int ACT_GELU = 0, ACT_TANH = 1, ACT_RELU = 2, ACT_NONE = 3;

template <int ACT>
__device__ __forceinline__ float act_f(float x) {
  if (ACT == ACT_GELU) return hx::gelu_f(x);
  if (ACT == ACT_TANH) return tanhf(x);
  if (ACT == ACT_RELU) return fmaxf(x, 0.f);
  return x;
}

// VEC adjacent elements per lane = one 16-B access of the activations (4 fp32 / 8 bf16; fp32
// bias rows of 8 take two); VEC == 4 for bf16 is the fallback when N is not a multiple of 8
template <typename T, int VEC>
__device__ __forceinline__ void ldv(const T* p, float (&v)[VEC]) {
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int k = 0; k < VEC; k += 4) {
      const float4 x = *reinterpret_cast<const float4*>(p + k);
      v[k] = x.x; v[k + 1] = x.y; v[k + 2] = x.z; v[k + 3] = x.w;
    }
  } else if constexpr (VEC == 8) {
    const uint4 x = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(w[k] << 16);
      v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  } else {
    const float4 x = hx::load4(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  }
}
template <typename T, int VEC>
__device__ __forceinline__ void stv(T* p, const float (&v)[VEC]) {
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int k = 0; k < VEC; k += 4) *reinterpret_cast<float4*>(p + k) = make_float4(v[k], v[k + 1], v[k + 2], v[k + 3]);
  } else if constexpr (VEC == 8) {
    uint4 x;
    x.x = hx::f2bf(v[0]) | ((uint32_t)hx::f2bf(v[1]) << 16);
    x.y = hx::f2bf(v[2]) | ((uint32_t)hx::f2bf(v[3]) << 16);
    x.z = hx::f2bf(v[4]) | ((uint32_t)hx::f2bf(v[5]) << 16);
    x.w = hx::f2bf(v[6]) | ((uint32_t)hx::f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(p) = x;
  } else {
    hx::store4(p, make_float4(v[0], v[1], v[2], v[3]));
  }
}

// grid-stride over VEC-element vectors; the (row, column) position advances incrementally by
// the constant grid stride (no 64-bit division per element)
template <typename T, int ACT, int VEC>
__global__ __launch_bounds__(NT) void bias_act_fwd_k(const T* __restrict__ y, const float* __restrict__ b,
                                                   T* __restrict__ out, int64_t rows, int N, int step_cols) {
  const int nv = N / VEC;
  const int64_t nvec = rows * (int64_t)nv;
  int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x;
  int c = (int)(i % nv);       // once per thread
  const int64_t stride = (int64_t)gridDim.x * NT;
  for (; i < nvec; i += stride) {
    float v[VEC];
    ldv<T, VEC>(y + i * VEC, v);
    if (b) {
      float bb[VEC];
      ldv<float, VEC>(b + c * VEC, bb);
#pragma unroll
      for (int k = 0; k < VEC; ++k) v[k] += bb[k];
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) v[k] = act_f<ACT>(v[k]);
    stv<T, VEC>(out + i * VEC, v);
    c += step_cols;
    if (c >= nv) c -= nv;
  }
}

// Column-tiled backward with fused column partials.
// grid: (ceil(N / (64 VEC)) column tiles, ceil(rows/64) row chunks); block = 4 waves.
// lane -> VEC adjacent columns (16 B), wave w -> rows w, w+4, ... of the chunk (two rows in
// flight per iteration); the 4 waves' partials are combined in LDS -> partial[chunk][N].
template <typename T, int ACT, int VEC>
__global__ __launch_bounds__(NT) void bias_act_bwd_k(const T* __restrict__ dout, const T* __restrict__ y,
                                                   const float* __restrict__ b, const T* __restrict__ saved_out,
                                                   T* __restrict__ dy, float* __restrict__ partial, int64_t rows,
                                                   int N) {
  __shared__ float red[4][VEC][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = (blockIdx.x * 64 + lane) * VEC;
  const int64_t r0 = (int64_t)blockIdx.y * hx::kRowChunk;
  const int64_t r1 = r0 + hx::kRowChunk < rows ? r0 + hx::kRowChunk : rows;
  float acc[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
  auto row = [&](int64_t r, const float (&bb)[VEC]) {
    const int64_t o = r * N + j;
    float d[VEC], g[VEC];
    ldv<T, VEC>(dout + o, d);
    if (ACT == ACT_GELU) {
      ldv<T, VEC>(y + o, g);
#pragma unroll
      for (int k = 0; k < VEC; ++k) g[k] = hx::gelu_grad_f(g[k] + bb[k]);
    } else if (ACT == ACT_TANH) {
      ldv<T, VEC>(saved_out + o, g);
#pragma unroll
      for (int k = 0; k < VEC; ++k) g[k] = 1.f - g[k] * g[k];
    } else if (ACT == ACT_RELU) {
      ldv<T, VEC>(saved_out + o, g);
#pragma unroll
      for (int k = 0; k < VEC; ++k) g[k] = g[k] > 0.f ? 1.f : 0.f;
    } else {
#pragma unroll
      for (int k = 0; k < VEC; ++k) g[k] = 1.f;
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      d[k] *= g[k];
      acc[k] += d[k];
    }
    if (dy) stv<T, VEC>(dy + o, d);
  };
  if (j < N) {
    float bb[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) bb[k] = 0.f;
    if (b) ldv<float, VEC>(b + j, bb);
    int64_t r = r0 + w;
    for (; r + 4 < r1; r += 8) {
      row(r, bb);
      row(r + 4, bb);
    }
    for (; r < r1; r += 4) row(r, bb);
  }
  if (!partial) return;
#pragma unroll
  for (int k = 0; k < VEC; ++k) red[w][k][lane] = acc[k];
  __syncthreads();
  if (w == 0 && j < N) {
    float o[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) o[k] = (red[0][k][lane] + red[1][k][lane]) + (red[2][k][lane] + red[3][k][lane]);
    float* dst = partial + (int64_t)blockIdx.y * N + j;
#pragma unroll
    for (int k = 0; k < VEC; k += 4) *reinterpret_cast<float4*>(dst + k) = make_float4(o[k], o[k + 1], o[k + 2], o[k + 3]);
  }
}


// scalar-column variant (any N); the optional device scalar scales the RESULT
// (the input is only read: scaling it in place would double the HBM traffic)
template <typename T>
__global__ __launch_bounds__(NT) void colsum_scalar_k(const T* __restrict__ x, const float* __restrict__ scale,
                                                    float* __restrict__ partial, int64_t rows, int N, int64_t ld) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.y * hx::kRowChunk;
  const int64_t r1 = r0 + hx::kRowChunk < rows ? r0 + hx::kRowChunk : rows;
  float acc = 0.f;
  if (j < N) {
    // 4 independent rows per iteration keep 4 loads in flight per lane
    float a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int64_t r = r0 + w;
    for (; r + 12 < r1; r += 16) {
      acc += hx::io<T>::ld(x + r * ld + j);
      a1 += hx::io<T>::ld(x + (r + 4) * ld + j);
      a2 += hx::io<T>::ld(x + (r + 8) * ld + j);
      a3 += hx::io<T>::ld(x + (r + 12) * ld + j);
    }
    for (; r < r1; r += 4) acc += hx::io<T>::ld(x + r * ld + j);
    acc = (acc + a1) + (a2 + a3);
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && j < N) {
    const float sc = scale ? scale[0] : 1.f;
    partial[(int64_t)blockIdx.y * N + j] = ((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane])) * sc;
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void dropout_k(const T* __restrict__ x, T* __restrict__ out, int64_t n,
                                              float keep_prob, const uint64_t* __restrict__ seedp, uint64_t stream) {
  const uint64_t seed = *seedp;   // per-update Philox key, device-resident (graph-safe)
  const float inv_keep = keep_prob > 0.f ? 1.f / keep_prob : 0.f;
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * NT) {
    float4 v = hx::load4(x + i * 4);
    const uint32_t k = hx::keep4(seed, stream, (uint64_t)i, keep_prob);
    v.x = (k & 1) ? v.x * inv_keep : 0.f;
    v.y = (k & 2) ? v.y * inv_keep : 0.f;
    v.z = (k & 4) ? v.z * inv_keep : 0.f;
    v.w = (k & 8) ? v.w * inv_keep : 0.f;
    hx::store4(out + i * 4, v);
  }
  // tail
  if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 3)) {
    const int64_t q = n4;
    const uint32_t k = hx::keep4(seed, stream, (uint64_t)q, keep_prob);
    for (int64_t e = q * 4; e < n; ++e) {
      const float v = hx::io<T>::ld(x + e);
      hx::io<T>::st(out + e, ((k >> (e - q * 4)) & 1) ? v * inv_keep : 0.f);
    }
  }
}

inline int egrid(int64_t n_vec) {
  int64_t b = (n_vec + NT - 1) / NT;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

inline int nchunks(int64_t rows) { return (int)((rows + hx::kRowChunk - 1) / hx::kRowChunk); }

template <typename T, int VEC>
void bias_act_fwd_v(int act, const void* y, const float* b, void* out, int64_t rows, int N, hipStream_t s) {
  const int nv = N / VEC;
  const int g = egrid(rows * (int64_t)nv);
  const int64_t stride = (int64_t)g * NT;
  const int sc = (int)(stride % nv);
  switch (act) {
    case ACT_GELU: bias_act_fwd_k<T, ACT_GELU, VEC><<<g, NT, 0, s>>>((const T*)y, b, (T*)out, rows, N, sc); break;
    case ACT_TANH: bias_act_fwd_k<T, ACT_TANH, VEC><<<g, NT, 0, s>>>((const T*)y, b, (T*)out, rows, N, sc); break;
    case ACT_RELU: bias_act_fwd_k<T, ACT_RELU, VEC><<<g, NT, 0, s>>>((const T*)y, b, (T*)out, rows, N, sc); break;
    default: bias_act_fwd_k<T, ACT_NONE, VEC><<<g, NT, 0, s>>>((const T*)y, b, (T*)out, rows, N, sc); break;
  }
}

template <typename T>
void bias_act_fwd_t(int act, const void* y, const float* b, void* out, int64_t rows, int N, hipStream_t s) {
  if (sizeof(T) == 2 && N % 8 == 0) bias_act_fwd_v<T, 8>(act, y, b, out, rows, N, s);
  else bias_act_fwd_v<T, 4>(act, y, b, out, rows, N, s);
}

template <typename T, int VEC>
void bias_act_bwd_v(int act, const void* dout, const void* y, const float* b, const void* saved_out, void* dy,
                    float* partial, float* dbias, int64_t rows, int N, int accumulate, hipStream_t s) {
  const int ncb = (N + 64 * VEC - 1) / (64 * VEC);
  const int nch = nchunks(rows);
  dim3 g(ncb, nch);
  float* part = dbias ? partial : nullptr;
#define HX_BAB(A)                                                                                            \
  bias_act_bwd_k<T, A, VEC><<<g, NT, 0, s>>>((const T*)dout, (const T*)y, b, (const T*)saved_out, (T*)dy, part, \
                                             rows, N)
  switch (act) {
    case ACT_GELU: HX_BAB(ACT_GELU); break;
    case ACT_TANH: HX_BAB(ACT_TANH); break;
    case ACT_RELU: HX_BAB(ACT_RELU); break;
    default: HX_BAB(ACT_NONE); break;
  }
#undef HX_BAB
  if (dbias) hx::fold_rows(partial, nch, N, N, N, dbias, nullptr, nullptr, accumulate, s);
}

template <typename T>
void bias_act_bwd_t(int act, const void* dout, const void* y, const float* b, const void* saved_out, void* dy,
                    float* partial, float* dbias, int64_t rows, int N, int accumulate, hipStream_t s) {
  if (sizeof(T) == 2 && N % 8 == 0)
    bias_act_bwd_v<T, 8>(act, dout, y, b, saved_out, dy, partial, dbias, rows, N, accumulate, s);
  else
    bias_act_bwd_v<T, 4>(act, dout, y, b, saved_out, dy, partial, dbias, rows, N, accumulate, s);
}

}  // namespace

int hx_colsum_ws_floats(int64_t rows, int N) { return nchunks(rows) * N; }

void hx_bias_act_fwd(int bf16, int act, const void* y, const float* b, void* out, int64_t rows, int N,
                     hipStream_t s) {
  if (bf16) bias_act_fwd_t<uint16_t>(act, y, b, out, rows, N, s);
  else bias_act_fwd_t<float>(act, y, b, out, rows, N, s);
}

void hx_bias_act_bwd(int bf16, int act, const void* dout, const void* y, const float* b, const void* saved_out,
                     void* dy, float* partial, float* dbias, int64_t rows, int N, int accumulate, hipStream_t s) {
  if (bf16) bias_act_bwd_t<uint16_t>(act, dout, y, b, saved_out, dy, partial, dbias, rows, N, accumulate, s);
  else bias_act_bwd_t<float>(act, dout, y, b, saved_out, dy, partial, dbias, rows, N, accumulate, s);
}

void hx_colsum(int bf16, void* x, const float* scale, float* partial, float* out, int64_t rows, int N,
               int accumulate, hipStream_t s, int64_t ld) {
  if (ld < 0) ld = N;
  if (N % 4 == 0 && scale == nullptr && ld == N) {
    // vector path reusing the bias-act backward with identity activation (no dy written)
    hx_bias_act_bwd(bf16, ACT_NONE, x, nullptr, nullptr, nullptr, nullptr, partial, out, rows, N, accumulate, s);
    return;
  }
  const int ncb = (N + 63) / 64;
  const int nch = nchunks(rows);
  dim3 g(ncb, nch);
  if (bf16) colsum_scalar_k<uint16_t><<<g, NT, 0, s>>>((const uint16_t*)x, scale, partial, rows, N, ld);
  else colsum_scalar_k<float><<<g, NT, 0, s>>>((const float*)x, scale, partial, rows, N, ld);
  hx::fold_rows(partial, nch, N, N, N, out, nullptr, nullptr, accumulate, s);
}

void hx_dropout(int bf16, const void* x, void* out, int64_t n, float keep_prob, const uint64_t* seed, uint64_t stream,
                hipStream_t s) {
  const int g = egrid(n / 4 + 1);
  if (bf16) dropout_k<uint16_t><<<g, NT, 0, s>>>((const uint16_t*)x, (uint16_t*)out, n, keep_prob, seed, stream);
  else dropout_k<float><<<g, NT, 0, s>>>((const float*)x, (float*)out, n, keep_prob, seed, stream);
}
