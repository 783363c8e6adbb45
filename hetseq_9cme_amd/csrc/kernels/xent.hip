// Fused softmax-cross-entropy over the (masked-row) MLM decoder logits.
//
// Reference (bert_modeling.py:544-547, :899-901): decoder GEMM over ALL B*S rows,
// separate ``+ bias`` pass, then CrossEntropyLoss(ignore_index=-1) = log_softmax +
// nll + their backward (500 MB - 2 GB of fp32 logits per step).
// Here the decoder only sees the gathered masked rows and this ONE kernel:
//   * adds the decoder bias on the fly (bias never materialised with the logits),
//   * computes the row's log-sum-exp with an online (max, sum) pass,
//   * writes loss_row = lse - z[label]  (0 for ignored rows),
//   * overwrites the logits IN PLACE with softmax(z) - onehot(label)  (0 for
//     ignored rows) -- the unscaled gradient, so backward needs no extra buffer.
// Backward then only scales rows by dL/dloss / count and folds the bias gradient
// (hx_colsum with a device scale).  One workgroup per row; for V <= 32768 (BERT:
// 30522 -> 120 columns per lane) the row stays in registers between the max, sum
// and write passes: one read + one write of the 122 KB row, one exp per element.
// Larger vocabularies use the two-read online-softmax variant.
#include "hx_launch.h"
#include "hx_vec.h"

namespace {

constexpr int NT = 256;

template <typename T>
__global__ __launch_bounds__(NT) void softmax_xent_k(T* __restrict__ logits, const float* __restrict__ bias,
                                                   const int64_t* __restrict__ labels, float* __restrict__ loss,
                                                   int V, int64_t ld, int64_t ignore_index) {
  __shared__ float sm[NT / 64], ss[NT / 64];
  const int64_t row = blockIdx.x;
  T* x = logits + row * ld;
  const int64_t lab = labels[row];
  const bool valid = lab != ignore_index && lab >= 0 && lab < V;
  if (!valid) {
    for (int j = threadIdx.x; j < V; j += NT) hx::io<T>::st(x + j, 0.f);
    if (threadIdx.x == 0) loss[row] = 0.f;
    return;
  }
  // online max / sum
  float m = -INFINITY, s = 0.f;
  for (int j = threadIdx.x; j < V; j += NT) {
    const float z = hx::io<T>::ld(x + j) + (bias ? bias[j] : 0.f);
    if (z > m) {
      s = s * __expf(m - z) + 1.f;
      m = z;
    } else {
      s += __expf(z - m);
    }
  }
  // wave combine
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float mo = __shfl_xor(m, o, 64), so = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, mo);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (mo == -INFINITY ? 0.f : so * __expf(mo - mn));
    m = mn;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm[w] = m;
    ss[w] = s;
  }
  __syncthreads();
  float M = sm[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) M = fmaxf(M, sm[i]);
  float Ssum = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) Ssum += ss[i] * __expf(sm[i] - M);
  const float lse = M + __logf(Ssum);
  const float inv = 1.f / Ssum;
  float zl = 0.f;
  for (int j = threadIdx.x; j < V; j += NT) {
    const float z = hx::io<T>::ld(x + j) + (bias ? bias[j] : 0.f);
    float p = __expf(z - M) * inv;
    if (j == lab) {
      zl = z;
      p -= 1.f;
    }
    hx::io<T>::st(x + j, p);
  }
  if ((int)(lab % NT) == (int)threadIdx.x) loss[row] = lse - zl;
}

// Register-resident row (NR threads): lane t holds columns t, t + NR, ..., t + (K-1)*NR.
// Buffer loads/stores (hx::Buf): one lane offset + a uniform offset per chunk, so the
// K values are the only per-element registers; out-of-row stores are dropped by the
// descriptor's range.
template <typename T, int NR, int K, bool kBias>
__global__ __launch_bounds__(NR) __attribute__((amdgpu_waves_per_eu(8, 8))) void softmax_xent_reg_k(
    T* __restrict__ logits, const float* __restrict__ bias, const int64_t* __restrict__ labels,
    float* __restrict__ loss, int V, int64_t ld, int64_t ignore_index) {
  __shared__ float red[NR / 64];
  const int64_t row = blockIdx.x;
  const hx::Buf xb(logits + row * ld, (uint32_t)V * sizeof(T));
  const int64_t lab = labels[row];
  const bool valid = lab != ignore_index && lab >= 0 && lab < V;
  const int t = threadIdx.x, w = t >> 6;
  if (!valid) {
#pragma unroll
    for (int k = 0; k < K; ++k) hx::bio<T>::st(xb, t, k * NR, 0.f);
    if (t == 0) loss[row] = 0.f;
    return;
  }
  float v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = hx::bio<T>::ld(xb, t, k * NR);
  if constexpr (kBias) {
    const hx::Buf bb(bias, (uint32_t)V * 4);
    // in groups of 8 behind scheduling barriers: the bias loads (L2 hits) never need
    // K more registers while the row loads are in flight
#pragma unroll
    for (int k0 = 0; k0 < K; k0 += 8) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = k0; k < k0 + 8 && k < K; ++k) v[k] += hx::bio<float>::ld(bb, t, k * NR);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    // padding columns load as 0: mask them, behind a wave-uniform test so full chunks
    // carry no per-element select (and no second copy of the value)
    if ((k + 1) * NR > V) v[k] = t + k * NR < V ? v[k] : -INFINITY;
    m = fmaxf(m, v[k]);
  }
  m = hx::wave_max(m);
  if ((t & 63) == 0) red[w] = m;
  __syncthreads();
  float M = red[0];
#pragma unroll
  for (int i = 1; i < NR / 64; ++i) M = fmaxf(M, red[i]);
  __syncthreads();
  // the label's logit (wave-uniform address: scalar loads)
  const float zl = hx::io<T>::ld(logits + row * ld + lab) + (kBias ? bias[lab] : 0.f);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    v[k] = __expf(v[k] - M);   // exp(-inf) = 0 for the padding columns
    s += v[k];
  }
  s = hx::wave_sum(s);
  if ((t & 63) == 0) red[w] = s;
  __syncthreads();
  float S = 0.f;
#pragma unroll
  for (int i = 0; i < NR / 64; ++i) S += red[i];
  const float inv = 1.f / S;
#pragma unroll
  for (int k = 0; k < K; ++k) hx::bio<T>::st(xb, t, k * NR, v[k] * inv);
  // the lane that just wrote the label's column rewrites it as p - 1 (same lane, same
  // address: ordered after its own store)
  if ((int)(lab % NR) == t) {
    hx::bio<T>::st(xb, (uint32_t)lab, 0, __expf(zl - M) * inv - 1.f);
    loss[row] = M + __logf(S) - zl;
  }
}

}  // namespace

void hx_softmax_xent(int bf16, void* logits, const float* bias, const int64_t* labels, float* loss, int64_t rows,
                     int V, int64_t ld, int64_t ignore_index, hipStream_t s) {
  if (rows <= 0) return;
#define HX_XENT_REG2(NRR, KK, BB)                                                                            \
  if (bf16)                                                                                                 \
    softmax_xent_reg_k<uint16_t, NRR, KK, BB>                                                               \
        <<<(unsigned)rows, NRR, 0, s>>>((uint16_t*)logits, bias, labels, loss, V, ld, ignore_index);        \
  else                                                                                                      \
    softmax_xent_reg_k<float, NRR, KK, BB>                                                                  \
        <<<(unsigned)rows, NRR, 0, s>>>((float*)logits, bias, labels, loss, V, ld, ignore_index);
#define HX_XENT_REG(NRR, KK) \
  if (bias) {                \
    HX_XENT_REG2(NRR, KK, true) \
  } else {                   \
    HX_XENT_REG2(NRR, KK, false) \
  }
  // 1024 threads x 32 columns: ~60 VGPRs, so two rows (32 waves) are in flight per CU
  if (V <= 16 * 256) {
    HX_XENT_REG(256, 16)
  } else if (V <= 16 * 1024) {
    HX_XENT_REG(1024, 16)
  } else if (V <= 32 * 1024) {
    HX_XENT_REG(1024, 32)
  } else if (bf16) {
    softmax_xent_k<uint16_t><<<(unsigned)rows, NT, 0, s>>>((uint16_t*)logits, bias, labels, loss, V, ld, ignore_index);
  } else {
    softmax_xent_k<float><<<(unsigned)rows, NT, 0, s>>>((float*)logits, bias, labels, loss, V, ld, ignore_index);
  }
#undef HX_XENT_REG
#undef HX_XENT_REG2
}
