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
// (hx_colsum with a device scale).  One workgroup per row; V = 30522 -> 120 columns
// per lane, two reads + one write of the row.
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

}  // namespace

void hx_softmax_xent(int bf16, void* logits, const float* bias, const int64_t* labels, float* loss, int64_t rows,
                     int V, int64_t ld, int64_t ignore_index, hipStream_t s) {
  if (rows <= 0) return;
  if (bf16)
    softmax_xent_k<uint16_t><<<(unsigned)rows, NT, 0, s>>>((uint16_t*)logits, bias, labels, loss, V, ld, ignore_index);
  else
    softmax_xent_k<float><<<(unsigned)rows, NT, 0, s>>>((float*)logits, bias, labels, loss, V, ld, ignore_index);
}
