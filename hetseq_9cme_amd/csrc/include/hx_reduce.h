// Column-partial folding shared by the bias-grad / LayerNorm-grad reductions.
#pragma once
#include "hx_common.h"

namespace hx {
namespace {  // internal linkage: each kernel TU gets its own copy

constexpr int kFoldNT = 256;
constexpr int kRowChunk = 64;   // rows per column-partial chunk

// partial[r * stride + c] for r < nrows, c < ncols  ->  sum over r.
// Column c goes to out[c / seg][c % seg] (out0/out1/out2, nullptr = skip).
// Block = 4 waves over 64 columns (lane = column); waves split the rows, LDS combine.
// columns [0, nsum) of the [nrows][stride] partials are summed (segments of seg columns into out0 /
// out1 / out2); columns [nsum, ncols) take the MAX instead (into outm: column-maxima partials)
__global__ __launch_bounds__(kFoldNT) void fold_rows_k(const float* __restrict__ partial, int nrows,
                                                     int64_t stride, int ncols, int seg, float* __restrict__ out0,
                                                     float* __restrict__ out1, float* __restrict__ out2,
                                                     int accumulate, int nsum, float* __restrict__ outm) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const bool mx = c >= nsum;
  float a = 0.f;
  if (c < ncols) {
    int r = w;
#pragma unroll 4
    for (; r + 12 < nrows; r += 16) {
      const float x0 = partial[(int64_t)r * stride + c];
      const float x1 = partial[(int64_t)(r + 4) * stride + c];
      const float x2 = partial[(int64_t)(r + 8) * stride + c];
      const float x3 = partial[(int64_t)(r + 12) * stride + c];
      a = mx ? fmaxf(fmaxf(a, fmaxf(x0, x1)), fmaxf(x2, x3)) : a + ((x0 + x1) + (x2 + x3));
    }
    for (; r < nrows; r += 4) {
      const float x = partial[(int64_t)r * stride + c];
      a = mx ? fmaxf(a, x) : a + x;
    }
  }
  red[w][lane] = a;
  __syncthreads();
  if (w == 0 && c < ncols) {
    if (mx) {
      outm[c - nsum] = fmaxf(fmaxf(red[0][lane], red[1][lane]), fmaxf(red[2][lane], red[3][lane]));
      return;
    }
    const float t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    const int q = c / seg, j = c - q * seg;
    float* o = q == 0 ? out0 : (q == 1 ? out1 : out2);
    if (o) o[j] = accumulate ? o[j] + t : t;
  }
}

inline void fold_rows(const float* partial, int nrows, int64_t stride, int ncols, int seg, float* o0, float* o1,
                      float* o2, int accumulate, hipStream_t s, int nsum = -1, float* outm = nullptr) {
  fold_rows_k<<<(ncols + 63) / 64, kFoldNT, 0, s>>>(partial, nrows, stride, ncols, seg, o0, o1, o2, accumulate,
                                                    nsum < 0 ? ncols : nsum, outm);
}

}  // namespace
}  // namespace hx
