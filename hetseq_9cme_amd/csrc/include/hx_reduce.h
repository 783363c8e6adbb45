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

// the same fold with more, narrower blocks: the fold is bound by how much one block can pull
// (r5n: 12 blocks of 256 columns x 512 partial rows each reading 512 KB -> 12 us), so a block
// takes 32 columns (8 lanes x float4) over 32 row slots (4 waves x 8), four loads in flight per
// lane, and a [32][32] LDS combine.  Needs stride, ncols, seg and nsum multiples of 4 and a 16-B
// aligned base.
constexpr int kFold4NT = 256;
__global__ __launch_bounds__(kFold4NT) void fold_rows4_k(const float* __restrict__ partial, int nrows, int64_t stride,
                                                       int ncols, int seg, float* __restrict__ out0,
                                                       float* __restrict__ out1, float* __restrict__ out2,
                                                       int accumulate, int nsum, float* __restrict__ outm) {
  __shared__ float4 red[32][8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane & 7, slot = w * 8 + (lane >> 3);   // column quad, row slot (0 .. 31)
  const int c = blockIdx.x * 32 + 4 * q;
  const bool mx = c >= nsum;
  auto acc = [&](float4& a, const float4& x) {
    if (mx) {
      a.x = fmaxf(a.x, x.x); a.y = fmaxf(a.y, x.y); a.z = fmaxf(a.z, x.z); a.w = fmaxf(a.w, x.w);
    } else {
      a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
    }
  };
  float4 a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < ncols) {
    const float* p = partial + c;
    int r = slot;
    for (; r + 96 < nrows; r += 128) {
      float4 x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = *reinterpret_cast<const float4*>(p + (int64_t)(r + 32 * j) * stride);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc(a[j], x[j]);
    }
    for (; r < nrows; r += 32) acc(a[0], *reinterpret_cast<const float4*>(p + (int64_t)r * stride));
  }
  acc(a[0], a[1]);
  acc(a[2], a[3]);
  acc(a[0], a[2]);
  red[slot][q] = a[0];
  __syncthreads();
  if (threadIdx.x < 8 && c < ncols) {   // threads 0 .. 7: q == threadIdx.x, slot 0
    float4 v = red[0][q];
#pragma unroll
    for (int k = 1; k < 32; ++k) acc(v, red[k][q]);
    if (mx) {
      *reinterpret_cast<float4*>(outm + (c - nsum)) = v;
      return;
    }
    const int qq = c / seg, j = c - qq * seg;
    float* o = qq == 0 ? out0 : (qq == 1 ? out1 : out2);
    if (o) {
      float4* op = reinterpret_cast<float4*>(o + j);
      if (accumulate) {
        const float4 x = *op;
        v.x += x.x; v.y += x.y; v.z += x.z; v.w += x.w;
      }
      *op = v;
    }
  }
}

inline void fold_rows(const float* partial, int nrows, int64_t stride, int ncols, int seg, float* o0, float* o1,
                      float* o2, int accumulate, hipStream_t s, int nsum = -1, float* outm = nullptr) {
  if (nsum < 0) nsum = ncols;
  const auto a16 = [](const void* p) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  if (stride % 4 == 0 && ncols % 4 == 0 && seg % 4 == 0 && nsum % 4 == 0 && a16(partial) && a16(o0) && a16(o1) &&
      a16(o2) && a16(outm)) {
    fold_rows4_k<<<(ncols + 31) / 32, kFold4NT, 0, s>>>(partial, nrows, stride, ncols, seg, o0, o1, o2, accumulate,
                                                         nsum, outm);
    return;
  }
  fold_rows_k<<<(ncols + 63) / 64, kFoldNT, 0, s>>>(partial, nrows, stride, ncols, seg, o0, o1, o2, accumulate,
                                                    nsum, outm);
}

}  // namespace
}  // namespace hx
