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

// the same fold, 4 columns per lane: a block = 16 waves over 256 columns (float4 loads, four
// independent accumulators per lane), so the few column blocks of a bias / LayerNorm gradient
// each keep 16 x 4 loads in flight per row pass instead of one (the fold is latency-bound: ~12
// blocks on 256 CUs).  Needs stride, ncols, seg and nsum multiples of 4 and a 16-B aligned base.
constexpr int kFold4NT = 1024;
__global__ __launch_bounds__(kFold4NT) void fold_rows4_k(const float* __restrict__ partial, int nrows, int64_t stride,
                                                       int ncols, int seg, float* __restrict__ out0,
                                                       float* __restrict__ out1, float* __restrict__ out2,
                                                       int accumulate, int nsum, float* __restrict__ outm) {
  __shared__ float4 red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + lane) * 4;
  const bool mx = c >= nsum;
  float4 a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < ncols) {
    const float* p = partial + c;
    int r = w;
    for (; r + 48 < nrows; r += 64) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 x = *reinterpret_cast<const float4*>(p + (int64_t)(r + 16 * j) * stride);
        if (mx) {
          a[j].x = fmaxf(a[j].x, x.x); a[j].y = fmaxf(a[j].y, x.y); a[j].z = fmaxf(a[j].z, x.z); a[j].w = fmaxf(a[j].w, x.w);
        } else {
          a[j].x += x.x; a[j].y += x.y; a[j].z += x.z; a[j].w += x.w;
        }
      }
    }
    for (; r < nrows; r += 16) {
      const float4 x = *reinterpret_cast<const float4*>(p + (int64_t)r * stride);
      if (mx) {
        a[0].x = fmaxf(a[0].x, x.x); a[0].y = fmaxf(a[0].y, x.y); a[0].z = fmaxf(a[0].z, x.z); a[0].w = fmaxf(a[0].w, x.w);
      } else {
        a[0].x += x.x; a[0].y += x.y; a[0].z += x.z; a[0].w += x.w;
      }
    }
  }
  float4 t;
  if (mx) {
    t.x = fmaxf(fmaxf(a[0].x, a[1].x), fmaxf(a[2].x, a[3].x));
    t.y = fmaxf(fmaxf(a[0].y, a[1].y), fmaxf(a[2].y, a[3].y));
    t.z = fmaxf(fmaxf(a[0].z, a[1].z), fmaxf(a[2].z, a[3].z));
    t.w = fmaxf(fmaxf(a[0].w, a[1].w), fmaxf(a[2].w, a[3].w));
  } else {
    t.x = (a[0].x + a[1].x) + (a[2].x + a[3].x);
    t.y = (a[0].y + a[1].y) + (a[2].y + a[3].y);
    t.z = (a[0].z + a[1].z) + (a[2].z + a[3].z);
    t.w = (a[0].w + a[1].w) + (a[2].w + a[3].w);
  }
  red[w][lane] = t;
  __syncthreads();
  if (w == 0 && c < ncols) {
    float4 v = red[0][lane];
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      const float4 x = red[k][lane];
      if (mx) {
        v.x = fmaxf(v.x, x.x); v.y = fmaxf(v.y, x.y); v.z = fmaxf(v.z, x.z); v.w = fmaxf(v.w, x.w);
      } else {
        v.x += x.x; v.y += x.y; v.z += x.z; v.w += x.w;
      }
    }
    if (mx) {
      *reinterpret_cast<float4*>(outm + (c - nsum)) = v;
      return;
    }
    const int q = c / seg, j = c - q * seg;
    float* o = q == 0 ? out0 : (q == 1 ? out1 : out2);
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
    fold_rows4_k<<<(ncols + 255) / 256, kFold4NT, 0, s>>>(partial, nrows, stride, ncols, seg, o0, o1, o2, accumulate,
                                                         nsum, outm);
    return;
  }
  fold_rows_k<<<(ncols + 63) / 64, kFoldNT, 0, s>>>(partial, nrows, stride, ncols, seg, o0, o1, o2, accumulate,
                                                    nsum, outm);
}

}  // namespace
}  // namespace hx
