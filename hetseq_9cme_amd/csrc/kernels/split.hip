// fp32 -> bf16 "planes" for fp32 GEMMs emulated on the bf16 matrix cores.
//
// gfx950 runs bf16 MFMA at 16x the rate of its f32-input MFMA (2.5 PF vs 157 TF dense).
// An fp32 value x is written as a sum of bf16 pieces: x0 = bf16(x), x1 = bf16(x - x0),
// x2 = bf16(x - x0 - x1) (round-to-nearest-even each time), so x = x0 + x1 + O(2^-18 |x|)
// with two pieces and x0 + x1 + x2 + O(2^-27 |x|) with three.  A product a.b becomes a sum
// of piece products, each EXACT in the MFMA's fp32 accumulator (8 x 8 significand bits):
//   3 passes: a0 b0 + a1 b0 + a0 b1                       (dropped terms ~2^-17 |ab|)
//   6 passes: + a2 b0 + a1 b1 + a0 b2                     (dropped terms ~2^-26 |ab|)
// Stacking the pass operands along the reduction dimension turns the sum into ONE ordinary
// bf16 GEMM with K' = passes * K (ops/split_gemm.py explains the plane orders that make the
// forward, data-gradient and weight-gradient GEMMs pair the right pieces).
//
// This kernel writes the planes: row r of x [R][D] becomes `npl` consecutive bf16 rows
// (interleaved: out[(r * npl + j) * D + c]) or plane j becomes a block of R rows (stacked:
// out[(j * R + r) * D + c]); plane j holds piece order[j].  One pass over x, 8 elements per
// lane (two 16-B loads, one 16-B store per plane), HBM-bound; other shapes take the
// one-element-per-lane form below, which can also zero-pad rows / columns.
#include <algorithm>

#include "hx_launch.h"
#include "hx_common.h"

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)hx::f2bf(a) | ((uint32_t)hx::f2bf(b) << 16);
}

template <int NPIECE, bool kNT>
__global__ __launch_bounds__(256) void split_planes_k(const float* __restrict__ x, int64_t ldx,
                                                      uint16_t* __restrict__ out, int64_t R, int D, int npl,
                                                      uint32_t order, int stacked) {
  const int d8 = D >> 3;
  const int64_t n8 = R * d8;
  const int64_t row_stride = stacked ? (int64_t)D : (int64_t)npl * D;
  const int64_t plane_stride = stacked ? R * D : (int64_t)D;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / d8;
    const int c = (int)(i - r * d8) * 8;
    const float4 u = *reinterpret_cast<const float4*>(x + r * ldx + c);
    const float4 v = *reinterpret_cast<const float4*>(x + r * ldx + c + 4);
    float p[NPIECE][8];
    float e[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < NPIECE; ++k)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float q = hx::bf2f(hx::f2bf(e[t]));
        p[k][t] = q;
        e[t] -= q;    // exact: the residual of a round-to-nearest bf16 fits in fp32
      }
    u32x4 w[NPIECE];
#pragma unroll
    for (int k = 0; k < NPIECE; ++k)
      w[k] = u32x4{pack2(p[k][0], p[k][1]), pack2(p[k][2], p[k][3]), pack2(p[k][4], p[k][5]),
                   pack2(p[k][6], p[k][7])};
    uint16_t* o = out + r * row_stride + c;
    for (int j = 0; j < npl; ++j) {
      const int k = (order >> (4 * j)) & 15;
      const u32x4 v = w[k < NPIECE ? k : NPIECE - 1];
      if constexpr (kNT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(o + j * plane_stride));
      else *reinterpret_cast<u32x4*>(o + j * plane_stride) = v;
    }
  }
}

// General form: any D / row stride / alignment, rows padded to Rp and columns to Dp with
// zeros (e.g. the MLM decoder's 30522-wide logits gradient, padded to a multiple of 64 so
// the bf16 planes have 16-B aligned rows for the GEMM).  One element per lane.
template <int NPIECE>
__global__ __launch_bounds__(256) void split_planes_any_k(const float* __restrict__ x, int64_t ldx,
                                                          uint16_t* __restrict__ out, int64_t R, int D, int64_t Rp,
                                                          int Dp, int npl, uint32_t order, int stacked) {
  const int64_t n = Rp * Dp;
  const int64_t row_stride = stacked ? (int64_t)Dp : (int64_t)npl * Dp;
  const int64_t plane_stride = stacked ? Rp * Dp : (int64_t)Dp;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / Dp;
    const int c = (int)(i - r * Dp);
    float e = (r < R && c < D) ? x[r * ldx + c] : 0.f;
    uint16_t p[NPIECE];
#pragma unroll
    for (int k = 0; k < NPIECE; ++k) {
      p[k] = hx::f2bf(e);
      e -= hx::bf2f(p[k]);
    }
    uint16_t* o = out + r * row_stride + c;
    for (int j = 0; j < npl; ++j) {
      const int k = (order >> (4 * j)) & 15;
      o[j * plane_stride] = p[k < NPIECE ? k : NPIECE - 1];
    }
  }
}

// Interleaved planes of a matrix whose rows are only 8-B aligned (odd width: the MLM
// decoder's [rows, 30522] logits gradient), columns zero-padded to Dp (a multiple of 8):
// 8 columns per lane from four 8-B loads, one 16-B nontemporal store per plane.
template <int NPIECE>
__global__ __launch_bounds__(256) void split_planes_pad8_k(const float* __restrict__ x, int64_t ldx,
                                                           uint16_t* __restrict__ out, int64_t R, int D, int Dp,
                                                           int npl, uint32_t order) {
  const int d8 = Dp >> 3;
  const int64_t n8 = R * d8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / d8;
    const int c = (int)(i - r * d8) * 8;
    float e[8];
    const float* xr = x + r * ldx + c;
    if (c + 8 <= D) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float2 v = *reinterpret_cast<const float2*>(xr + 2 * k);
        e[2 * k] = v.x;
        e[2 * k + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) e[k] = c + k < D ? xr[k] : 0.f;
    }
    u32x4 w[NPIECE];
#pragma unroll
    for (int p = 0; p < NPIECE; ++p) {
      uint32_t q[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        q[t] = hx::f2bf(e[t]);
        e[t] -= hx::bf2f((uint16_t)q[t]);
      }
      w[p] = u32x4{q[0] | (q[1] << 16), q[2] | (q[3] << 16), q[4] | (q[5] << 16), q[6] | (q[7] << 16)};
    }
    uint16_t* o = out + r * (int64_t)npl * Dp + c;
    for (int j = 0; j < npl; ++j) {
      const int k = (order >> (4 * j)) & 15;
      __builtin_nontemporal_store(w[k < NPIECE ? k : NPIECE - 1], reinterpret_cast<u32x4*>(o + (int64_t)j * Dp));
    }
  }
}

// Weight pieces in both layouts the split GEMMs read (ops/split_gemm.py), one pass over W:
//   wf[n][p][k] = piece p of W[n][k]   (forward: B operand of y = x W^T)
//   wt[k][p][n] = piece p of W[n][k]   (data gradient: B operand of dx = dy W = dy (W^T)^T)
// 64 x 64 tiles: coalesced float4 reads, wf written directly, wt through an LDS transpose.
// BF / BT: wf / wt in the B16 layout (gemm_split.hip).
//
// element offset of (row, piece p, column c) in a [rows][NPC * C] pieces matrix: natural
// [rows][NPC][C], or the B16 layout [rows][C / 16][NPC][16] (gemm_split.hip)
template <int NPC, bool B16>
__device__ __forceinline__ int64_t pc_off(int64_t row, int p, int c, int C) {
  return B16 ? row * NPC * C + (c >> 4) * (16 * NPC) + p * 16 + (c & 15) : (row * NPC + p) * C + c;
}

template <int NPC, bool BF, bool BT>
__device__ __forceinline__ void split_weight_tile(const float* __restrict__ W, int N, int K, uint16_t* __restrict__ wf,
                                                  uint16_t* __restrict__ wt, int k0, int n0,
                                                  uint16_t (&tile)[NPC][64][66]) {
  const int t = threadIdx.x, c4 = (t & 15) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (t >> 4) + 16 * i;
    const float4 v = *reinterpret_cast<const float4*>(W + (int64_t)(n0 + r) * K + k0 + c4);
    float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int p = 0; p < NPC; ++p) {
      uint16_t q[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        q[j] = hx::f2bf(e[j]);
        e[j] -= hx::bf2f(q[j]);
        tile[p][r][c4 + j] = q[j];
      }
      uint2 packed = make_uint2(q[0] | ((uint32_t)q[1] << 16), q[2] | ((uint32_t)q[3] << 16));
      *reinterpret_cast<uint2*>(wf + pc_off<NPC, BF>(n0 + r, p, k0 + c4, K)) = packed;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kk = (t >> 4) + 16 * i;   // row of wt inside the tile
#pragma unroll
    for (int p = 0; p < NPC; ++p) {
      uint16_t q[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) q[j] = tile[p][c4 + j][kk];
      uint2 packed = make_uint2(q[0] | ((uint32_t)q[1] << 16), q[2] | ((uint32_t)q[3] << 16));
      *reinterpret_cast<uint2*>(wt + pc_off<NPC, BT>(k0 + kk, p, n0 + c4, N)) = packed;
    }
  }
}

template <int NPC, bool BF, bool BT>
__global__ __launch_bounds__(256) void split_weight_k(const float* __restrict__ W, int N, int K,
                                                     uint16_t* __restrict__ wf, uint16_t* __restrict__ wt) {
  __shared__ uint16_t tile[NPC][64][66];
  split_weight_tile<NPC, BF, BT>(W, N, K, wf, wt, blockIdx.x * 64, blockIdx.y * 64, tile);
}

// Every weight of a forward in ONE launch (HxWeightBatch: up to HX_WBATCH weights, their 64 x 64
// tiles numbered consecutively): the per-weight launches are latency-bound at BERT-base sizes
// (768 x 768: 144 workgroups, fewer than the CUs; ~10 us each for ~2 us of traffic).
template <int NPC>
__global__ __launch_bounds__(256) void split_weight_many_k(HxWeightBatch d) {
  __shared__ uint16_t tile[NPC][64][66];
  const int b = blockIdx.x;
  int i = 0;
  while (i + 1 < d.n && b >= d.start[i + 1]) ++i;   // uniform per workgroup
  const int tk = d.K[i] / 64, loc = b - d.start[i];
  const int k0 = (loc % tk) * 64, n0 = (loc / tk) * 64;
  const int m = d.mask[i];
  if constexpr (NPC == 3) {
    if (m == 3) split_weight_tile<3, true, true>(d.W[i], d.N[i], d.K[i], d.wf[i], d.wt[i], k0, n0, tile);
    else if (m == 1) split_weight_tile<3, true, false>(d.W[i], d.N[i], d.K[i], d.wf[i], d.wt[i], k0, n0, tile);
    else if (m == 2) split_weight_tile<3, false, true>(d.W[i], d.N[i], d.K[i], d.wf[i], d.wt[i], k0, n0, tile);
    else split_weight_tile<3, false, false>(d.W[i], d.N[i], d.K[i], d.wf[i], d.wt[i], k0, n0, tile);
  } else {
    split_weight_tile<2, false, false>(d.W[i], d.N[i], d.K[i], d.wf[i], d.wt[i], k0, n0, tile);
  }
}

// Transposed planes of a weight, the data-gradient operand in "NT" form:
//   out[k][j * Np + n] = piece order[j] of W[n][k]   (zero for N <= n < Np)
// so dx = dy' . out^T reads both operands along the reduction dimension like the forward
// GEMM does (measured on MI355X, BERT-base shapes: 7-15 % faster than the NN product with
// the stacked [npl * Np, K] planes, tools/probe/dgrad_layout_probe.py).  64 x 64 tiles:
// coalesced float4 reads of W, pieces transposed through LDS, 16-B row-segment stores.
template <int NPIECE>
__global__ __launch_bounds__(256) void split_planes_t_k(const float* __restrict__ W, int64_t ldw, int N, int K,
                                                        uint16_t* __restrict__ out, int Np, int npl,
                                                        uint32_t order) {
  __shared__ uint16_t tile[NPIECE][64][72];   // [piece][k][n], rows padded to 144 B (16-B aligned)
  const int n0 = blockIdx.x * 64, k0 = blockIdx.y * 64;
  const int t = threadIdx.x, c4 = (t & 15) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (t >> 4) + 16 * i;   // row n0 + r of W
    float e[4] = {0.f, 0.f, 0.f, 0.f};
    if (n0 + r < N) {
      const float4 v = *reinterpret_cast<const float4*>(W + (int64_t)(n0 + r) * ldw + k0 + c4);
      e[0] = v.x; e[1] = v.y; e[2] = v.z; e[3] = v.w;
    }
#pragma unroll
    for (int p = 0; p < NPIECE; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint16_t q = hx::f2bf(e[j]);
        e[j] -= hx::bf2f(q);
        tile[p][c4 + j][r] = q;
      }
  }
  __syncthreads();
  // 64 k-rows x 8 chunks of 8 n per piece: two 16-B chunks per thread and plane
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = t + 256 * i, kk = e >> 3, ch = e & 7;
    uint16_t* o = out + (int64_t)(k0 + kk) * npl * Np + n0 + 8 * ch;
    for (int j = 0; j < npl; ++j) {
      const int p = (order >> (4 * j)) & 15;
      const u32x4 v = *reinterpret_cast<const u32x4*>(&tile[p < NPIECE ? p : NPIECE - 1][kk][8 * ch]);
      *reinterpret_cast<u32x4*>(o + (int64_t)j * Np) = v;
    }
  }
}

}  // namespace

void hx_split_planes_t(const float* W, int64_t ldw, int N, int K, uint16_t* out, int Np, int npieces, int npl,
                       uint32_t order, hipStream_t s) {
  dim3 g(Np / 64, K / 64);
  if (npieces == 3)
    split_planes_t_k<3><<<g, 256, 0, s>>>(W, ldw, N, K, out, Np, npl, order);
  else
    split_planes_t_k<2><<<g, 256, 0, s>>>(W, ldw, N, K, out, Np, npl, order);
}

void hx_split_planes(const float* x, int64_t ldx, uint16_t* out, int64_t R, int D, int64_t Rp, int Dp,
                     int npieces, int npl, uint32_t order, int stacked, hipStream_t s) {
  const bool vec = D % 8 == 0 && Dp == D && Rp == R && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0;
  if (vec) {
    const int64_t n8 = R * (D / 8);
    if (n8 <= 0) return;
    const int blocks = (int)std::min<int64_t>((n8 + 255) / 256, 8192);
    const bool nt = hx::nt_stores();
    if (npieces == 3 && nt)
      split_planes_k<3, true><<<blocks, 256, 0, s>>>(x, ldx, out, R, D, npl, order, stacked);
    else if (npieces == 3)
      split_planes_k<3, false><<<blocks, 256, 0, s>>>(x, ldx, out, R, D, npl, order, stacked);
    else if (nt)
      split_planes_k<2, true><<<blocks, 256, 0, s>>>(x, ldx, out, R, D, npl, order, stacked);
    else
      split_planes_k<2, false><<<blocks, 256, 0, s>>>(x, ldx, out, R, D, npl, order, stacked);
    return;
  }
  if (!stacked && Rp == R && Dp % 8 == 0 && ldx % 2 == 0 && ((uintptr_t)x & 7) == 0) {
    const int64_t n8 = R * (Dp / 8);
    if (n8 <= 0) return;
    const int blocks = (int)std::min<int64_t>((n8 + 255) / 256, 8192);
    if (npieces == 3)
      split_planes_pad8_k<3><<<blocks, 256, 0, s>>>(x, ldx, out, R, D, Dp, npl, order);
    else
      split_planes_pad8_k<2><<<blocks, 256, 0, s>>>(x, ldx, out, R, D, Dp, npl, order);
    return;
  }
  const int64_t n = Rp * Dp;
  if (n <= 0) return;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 16384);
  if (npieces == 3)
    split_planes_any_k<3><<<blocks, 256, 0, s>>>(x, ldx, out, R, D, Rp, Dp, npl, order, stacked);
  else
    split_planes_any_k<2><<<blocks, 256, 0, s>>>(x, ldx, out, R, D, Rp, Dp, npl, order, stacked);
}

void hx_split_weight_many(const HxWeightBatch& d, int npieces, hipStream_t s) {
  if (d.n < 1 || d.start[d.n] < 1) return;
  if (npieces == 3) split_weight_many_k<3><<<d.start[d.n], 256, 0, s>>>(d);
  else split_weight_many_k<2><<<d.start[d.n], 256, 0, s>>>(d);
}

void hx_split_weight(const float* W, int N, int K, int npieces, uint16_t* wf, uint16_t* wt, hipStream_t s, int b16) {
  dim3 g(K / 64, N / 64);
  if (npieces == 3) {
    if (b16 == 3) split_weight_k<3, true, true><<<g, 256, 0, s>>>(W, N, K, wf, wt);
    else if (b16 == 1) split_weight_k<3, true, false><<<g, 256, 0, s>>>(W, N, K, wf, wt);
    else if (b16 == 2) split_weight_k<3, false, true><<<g, 256, 0, s>>>(W, N, K, wf, wt);
    else split_weight_k<3, false, false><<<g, 256, 0, s>>>(W, N, K, wf, wt);
  } else {
    split_weight_k<2, false, false><<<g, 256, 0, s>>>(W, N, K, wf, wt);
  }
}
