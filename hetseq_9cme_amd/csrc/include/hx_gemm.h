// Low-level pieces shared by the fp16x3 GEMM kernels (gemm_f16.hip): LDS-DMA issue / retire,
// raw buffer descriptors, the 64-B-row LDS image swizzle, DPP quad transposes, and the per-tensor
// power-of-two scale of the fp16 split.
#pragma once
#include "hx_common.h"

namespace hx {
namespace g {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

// one LDS-DMA wave-instruction: 16 B per lane from buffer byte voff (zeros past the buffer's end)
// to LDS bytes [lds_addr + 16 lane, + 16); lds_addr is wave-uniform.  From asm, so the compiler
// does not drain it (vmcnt(0)) before the next LDS read; the caller retires it with a counted
// wait before the barrier that publishes the stage.  M0 is written and restored inside.
__device__ __forceinline__ void dma16(u32x4 rsrc, uint32_t lds_addr, uint32_t voff) {
  const uint32_t m = __builtin_amdgcn_readfirstlane(lds_addr);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(m), "s"(rsrc)
               : "memory");
}
template <int N>
__device__ __forceinline__ void dma_wait() {   // at most N of this wave's vector-memory ops in flight
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// raw buffer descriptor over [p, p + bytes): stride 0, reads past the end return zeros
__device__ __forceinline__ u32x4 rsrc_of(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)(size_t)p;
  return u32x4{(uint32_t)a, (uint32_t)(a >> 32) & 0xffffu, bytes, 0x00020000u};
}

// LDS image of a [rows][64 B] tile (one 16-deep k step of fp32 A, or of the two fp16 pieces of B):
// 16-B chunk ch of row r at off(r, ch).  The 16-lane groups of a ds_read_b128 fragment read (32
// consecutive rows, one chunk) hit 16 distinct 4-bank slots.  lane_src: the (row within a 1-KiB
// DMA piece, chunk) lane L fetches so that the lane-linear DMA write lands that image.
__device__ __forceinline__ int img_off(int r, int ch) { return r * 64 + 16 * (ch ^ ((r >> 2) & 3)); }
__device__ __forceinline__ void img_lane_src(int L, int& rl, int& ch) {
  rl = L >> 2;
  ch = (L & 3) ^ (L >> 4);
}

// quad permutes (DPP): value of lane (lane ^ 1) / (lane ^ 2)
__device__ __forceinline__ float qx1(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float qx2(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
}
// v[i] = row i (of 4 consecutive rows), column c = lane's column  ->  v[i] = row (lane & 3),
// column (c & ~3) + i.  Two exchange steps inside each quad of lanes.
__device__ __forceinline__ void transpose4(float (&v)[4], int lane) {
  const bool odd = lane & 1, hi = lane & 2;
  float s0 = qx1(odd ? v[0] : v[1]);
  float s2 = qx1(odd ? v[2] : v[3]);
  if (odd) {
    v[0] = s0;
    v[2] = s2;
  } else {
    v[1] = s0;
    v[3] = s2;
  }
  float t0 = qx2(hi ? v[0] : v[2]);
  float t1 = qx2(hi ? v[1] : v[3]);
  if (hi) {
    v[0] = t0;
    v[1] = t1;
  } else {
    v[2] = t0;
    v[3] = t1;
  }
}

// ---- the fp16 split: x = 2^-E (h0 + h1), h0 = fp16(2^E x), h1 = fp16(2^E x - h0), both
// round-to-nearest-even.  E puts the tensor's largest magnitude in [2^14, 2^15) (fp16 max 65504),
// so every element keeps 22 significant bits (|x - 2^-E (h0 + h1)| <= 2^-22 |x|) down to 2^-16 of
// that maximum and an absolute error below 2^-40 of it beneath.  The same amax gives the same E in
// the producer of a piece tensor (weights) and in every GEMM that undoes the scale.
__device__ __forceinline__ int f16_scale_exp(float amax) {
  if (!(amax > 0.f) || __builtin_isinf(amax)) return 0;   // zero / NaN / inf: unscaled
  int e;
  (void)frexpf(amax, &e);   // amax = m 2^e, m in [0.5, 1)
  const int E = 15 - e;
  return E < -120 ? -120 : (E > 120 ? 120 : E);
}
// max |x| over n partial maxima (any order: max is exact), every thread of the block gets it;
// red: >= blockDim.x / 64 floats of LDS
__device__ __forceinline__ float block_amax(const float* __restrict__ p, int n, float* red) {
  float m = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) m = fmaxf(m, p[i]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = m;
  __syncthreads();
  m = red[0];
  for (int i = 1; i < nw; ++i) m = fmaxf(m, red[i]);
  return m;
}
// 8 fp32 values (already scaled) -> their two fp16 pieces
__device__ __forceinline__ void split2(const f32x8 y, f16x8& h0, f16x8& h1) {
  h0 = __builtin_convertvector(y, f16x8);
  h1 = __builtin_convertvector(y - __builtin_convertvector(h0, f32x8), f16x8);
}

// 4 consecutive fp32 values of a row (columns c .. c + 3, c % 4 == 0) -> their two pieces at scale
// s, into the row's P2 image (piece p of column c at (c / 16) 32 + p 16 + c % 16): two 8-B stores.
// Bit-identical to the GEMM's in-register split (s x is exact; the residual is exact in fp32).
__device__ __forceinline__ void store_p2x4(uint16_t* __restrict__ row, int c, float4 v, float s) {
  const float x[4] = {v.x * s, v.y * s, v.z * s, v.w * s};
  uint32_t q0[2], q1[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const _Float16 a0 = (_Float16)x[2 * j], b0 = (_Float16)x[2 * j + 1];
    const _Float16 a1 = (_Float16)(x[2 * j] - (float)a0), b1 = (_Float16)(x[2 * j + 1] - (float)b0);
    q0[j] = __builtin_bit_cast(uint16_t, a0) | ((uint32_t)__builtin_bit_cast(uint16_t, b0) << 16);
    q1[j] = __builtin_bit_cast(uint16_t, a1) | ((uint32_t)__builtin_bit_cast(uint16_t, b1) << 16);
  }
  uint16_t* p = row + (c >> 4) * 32 + (c & 15);
  *reinterpret_cast<uint2*>(p) = make_uint2(q0[0], q0[1]);
  *reinterpret_cast<uint2*>(p + 16) = make_uint2(q1[0], q1[1]);
}

}  // namespace g
}  // namespace hx
