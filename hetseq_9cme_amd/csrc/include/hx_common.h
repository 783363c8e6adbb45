// Shared device helpers for the CDNA4 (gfx950) kernels.
//  * wave64 reductions (CDNA wavefront = 64 lanes; never warp-32 idioms)
//  * Philox4x32-10 counter-based RNG: dropout masks are a pure function of
//    (seed, stream id, element index), so the backward pass REGENERATES the mask
//    instead of storing it, and the result is independent of launch geometry.
//  * bf16 helpers (round-to-nearest-even via the hardware cvt).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdlib.h>

#define HX_WAVE 64

namespace hx {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). ``scratch`` >= NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x < 64) {
    r = (threadIdx.x < NT / 64) ? scratch[threadIdx.x] : 0.f;
    r = wave_sum(r);
    if (threadIdx.x == 0) scratch[0] = r;
  }
  __syncthreads();
  r = scratch[0];
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------- Philox4x32-10
struct u32x4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32->64 multiply per product (v_mad_u64_u32) instead of mul_hi + mul_lo
    const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// 4 uniforms in [0,1) for elements [4*q, 4*q+4) of dropout stream ``stream``.
__device__ __forceinline__ void rand4(uint64_t seed, uint64_t stream, uint64_t q, float u[4]) {
  u32x4 c{(uint32_t)q, (uint32_t)(q >> 32), (uint32_t)stream, (uint32_t)(stream >> 32)};
  u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float s = 5.9604644775390625e-08f;  // 2^-24
  u[0] = (r.x >> 8) * s;
  u[1] = (r.y >> 8) * s;
  u[2] = (r.z >> 8) * s;
  u[3] = (r.w >> 8) * s;
}

// keep-mask bits (bit j set = keep element 4q+j)
__device__ __forceinline__ uint32_t keep4(uint64_t seed, uint64_t stream, uint64_t q, float keep_prob) {
  float u[4];
  rand4(seed, stream, q, u);
  return (u[0] < keep_prob ? 1u : 0u) | (u[1] < keep_prob ? 2u : 0u) | (u[2] < keep_prob ? 4u : 0u) |
         (u[3] < keep_prob ? 8u : 0u);
}

// 8 keep decisions from ONE Philox call: 16-bit uniforms vs a 16-bit threshold
// t16 = round(keep * 65536) (keep-probability error < 2^-17).  bit j <-> decision j
// (word j>>1, low half for even j).
__device__ __forceinline__ uint32_t keep8(uint64_t seed, uint64_t stream, uint64_t q, uint32_t t16) {
  u32x4 c{(uint32_t)q, (uint32_t)(q >> 32), (uint32_t)stream, (uint32_t)(stream >> 32)};
  const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return ((r.x & 0xFFFFu) < t16 ? 1u : 0u) | ((r.x >> 16) < t16 ? 2u : 0u) | ((r.y & 0xFFFFu) < t16 ? 4u : 0u) |
         ((r.y >> 16) < t16 ? 8u : 0u) | ((r.z & 0xFFFFu) < t16 ? 16u : 0u) | ((r.z >> 16) < t16 ? 32u : 0u) |
         ((r.w & 0xFFFFu) < t16 ? 64u : 0u) | ((r.w >> 16) < t16 ? 128u : 0u);
}

// ---------------------------------------------------------------- bf16
__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&b);
}

template <typename T>
struct io;
template <>
struct io<float> {
  __device__ __forceinline__ static float ld(const float* p) { return *p; }
  __device__ __forceinline__ static void st(float* p, float v) { *p = v; }
};
template <>
struct io<uint16_t> {
  __device__ __forceinline__ static float ld(const uint16_t* p) { return bf2f(*p); }
  __device__ __forceinline__ static void st(uint16_t* p, float v) { *p = f2bf(v); }
};

// Buffer-resource IO: a scalar (SGPR) descriptor over `bytes` bytes, a per-lane 32-bit
// byte offset and a wave-uniform byte offset.  Unrolled strided loops then issue
// `buffer_load v, v_off, s[rsrc], s_off` instead of materialising one 64-bit VGPR
// address per element; loads past `bytes` return 0 and stores past it are dropped.
struct Buf {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ Buf(const void* p, uint32_t bytes)
      : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000)) {}
};
template <typename T>
struct bio;
template <>
struct bio<float> {
  __device__ __forceinline__ static float ld(const Buf& b, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b.r, voff * 4, soff * 4, 0));
  }
  __device__ __forceinline__ static void st(const Buf& b, uint32_t voff, uint32_t soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), b.r, voff * 4, soff * 4, 0);
  }
};
template <>
struct bio<uint16_t> {
  __device__ __forceinline__ static float ld(const Buf& b, uint32_t voff, uint32_t soff) {
    return bf2f(__builtin_amdgcn_raw_buffer_load_b16(b.r, voff * 2, soff * 2, 0));
  }
  __device__ __forceinline__ static void st(const Buf& b, uint32_t voff, uint32_t soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b16(f2bf(v), b.r, voff * 2, soff * 2, 0);
  }
};

// GELU as in the reference: x * 0.5 * (1 + erf(x / 1.41421))  (bert_modeling.py:104-111)
// GELU of the reference (bert_modeling.py:104-116): x/2 (1 + erf(x / 1.41421)) -- note the
// truncated sqrt(2) constant, kept for parity; the derivative below is of THAT function.
// Reciprocal constants instead of divisions (fp32 division is a ~10-instruction sequence).
__device__ __forceinline__ float gelu_f(float x) { return x * 0.5f * (1.0f + erff(x * (1.0f / 1.41421f))); }
__device__ __forceinline__ float gelu_pdf_f(float x) {   // x * d/dx of the erf term
  constexpr float inv_c2 = 1.0f / (1.41421f * 1.41421f);
  constexpr float k = 0.5f * 1.1283791670955126f / 1.41421f;   // (1/2)(2/sqrt(pi))/c
  return k * x * __expf(-(x * x) * inv_c2);
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  constexpr float inv_c = 1.0f / 1.41421f;
  const float cdf = 0.5f * (1.0f + erff(x * inv_c));
  return cdf + gelu_pdf_f(x);
}

}  // namespace hx
