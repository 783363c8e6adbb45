// Fused scaled-dot-product attention on bf16 matrix cores (v_mfma_f32_32x32x16_bf16,
// fp32 accumulate) for ``--precision bf16`` (reference math: hetseq/bert_modeling.py:351-377,
// SURVEY K04-K08).  The fp32 kernels (attention.hip) run fp32 MFMA at 1/16 of this
// rate; with bf16 activations the products can use bf16 operands directly.
//
// Forward, one workgroup = 4 waves x 32 queries, 64-key tiles, same "swapped"
// orientation as the fp32 kernel so the softmax row of a query lives in one lane pair:
//   S^T = K . Q^T     A = K rows (LDS, ds_read_b128), B = Q held in 4 bf16x8 VGPR fragments
//   O^T += V^T . P^T  B = the probability ACCUMULATOR packed to bf16 in place (no LDS trip)
// The 32x32x16 B operand wants, in lane half h, 8 consecutive k-slots; the accumulator
// holds keys crow(r, h) = (r&3) + 8(r>>2) + 4h in register r.  Instead of moving P
// between lanes, the k-slot -> key assignment of the PV product follows the
// accumulator: slot (group g, half h, element j) = key 16g + crow(8(g&1) + j, h) - ..,
// and V is staged into LDS TRANSPOSED with its keys permuted the same way
// (vpos() below), so each A fragment is one 16-B ds_read_b128 of a [dim][key] row.
//
// * K/V tiles double-buffered in LDS, the next tile's global loads in flight
//   (registers) during the current tile's math: one barrier per tile;
// * exp2 with the log2(e) scale folded into one FMA per probability;
// * dropout: the fp32 kernel's Philox counters and transposed [key][query-word]
//   bitmask (hx_attn.h), so masks do not depend on the activation precision;
// * QKV-projection bias added at load (fp32 add, one bf16 rounding -- what a bias
//   epilogue on the bf16 GEMM would produce).
#include "hx_launch.h"
#include "hx_vec.h"
#include "hx_attn.h"

namespace {

using hx::attn::crow;
using hx::attn::drop_step;
using hx::attn::f32x16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

constexpr int D = 64;
constexpr int RS = 72;   // LDS row stride (bf16): 144-B rows -> the 16 lanes of a b128 read group hit 16 slots
constexpr float L2E = 1.4426950408889634f;

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void unpack8(const uint4 v, float (&f)[8]) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ bf16x8 pack8(const float (&f)[8]) {
  const f32x8 v = {f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7]};
  return __builtin_convertvector(v, bf16x8);   // v_cvt_pk_bf16_f32 (RNE)
}
__device__ __forceinline__ uint4 as_u4(bf16x8 v) { return *reinterpret_cast<uint4*>(&v); }
template <int O>
__device__ __forceinline__ bf16x8 pack_acc(const f32x16& s) {
  const f32x8 v = {s[O], s[O + 1], s[O + 2], s[O + 3], s[O + 4], s[O + 5], s[O + 6], s[O + 7]};
  return __builtin_convertvector(v, bf16x8);
}
// 8 bf16 (+ fp32 bias) -> bf16x8 bits
__device__ __forceinline__ uint4 add_bias8(uint4 raw, const float* bp) {
  float f[8];
  unpack8(raw, f);
  const float4 b0 = *reinterpret_cast<const float4*>(bp), b1 = *reinterpret_cast<const float4*>(bp + 4);
  f[0] += b0.x; f[1] += b0.y; f[2] += b0.z; f[3] += b0.w;
  f[4] += b1.x; f[5] += b1.y; f[6] += b1.z; f[7] += b1.w;
  return as_u4(pack8(f));
}
// 4 bf16 (+ fp32 bias) -> 4 bf16 bits
__device__ __forceinline__ uint2 add_bias4(uint2 raw, const float* bp) {
  const float4 bb = *reinterpret_cast<const float4*>(bp);
  const float a0 = __uint_as_float(raw.x << 16) + bb.x, a1 = __uint_as_float(raw.x & 0xffff0000u) + bb.y;
  const float a2 = __uint_as_float(raw.y << 16) + bb.z, a3 = __uint_as_float(raw.y & 0xffff0000u) + bb.w;
  return make_uint2((uint32_t)hx::f2bf(a0) | ((uint32_t)hx::f2bf(a1) << 16),
                    (uint32_t)hx::f2bf(a2) | ((uint32_t)hx::f2bf(a3) << 16));
}

// key k (0..63 of a tile) -> its column in the transposed, permuted V image
__device__ __forceinline__ int vpos(int k) {
  const int kk = k & 15;
  return (k & ~15) + 8 * ((kk >> 2) & 1) + (kk & 3) + 4 * (kk >> 3);
}

// ============================================================================ forward
// grid (ceil(S/128), nh, B), block 256 = 4 waves x 32 queries.
template <bool kDrop>
__global__ __launch_bounds__(256) void attn_fwd_bf16_k(const uint16_t* __restrict__ qkv,
                                                       const float* __restrict__ qkv_bias,
                                                       const float* __restrict__ maskb, uint16_t* __restrict__ out,
                                                       float* __restrict__ lse, uint32_t* __restrict__ dmask, int S,
                                                       int nh, float keep, const uint64_t* __restrict__ seedp, uint64_t stream) {
  const uint64_t seed = *seedp;   // per-update Philox key, device-resident (graph-safe)
  __shared__ __attribute__((aligned(16))) uint16_t Ks[2][64 * RS];   // [key][dim]
  __shared__ __attribute__((aligned(16))) uint16_t Vt[2][64 * RS];   // [dim][vpos(key)]
  __shared__ float Ms[2][64];
  constexpr int kMaxStagedTiles = 8;   // S <= 512: mask words staged, stored after the loop
  __shared__ uint32_t Wst[kDrop ? kMaxStagedTiles * 256 : 1];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.z, hd = blockIdx.y;
  const int H = nh * D, H3 = 3 * H;
  const int q = blockIdx.x * 128 + w * 32 + l32;
  const int qc = q < S ? q : S - 1;            // rows past S: clamped loads, no stores
  const int Sp = (S + 127) & ~127;
  const int q0w = blockIdx.x * 128 + w * 32;
  const uint32_t t16 = (uint32_t)(keep * 65536.f + 0.5f);
  const float inv_keep = 1.f / keep;
  const uint16_t* base = qkv + (int64_t)b * S * H3 + hd * D;
  const int64_t bh = (int64_t)b * nh + hd;
  const float* kbias = qkv_bias ? qkv_bias + H + hd * D : nullptr;
  const float* vbias = qkv_bias ? qkv_bias + 2 * H + hd * D : nullptr;

  // Q fragments: lane (query, half h), fragment ks = dims 16ks + 8h .. +7, scaled by 1/8 (exact)
  bf16x8 qf[4];
  {
    const uint16_t* qp = base + (int64_t)qc * H3 + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(qp + 16 * ks), f);
      if (qkv_bias) {
        const float* bp = qkv_bias + hd * D + 16 * ks + 8 * h;
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += bp[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= 0.125f;
      qf[ks] = pack8(f);
    }
  }

  // ---- tile staging: K rows (2 x 16 B per thread), V key pairs x 4 dims (2 x 2 x 8 B)
  uint4 kr[2];
  uint2 vr[2][2];
  float mr = 0.f;
  auto stage_load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i, row = e >> 3, c8 = (e & 7) * 8;
      const int key = kt + row < S ? kt + row : S - 1;
      kr[i] = *reinterpret_cast<const uint4*>(base + (int64_t)key * H3 + H + c8);
      const int dq = e & 15, kp = e >> 4;
      const int k0 = kt + 2 * kp < S ? kt + 2 * kp : S - 1, k1 = kt + 2 * kp + 1 < S ? kt + 2 * kp + 1 : S - 1;
      vr[i][0] = *reinterpret_cast<const uint2*>(base + (int64_t)k0 * H3 + 2 * H + 4 * dq);
      vr[i][1] = *reinterpret_cast<const uint2*>(base + (int64_t)k1 * H3 + 2 * H + 4 * dq);
    }
    if (tid < 64) mr = kt + tid < S ? maskb[(int64_t)b * S + kt + tid] : -INFINITY;
  };
  auto stage_store = [&](int cb) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i, row = e >> 3, c8 = (e & 7) * 8;
      uint4 kv = kr[i];
      if (kbias) kv = add_bias8(kv, kbias + c8);
      *reinterpret_cast<uint4*>(&Ks[cb][row * RS + c8]) = kv;
      const int dq = e & 15, kp = e >> 4;
      uint2 v0 = vr[i][0], v1 = vr[i][1];
      if (vbias) {
        v0 = add_bias4(v0, vbias + 4 * dq);
        v1 = add_bias4(v1, vbias + 4 * dq);
      }
      uint32_t* vt = reinterpret_cast<uint32_t*>(&Vt[cb][(4 * dq) * RS + vpos(2 * kp)]);
      constexpr int RW = RS / 2;   // row stride in 32-bit words
      vt[0] = (v0.x & 0xffffu) | (v1.x << 16);
      vt[RW] = (v0.x >> 16) | (v1.x & 0xffff0000u);
      vt[2 * RW] = (v0.y & 0xffffu) | (v1.y << 16);
      vt[3 * RW] = (v0.y >> 16) | (v1.y & 0xffff0000u);
    }
    if (tid < 64) Ms[cb][tid] = mr;
  };

  f32x16 o0 = {0}, o1 = {0};
  float m_run = -INFINITY, l_run = 0.f;
  const int nt = (S + 63) >> 6;
  stage_load(0);
  stage_store(0);
  __syncthreads();

  for (int t = 0; t < nt; ++t) {
    const int kt = t * 64, cb = t & 1;
    if (t + 1 < nt) stage_load(kt + 64);   // in flight during this tile's math

    uint32_t keepbits[4] = {0u, 0u, 0u, 0u};
    if (kDrop) {
      // Philox chain first: it has no input from the tile's math and fills the MFMA shadow
      const uint64_t cbase = hx::attn::drop_counter(bh, S, q, Sp, kt, h);
#pragma unroll
      for (int j = 0; j < 4; ++j) keepbits[j] = hx::keep8(seed, stream, cbase + j, t16);
    }
    // ---- S^T = K . Q^T, two 32-key blocks; keys on the accumulator rows, queries on lanes
    f32x16 s0 = {0}, s1 = {0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 ka = *reinterpret_cast<const bf16x8*>(&Ks[cb][l32 * RS + 16 * ks + 8 * h]);
      const bf16x8 kb = *reinterpret_cast<const bf16x8*>(&Ks[cb][(32 + l32) * RS + 16 * ks + 8 * h]);
      s0 = mfma(ka, qf[ks], s0);
      s1 = mfma(kb, qf[ks], s1);
    }
    // + mask, running max, exp2, row sum
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s0[r] += Ms[cb][crow(r, h)];
      s1[r] += Ms[cb][32 + crow(r, h)];
      mx = fmaxf(mx, fmaxf(s0[r], s1[r]));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * L2E);
    const float mL = m_new * L2E;
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s0[r] = __builtin_amdgcn_exp2f(fmaf(s0[r], L2E, -mL));
      s1[r] = __builtin_amdgcn_exp2f(fmaf(s1[r], L2E, -mL));
      rs += s0[r] + s1[r];
    }
    rs += __shfl_xor(rs, 32, 64);
    l_run = l_run * alpha + rs;
    m_run = m_new;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      o0[r] *= alpha;
      o1[r] *= alpha;
    }
    if (kDrop) {
      uint32_t myword = 0;
      drop_step<0>(s0, s1, keepbits, inv_keep, myword);
      if (Sp <= kMaxStagedTiles * 64)
        Wst[t * 256 + w * 64 + lane] = myword;
      else
        dmask[((int64_t)bh * Sp + kt + lane) * (Sp >> 5) + (q0w >> 5)] = myword;
    }
    // ---- O^T += V^T . P^T : P packed to bf16 in place, V^T rows from the transposed image
    const bf16x8 p0 = pack_acc<0>(s0), p1 = pack_acc<8>(s0), p2 = pack_acc<0>(s1), p3 = pack_acc<8>(s1);
    const uint16_t* v0r = &Vt[cb][l32 * RS + 8 * h];
    const uint16_t* v1r = &Vt[cb][(32 + l32) * RS + 8 * h];
    o0 = mfma(*reinterpret_cast<const bf16x8*>(v0r), p0, o0);
    o1 = mfma(*reinterpret_cast<const bf16x8*>(v1r), p0, o1);
    o0 = mfma(*reinterpret_cast<const bf16x8*>(v0r + 16), p1, o0);
    o1 = mfma(*reinterpret_cast<const bf16x8*>(v1r + 16), p1, o1);
    o0 = mfma(*reinterpret_cast<const bf16x8*>(v0r + 32), p2, o0);
    o1 = mfma(*reinterpret_cast<const bf16x8*>(v1r + 32), p2, o1);
    o0 = mfma(*reinterpret_cast<const bf16x8*>(v0r + 48), p3, o0);
    o1 = mfma(*reinterpret_cast<const bf16x8*>(v1r + 48), p3, o1);
    if (t + 1 < nt) stage_store(cb ^ 1);   // the other buffer: every wave left it at the last barrier
    __syncthreads();
  }

  // ---- epilogue
  if (kDrop && Sp <= kMaxStagedTiles * 64) {
    for (int t = 0; t < nt; ++t)
      dmask[((int64_t)bh * Sp + t * 64 + lane) * (Sp >> 5) + (q0w >> 5)] = Wst[t * 256 + w * 64 + lane];
  }
  if (q >= S) return;
  const float inv_l = 1.f / l_run;
  uint16_t* op = out + ((int64_t)b * S + q) * H + hd * D;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d0 = 8 * g + 4 * h;
    hx::store4(op + d0, make_float4(o0[4 * g] * inv_l, o0[4 * g + 1] * inv_l, o0[4 * g + 2] * inv_l,
                                    o0[4 * g + 3] * inv_l));
    hx::store4(op + 32 + d0, make_float4(o1[4 * g] * inv_l, o1[4 * g + 1] * inv_l, o1[4 * g + 2] * inv_l,
                                         o1[4 * g + 3] * inv_l));
  }
  if (h == 0) lse[bh * S + q] = m_run + __logf(l_run);
}

// ============================================================================ backward
// grid (ceil(S/128), nh, B), block 256 = 4 waves; wave w owns keys kbase + 32w .. +31 ON THE
// LANES for the whole kernel (its K and V rows live in registers as bf16 fragments) and the
// workgroup sweeps 32-query tiles:
//   S  = Qs . K^T,  dP = dO . V^T         (32x32x16: A = LDS rows of the tile, B = key registers)
//   P  = exp2(S log2e + (mask - lse) log2e),  Pd = P drop/keep,  dS = P (dP drop/keep - D)
//   dV += Pd^T . dO,  dK += dS^T . Qs       (A = the P / dS accumulators packed to bf16 in place;
//                                            B = transposed, query-permuted images of dO / Q)
//   dQ  = dS . K over the block's 128 keys (16x16x32: dS through LDS once, K^T image; each
//                                            wave owns two of the eight 16x16 output tiles)
// D = rowsum(dO * O) is formed while staging the tile; the next tile's Q / dO / O / lse /
// dropout word are loaded into registers during the current tile's math.
constexpr int TS = 40;    // transposed 32-query image row stride (bf16): 80-B rows, conflict-free b128
constexpr int KTS = 136;  // K^T [dim][128 keys] and dS [query][128 keys] row stride (bf16)

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// 4 bf16 of one row (+ optional fp32 bias) * scale -> 4 bf16 (two words)
__device__ __forceinline__ uint2 prep4(uint2 raw, const float* bp, float scale) {
  float a0 = __uint_as_float(raw.x << 16), a1 = __uint_as_float(raw.x & 0xffff0000u);
  float a2 = __uint_as_float(raw.y << 16), a3 = __uint_as_float(raw.y & 0xffff0000u);
  if (bp) {
    const float4 bb = *reinterpret_cast<const float4*>(bp);
    a0 += bb.x; a1 += bb.y; a2 += bb.z; a3 += bb.w;
  }
  return make_uint2((uint32_t)hx::f2bf(a0 * scale) | ((uint32_t)hx::f2bf(a1 * scale) << 16),
                    (uint32_t)hx::f2bf(a2 * scale) | ((uint32_t)hx::f2bf(a3 * scale) << 16));
}
// rows r0, r1 (consecutive image positions) x 4 dims -> 4 words of a transposed image
__device__ __forceinline__ void put_t4(uint16_t* img, int stride, int dim0, int pos, uint2 r0, uint2 r1) {
  uint32_t* p = reinterpret_cast<uint32_t*>(img + dim0 * stride + pos);
  const int sw = stride / 2;
  p[0] = (r0.x & 0xffffu) | (r1.x << 16);
  p[sw] = (r0.x >> 16) | (r1.x & 0xffff0000u);
  p[2 * sw] = (r0.y & 0xffffu) | (r1.y << 16);
  p[3 * sw] = (r0.y >> 16) | (r1.y & 0xffff0000u);
}
__device__ __forceinline__ float dot4(uint2 a, uint2 b) {
  return __uint_as_float(a.x << 16) * __uint_as_float(b.x << 16) +
         __uint_as_float(a.x & 0xffff0000u) * __uint_as_float(b.x & 0xffff0000u) +
         __uint_as_float(a.y << 16) * __uint_as_float(b.y << 16) +
         __uint_as_float(a.y & 0xffff0000u) * __uint_as_float(b.y & 0xffff0000u);
}

template <bool kDrop>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_bwd_bf16_k(
    const uint16_t* __restrict__ qkv, const float* __restrict__ qkv_bias, float* __restrict__ dbias_part,
    const float* __restrict__ maskb, const uint16_t* __restrict__ dout, const uint16_t* __restrict__ outp,
    const float* __restrict__ lse, const uint32_t* __restrict__ dmask, uint16_t* __restrict__ dqkv,
    float* __restrict__ dq_acc, int dq_ld, int S, int nh, float keep) {
  __shared__ __attribute__((aligned(16))) uint16_t Kt[64 * KTS];    // K^T of the block's 128 keys
  __shared__ __attribute__((aligned(16))) uint16_t dSs[32 * KTS];   // dS [query][key] (bf16)
  __shared__ __attribute__((aligned(16))) uint16_t Qs[32 * RS];     // pre-scaled Q tile, rows
  __shared__ __attribute__((aligned(16))) uint16_t dOs[32 * RS];    // dO tile, rows
  __shared__ __attribute__((aligned(16))) uint16_t Qt[64 * TS];     // Q^T, queries permuted (vpos)
  __shared__ __attribute__((aligned(16))) uint16_t dOt[64 * TS];    // dO^T, queries permuted
  __shared__ float LsL[32], Ds[32];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.z, hd = blockIdx.y;
  const int H = nh * D, H3 = 3 * H;
  const int kbase = blockIdx.x * 128;
  const bool single = gridDim.x == 1;
  const int64_t bh = (int64_t)b * nh + hd;
  const float scale = 0.125f, inv_keep = 1.f / keep;
  const int Sp = (S + 127) & ~127;
  const int nwords = Sp >> 5;
  const uint16_t* base = qkv + (int64_t)b * S * H3 + hd * D;
  const float* qbias = qkv_bias ? qkv_bias + hd * D : nullptr;
  const float* kbias = qkv_bias ? qkv_bias + H + hd * D : nullptr;
  const float* vbias = qkv_bias ? qkv_bias + 2 * H + hd * D : nullptr;

  // ---- K^T image of the 128 keys (natural key order) for dQ: 64 key pairs x 16 dim quads
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = tid + 256 * i, dq = u & 15, kp = u >> 4;
    const int k0 = kbase + 2 * kp < S ? kbase + 2 * kp : S - 1;
    const int k1 = kbase + 2 * kp + 1 < S ? kbase + 2 * kp + 1 : S - 1;
    const uint2 r0 = prep4(*reinterpret_cast<const uint2*>(base + (int64_t)k0 * H3 + H + 4 * dq),
                           kbias ? kbias + 4 * dq : nullptr, 1.f);
    const uint2 r1 = prep4(*reinterpret_cast<const uint2*>(base + (int64_t)k1 * H3 + H + 4 * dq),
                           kbias ? kbias + 4 * dq : nullptr, 1.f);
    put_t4(Kt, KTS, 4 * dq, 2 * kp, r0, r1);
  }
  // ---- this lane's key: K and V fragments (B operands of S and dP), dims 16ks + 8h .. +7
  const int mykey = kbase + w * 32 + l32;
  const int mykc = mykey < S ? mykey : S - 1;
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int c = 16 * ks + 8 * h;
    uint4 kr = *reinterpret_cast<const uint4*>(base + (int64_t)mykc * H3 + H + c);
    uint4 vr = *reinterpret_cast<const uint4*>(base + (int64_t)mykc * H3 + 2 * H + c);
    if (kbias) kr = add_bias8(kr, kbias + c);
    if (vbias) vr = add_bias8(vr, vbias + c);
    kf[ks] = *reinterpret_cast<bf16x8*>(&kr);
    vf[ks] = *reinterpret_cast<bf16x8*>(&vr);
  }
  const float mkL = (mykey < S ? maskb[(int64_t)b * S + mykey] : -INFINITY) * L2E;

  const uint16_t* dout_b = dout + (int64_t)b * S * H + hd * D;
  const uint16_t* out_b = outp + (int64_t)b * S * H + hd * D;
  uint16_t* dqkv_b = dqkv + (int64_t)b * S * H3 + hd * D;
  float* dqa_b = dq_acc ? dq_acc + (int64_t)b * S * dq_ld + hd * D : nullptr;
  const float* lse_bh = lse + bh * S;
  const uint32_t* dmask_bh = kDrop ? dmask + bh * Sp * nwords : nullptr;
  const int moff = mykey * nwords;

  // staging unit of this thread: query pair (2qp, 2qp+1) x dims 4dq .. 4dq+3
  const int sdq = tid & 15, sqp = tid >> 4;
  uint2 pq[2], pd[2], po[2];
  float pl = 0.f;
  uint32_t pm = 0;
  auto ld_tile = [&](int qt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int qr = qt + 2 * sqp + i;
      const int r = qr < S ? qr : S - 1;
      pq[i] = *reinterpret_cast<const uint2*>(base + (int64_t)r * H3 + 4 * sdq);
      pd[i] = *reinterpret_cast<const uint2*>(dout_b + (int64_t)r * H + 4 * sdq);
      po[i] = *reinterpret_cast<const uint2*>(out_b + (int64_t)r * H + 4 * sdq);
    }
    const int lq = qt + (tid & 31);
    pl = lse_bh[lq < S ? lq : S - 1];
    if (kDrop) pm = dmask_bh[moff + (qt >> 5)];
  };
  ld_tile(0);

  // dQ tiles of this wave (16x16x32 layout): queries 16qh .., dims 32dp2 .. and 32dp2 + 16 ..
  const int qh = w & 1, dp2 = w >> 1;
  const int r16 = lane & 15, kg = lane >> 4;

  f32x16 dv0 = {0}, dv1 = {0}, dk0 = {0}, dk1 = {0};
  float cq0 = 0.f, cq1 = 0.f;

  for (int qt = 0; qt < S; qt += 32) {
    __syncthreads();   // the previous tile's images and dS are free
    {
      const uint2 q0 = prep4(pq[0], qbias ? qbias + 4 * sdq : nullptr, scale);
      const uint2 q1 = prep4(pq[1], qbias ? qbias + 4 * sdq : nullptr, scale);
      *reinterpret_cast<uint2*>(&Qs[(2 * sqp) * RS + 4 * sdq]) = q0;
      *reinterpret_cast<uint2*>(&Qs[(2 * sqp + 1) * RS + 4 * sdq]) = q1;
      *reinterpret_cast<uint2*>(&dOs[(2 * sqp) * RS + 4 * sdq]) = pd[0];
      *reinterpret_cast<uint2*>(&dOs[(2 * sqp + 1) * RS + 4 * sdq]) = pd[1];
      const int pos = vpos(2 * sqp);
      put_t4(Qt, TS, 4 * sdq, pos, q0, q1);
      put_t4(dOt, TS, 4 * sdq, pos, pd[0], pd[1]);
      float d0 = dot4(pd[0], po[0]), d1 = dot4(pd[1], po[1]);
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        d0 += __shfl_xor(d0, o, 64);
        d1 += __shfl_xor(d1, o, 64);
      }
      if (sdq == 0) {
        Ds[2 * sqp] = d0;
        Ds[2 * sqp + 1] = d1;
      }
      if (tid < 32) LsL[tid] = qt + tid < S ? pl * L2E : INFINITY;   // rows past S: P = 0
    }
    const uint32_t mword = pm;
    if (qt + 32 < S) ld_tile(qt + 32);   // in flight during this tile's math
    __syncthreads();

    // ---- S = Qs . K^T, dP = dO . V^T (queries on accumulator rows, keys on lanes)
    f32x16 sa = {0}, dpa = {0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 qa = *reinterpret_cast<const bf16x8*>(&Qs[l32 * RS + 16 * ks + 8 * h]);
      const bf16x8 da = *reinterpret_cast<const bf16x8*>(&dOs[l32 * RS + 16 * ks + 8 * h]);
      sa = mfma(qa, kf[ks], sa);
      dpa = mfma(da, vf[ks], dpa);
    }
    // ---- P, Pd, dS in place; dS also to LDS ([query][key], bf16) for dQ
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qr = crow(r, h);
      const float p = __builtin_amdgcn_exp2f(fmaf(sa[r], L2E, mkL - LsL[qr]));
      float keepf = 1.f;
      if (kDrop) keepf = ((mword >> qr) & 1) ? inv_keep : 0.f;
      sa[r] = p * keepf;
      dpa[r] = p * (dpa[r] * keepf - Ds[qr]);
      dSs[qr * KTS + w * 32 + l32] = hx::f2bf(dpa[r]);
    }
    // ---- dV += Pd^T . dO, dK += dS^T . Qs (k-slots = the accumulator's query rows)
    {
      const bf16x8 pa0 = pack_acc<0>(sa), pa1 = pack_acc<8>(sa);
      const bf16x8 sa0 = pack_acc<0>(dpa), sa1 = pack_acc<8>(dpa);
      const uint16_t* dt0 = &dOt[l32 * TS + 8 * h];
      const uint16_t* dt1 = &dOt[(32 + l32) * TS + 8 * h];
      const uint16_t* qt0 = &Qt[l32 * TS + 8 * h];
      const uint16_t* qt1 = &Qt[(32 + l32) * TS + 8 * h];
      dv0 = mfma(pa0, *reinterpret_cast<const bf16x8*>(dt0), dv0);
      dv1 = mfma(pa0, *reinterpret_cast<const bf16x8*>(dt1), dv1);
      dk0 = mfma(sa0, *reinterpret_cast<const bf16x8*>(qt0), dk0);
      dk1 = mfma(sa0, *reinterpret_cast<const bf16x8*>(qt1), dk1);
      dv0 = mfma(pa1, *reinterpret_cast<const bf16x8*>(dt0 + 16), dv0);
      dv1 = mfma(pa1, *reinterpret_cast<const bf16x8*>(dt1 + 16), dv1);
      dk0 = mfma(sa1, *reinterpret_cast<const bf16x8*>(qt0 + 16), dk0);
      dk1 = mfma(sa1, *reinterpret_cast<const bf16x8*>(qt1 + 16), dk1);
    }
    __syncthreads();   // every wave's dS columns are in LDS
    // ---- dQ = dS . K over the block's 128 keys
    f32x4 qa0 = {0.f, 0.f, 0.f, 0.f}, qa1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(&dSs[(qh * 16 + r16) * KTS + 32 * ks + 8 * kg]);
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(&Kt[(32 * dp2 + r16) * KTS + 32 * ks + 8 * kg]);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(&Kt[(32 * dp2 + 16 + r16) * KTS + 32 * ks + 8 * kg]);
      qa0 = mfma16(a, b0, qa0);
      qa1 = mfma16(a, b1, qa1);
    }
    const int q0 = qt + qh * 16 + 4 * kg;
    if (dbias_part) {   // rows past S hold exact zeros (their P, hence dS, is 0)
      cq0 += (qa0[0] + qa0[1]) + (qa0[2] + qa0[3]);
      cq1 += (qa1[0] + qa1[1]) + (qa1[2] + qa1[3]);
    }
    const int dcol = 32 * dp2 + r16;
    if (single) {
      uint16_t* dq = dqkv_b + (int64_t)q0 * H3 + dcol;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (q0 + r >= S) continue;
        dq[r * H3] = hx::f2bf(qa0[r] * scale);
        dq[r * H3 + 16] = hx::f2bf(qa1[r] * scale);
      }
    } else {
      float* dq = dqa_b + (int64_t)q0 * dq_ld + dcol;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (q0 + r >= S) continue;
        atomicAdd(dq + r * dq_ld, qa0[r] * scale);
        atomicAdd(dq + r * dq_ld + 16, qa1[r] * scale);
      }
    }
  }
  // ---- epilogue: dK (accumulated against pre-scaled Q: already scaled), dV
  uint16_t* dk = dqkv + (int64_t)b * S * H3 + H + hd * D;
  uint16_t* dvp = dqkv + (int64_t)b * S * H3 + 2 * H + hd * D;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int key = kbase + w * 32 + crow(r, h);
    if (key >= S) continue;
    dk[(int64_t)key * H3 + l32] = hx::f2bf(dk0[r]);
    dk[(int64_t)key * H3 + 32 + l32] = hx::f2bf(dk1[r]);
    dvp[(int64_t)key * H3 + l32] = hx::f2bf(dv0[r]);
    dvp[(int64_t)key * H3 + 32 + l32] = hx::f2bf(dv1[r]);
  }
  if (dbias_part) {
    // QKV-bias gradient = column sums of dQ, dK, dV (as in attention.hip): one row of 3H
    // partials per (batch, key block), folded into the bias-grad slots afterwards
    float sk0 = 0.f, sk1 = 0.f, sv0 = 0.f, sv1 = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sk0 += dk0[r]; sk1 += dk1[r]; sv0 += dv0[r]; sv1 += dv1[r];
    }
    sk0 += __shfl_xor(sk0, 32, 64); sk1 += __shfl_xor(sk1, 32, 64);
    sv0 += __shfl_xor(sv0, 32, 64); sv1 += __shfl_xor(sv1, 32, 64);
    cq0 += __shfl_xor(cq0, 16, 64); cq0 += __shfl_xor(cq0, 32, 64);
    cq1 += __shfl_xor(cq1, 16, 64); cq1 += __shfl_xor(cq1, 32, 64);
    cq0 *= scale;
    cq1 *= scale;
    __syncthreads();   // every wave is done with dSs
    float* red = reinterpret_cast<float*>(dSs);   // [4 waves][3][64] floats (3 KB of the 8.5 KB)
    if (lane < 32) {
      red[(w * 3 + 1) * 64 + l32] = sk0; red[(w * 3 + 1) * 64 + 32 + l32] = sk1;
      red[(w * 3 + 2) * 64 + l32] = sv0; red[(w * 3 + 2) * 64 + 32 + l32] = sv1;
    }
    if (lane < 16) {   // dQ columns 32dp2 + lane and 32dp2 + 16 + lane of this wave's query half
      red[(w * 3) * 64 + 32 * dp2 + lane] = cq0;
      red[(w * 3) * 64 + 32 * dp2 + 16 + lane] = cq1;
    }
    __syncthreads();
    if (tid < 192) {
      const int part = tid >> 6, c = tid & 63;
      float v;
      if (part == 0) {   // waves (0,1) own dQ columns 0..31, waves (2,3) own 32..63
        const int wa = c < 32 ? 0 : 2;
        v = red[(wa * 3) * 64 + c] + red[((wa + 1) * 3) * 64 + c];
      } else {
        v = (red[(0 * 3 + part) * 64 + c] + red[(1 * 3 + part) * 64 + c]) +
            (red[(2 * 3 + part) * 64 + c] + red[(3 * 3 + part) * 64 + c]);
      }
      dbias_part[((int64_t)b * gridDim.x + blockIdx.x) * H3 + part * H + hd * D + c] = v;
    }
  }
}

}  // namespace

void hx_attn_bwd_bf16(const void* qkv, const float* bias, float* dbias_part, const float* maskb, const void* dout,
                      const void* out, const float* lse, const uint32_t* dmask, void* dqkv, float* dq_acc, int dq_ld,
                      int B, int S, int nh, float keep, hipStream_t s) {
  dim3 grid((S + 127) / 128, nh, B);
  if (keep < 1.f)
    attn_bwd_bf16_k<true><<<grid, 256, 0, s>>>((const uint16_t*)qkv, bias, dbias_part, maskb, (const uint16_t*)dout,
                                               (const uint16_t*)out, lse, dmask, (uint16_t*)dqkv, dq_acc, dq_ld, S,
                                               nh, keep);
  else
    attn_bwd_bf16_k<false><<<grid, 256, 0, s>>>((const uint16_t*)qkv, bias, dbias_part, maskb,
                                                (const uint16_t*)dout, (const uint16_t*)out, lse, dmask,
                                                (uint16_t*)dqkv, dq_acc, dq_ld, S, nh, keep);
}

void hx_attn_fwd_bf16(const void* qkv, const float* bias, const float* maskb, void* out, float* lse, uint32_t* dmask,
                      int B, int S, int nh, float keep, const uint64_t* seed, uint64_t stream, hipStream_t s) {
  dim3 grid((S + 127) / 128, nh, B);
  if (keep < 1.f)
    attn_fwd_bf16_k<true><<<grid, 256, 0, s>>>((const uint16_t*)qkv, bias, maskb, (uint16_t*)out, lse, dmask, S, nh,
                                               keep, seed, stream);
  else
    attn_fwd_bf16_k<false><<<grid, 256, 0, s>>>((const uint16_t*)qkv, bias, maskb, (uint16_t*)out, lse, dmask, S,
                                                nh, keep, seed, stream);
}
