// fp32 attention forward on the bf16 matrix cores (--fp32-gemm bf16x3 / bf16x6).
//
// Same math and I/O as the fp32-MFMA forward (attention.hip: reference
// hetseq/bert_modeling.py:351-377; packed fp32 [B, S, 3H] QKV in, fp32
// [B, S, H] context + per-query logsumexp + transposed dropout bitmask out), but every
// product runs as bf16 x bf16 -> fp32 MFMAs on split operands (ops/split_gemm.py,
// split.hip): x = x0 + x1 + x2 (bf16 pieces, round-to-nearest each, |x - sum| <= 2^-26 |x|),
// and a dot product is the sum of the six piece products with i + j <= 2, each exact in the
// fp32 accumulator -- the "bf16x6" fp32-exact class.  v_mfma_f32_32x32x16_bf16 does 8x the
// k-depth of v_mfma_f32_32x32x2_f32 in half its cycles, so 6 passes cost ~3/8 of the fp32
// MFMA time.
//
// Structure (the bf16 kernel's, attention_bf16.hip, with pieces):
//  * one workgroup = 4 waves x 32 queries ON THE LANES, 64-key tiles, keys on the
//    accumulator rows: S^T = K . Q^T with Q's three piece fragments held in VGPRs;
//  * K is staged into LDS as three bf16 piece images [key][dim], V as three TRANSPOSED
//    piece images [dim][vpos(key)] whose key order follows the probability accumulator,
//    so O^T += V^T . P^T takes P's pieces straight from the accumulator (no LDS trip);
//  * the pieces are formed once per element while staging (fp32 loads + bias, split),
//    single-buffered (55 KiB: two workgroups per CU) with the next tile's fp32 loads in
//    flight in registers during the current tile's math;
//  * softmax, dropout (same Philox counters and bitmask as the other kernels), lse and
//    the epilogue are the fp32 kernel's.
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
constexpr int RS = 72;   // LDS row stride (bf16): 144-B rows, conflict-free 16-B fragment reads

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// (a, b) -> one word of their bf16 roundings (a low, b high); a and b become the residuals.
// The round trip back to fp32 is bit placement on the packed word: the compiler would
// otherwise re-convert each value on its own for the subtraction.
__device__ __forceinline__ uint32_t peel2(float& a, float& b) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  const f32x2_t v = {a, b};
  const uint32_t w = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
  a -= __uint_as_float(w << 16);
  b -= __uint_as_float(w & 0xffff0000u);
  return w;
}
// x -> three bf16 pieces (x0 + x1 + x2 = x to 2^-26 relative)
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
  float e[8] = {x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]};
  uint4 w[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    w[k].x = peel2(e[0], e[1]);
    w[k].y = peel2(e[2], e[3]);
    w[k].z = peel2(e[4], e[5]);
    w[k].w = peel2(e[6], e[7]);
  }
  p0 = __builtin_bit_cast(bf16x8, w[0]);
  p1 = __builtin_bit_cast(bf16x8, w[1]);
  p2 = __builtin_bit_cast(bf16x8, w[2]);
}
template <int O>
__device__ __forceinline__ void split_acc(const f32x16& s, bf16x8 (&p)[3]) {
  const float x[8] = {s[O], s[O + 1], s[O + 2], s[O + 3], s[O + 4], s[O + 5], s[O + 6], s[O + 7]};
  split8(x, p[0], p[1], p[2]);
}
// 4 fp32 -> three pieces of 4 bf16 (two words each)
__device__ __forceinline__ void split4(const float (&x)[4], uint2 (&p)[3]) {
  float e[4] = {x[0], x[1], x[2], x[3]};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    p[k].x = peel2(e[0], e[1]);
    p[k].y = peel2(e[2], e[3]);
  }
}
// two fp32 -> three pieces of 2 bf16 (one word each: value 0 low, value 1 high)
__device__ __forceinline__ void split2(float x0, float x1, uint32_t (&p)[3]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) p[k] = peel2(x0, x1);
}

// key k (0..63 of a tile) -> its column in the transposed, permuted V image (attention_bf16.hip)
__device__ __forceinline__ int vpos(int k) {
  const int kk = k & 15;
  return (k & ~15) + 8 * ((kk >> 2) & 1) + (kk & 3) + 4 * (kk >> 3);
}

// 6 piece pairs (i, j), i + j <= 2
#define HX_X6(ACC, A, B) \
  do {                                  \
    ACC = mfma(A[0], B[0], ACC);        \
    ACC = mfma(A[0], B[1], ACC);        \
    ACC = mfma(A[1], B[0], ACC);        \
    ACC = mfma(A[0], B[2], ACC);        \
    ACC = mfma(A[1], B[1], ACC);        \
    ACC = mfma(A[2], B[0], ACC);        \
  } while (0)

// grid (ceil(S/128), nh, B), block 256 = 4 waves x 32 queries.
template <bool kDrop>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_fwd_x6_k(
    const float* __restrict__ qkv, const float* __restrict__ qkv_bias, const float* __restrict__ maskb,
    float* __restrict__ out, float* __restrict__ lse, uint32_t* __restrict__ dmask, int S, int nh, float keep,
    const uint64_t* __restrict__ seedp, uint64_t stream, float* __restrict__ amax_part) {
  const uint64_t seed = *seedp;   // per-update Philox key, device-resident (graph-safe)
  __shared__ __attribute__((aligned(16))) uint16_t Ks[3][64 * RS];   // [piece][key][dim]
  __shared__ __attribute__((aligned(16))) uint16_t Vt[3][64 * RS];   // [piece][dim][vpos(key)]
  __shared__ float Ms[64];
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
  const float* base = qkv + (int64_t)b * S * H3 + hd * D;
  const int64_t bh = (int64_t)b * nh + hd;
  const float* kbias = qkv_bias ? qkv_bias + H + hd * D : nullptr;
  const float* vbias = qkv_bias ? qkv_bias + 2 * H + hd * D : nullptr;

  // Q pieces: lane (query, half h), fragment ks = dims 16ks + 8h .. +7, scaled by 1/8 (exact)
  bf16x8 qf[4][3];
  {
    const float* qp = base + (int64_t)qc * H3 + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const float4 a = *reinterpret_cast<const float4*>(qp + 16 * ks);
      const float4 c = *reinterpret_cast<const float4*>(qp + 16 * ks + 4);
      float f[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
      if (qkv_bias) {
        const float* bp = qkv_bias + hd * D + 16 * ks + 8 * h;
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += bp[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= 0.125f;
      split8(f, qf[ks][0], qf[ks][1], qf[ks][2]);
    }
  }

  // ---- tile staging: K rows (2 x 8 dims per thread), V key pairs x 4 dims (2 x 2 x 4)
  float4 kr[2][2], vr[2][2];
  float mr = 0.f;
  auto stage_load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i, row = e >> 3, c8 = (e & 7) * 8;
      const int key = kt + row < S ? kt + row : S - 1;
      const float* kp = base + (int64_t)key * H3 + H + c8;
      kr[i][0] = *reinterpret_cast<const float4*>(kp);
      kr[i][1] = *reinterpret_cast<const float4*>(kp + 4);
      const int kp2 = e & 31, dq = e >> 5;   // lanes over key pairs: the Vt stores spread over the banks
      const int k0 = kt + 2 * kp2 < S ? kt + 2 * kp2 : S - 1, k1 = kt + 2 * kp2 + 1 < S ? kt + 2 * kp2 + 1 : S - 1;
      vr[i][0] = *reinterpret_cast<const float4*>(base + (int64_t)k0 * H3 + 2 * H + 4 * dq);
      vr[i][1] = *reinterpret_cast<const float4*>(base + (int64_t)k1 * H3 + 2 * H + 4 * dq);
    }
    if (tid < 64) mr = kt + tid < S ? maskb[(int64_t)b * S + kt + tid] : -INFINITY;
  };
  auto stage_store = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i, row = e >> 3, c8 = (e & 7) * 8;
      float f[8] = {kr[i][0].x, kr[i][0].y, kr[i][0].z, kr[i][0].w, kr[i][1].x, kr[i][1].y, kr[i][1].z, kr[i][1].w};
      if (kbias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += kbias[c8 + j];
      }
      bf16x8 p[3];
      split8(f, p[0], p[1], p[2]);
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) *reinterpret_cast<bf16x8*>(&Ks[pc][row * RS + c8]) = p[pc];
      const int kp2 = e & 31, dq = e >> 5;
      float v0[4] = {vr[i][0].x, vr[i][0].y, vr[i][0].z, vr[i][0].w};
      float v1[4] = {vr[i][1].x, vr[i][1].y, vr[i][1].z, vr[i][1].w};
      if (vbias) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v0[j] += vbias[4 * dq + j];
          v1[j] += vbias[4 * dq + j];
        }
      }
      constexpr int RW = RS / 2;   // row stride in 32-bit words
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t pc[3];
        split2(v0[j], v1[j], pc);   // keys 2kp2 (low half), 2kp2 + 1 (high half)
        const int off = (4 * dq + j) * RW + (vpos(2 * kp2) >> 1);
        reinterpret_cast<uint32_t*>(Vt[0])[off] = pc[0];
        reinterpret_cast<uint32_t*>(Vt[1])[off] = pc[1];
        reinterpret_cast<uint32_t*>(Vt[2])[off] = pc[2];
      }
    }
    if (tid < 64) Ms[tid] = mr;
  };

  f32x16 o0 = {0}, o1 = {0};
  float m_run = -INFINITY, l_run = 0.f;
  const int nt = (S + 63) >> 6;
  stage_load(0);
  stage_store();
  __syncthreads();

  for (int t = 0; t < nt; ++t) {
    const int kt = t * 64;
    if (t + 1 < nt) stage_load(kt + 64);   // in flight during this tile's math

    uint32_t keepbits[4] = {0u, 0u, 0u, 0u};
    if (kDrop) {
      // Philox chain first: it has no input from the tile's math and fills the MFMA shadow
      const uint64_t cbase = hx::attn::drop_counter(bh, S, q, Sp, kt, h);
#pragma unroll
      for (int j = 0; j < 4; ++j) keepbits[j] = hx::keep8(seed, stream, cbase + j, t16);
    }
    // ---- S^T = K . Q^T, two 32-key blocks, six piece passes each
    f32x16 s0 = {0}, s1 = {0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 ka[3], kb[3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) {
        ka[pc] = *reinterpret_cast<const bf16x8*>(&Ks[pc][l32 * RS + 16 * ks + 8 * h]);
        kb[pc] = *reinterpret_cast<const bf16x8*>(&Ks[pc][(32 + l32) * RS + 16 * ks + 8 * h]);
      }
      HX_X6(s0, ka, qf[ks]);
      HX_X6(s1, kb, qf[ks]);
    }
    // + mask, running max, exp, row sum (the fp32 kernel's formulation)
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s0[r] += Ms[crow(r, h)];
      s1[r] += Ms[32 + crow(r, h)];
      mx = fmaxf(mx, fmaxf(s0[r], s1[r]));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = __expf(m_run - m_new);
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s0[r] = __expf(s0[r] - m_new);
      s1[r] = __expf(s1[r] - m_new);
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
    // ---- O^T += V^T . P^T : P's pieces from the accumulator, V^T rows from the piece images
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x8 pp[3];
      if (g == 0) split_acc<0>(s0, pp);
      else if (g == 1) split_acc<8>(s0, pp);
      else if (g == 2) split_acc<0>(s1, pp);
      else split_acc<8>(s1, pp);
      bf16x8 va[3], vb[3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) {
        va[pc] = *reinterpret_cast<const bf16x8*>(&Vt[pc][l32 * RS + 16 * g + 8 * h]);
        vb[pc] = *reinterpret_cast<const bf16x8*>(&Vt[pc][(32 + l32) * RS + 16 * g + 8 * h]);
      }
      HX_X6(o0, va, pp);
      HX_X6(o1, vb, pp);
    }
    __syncthreads();             // every wave is done with this tile's images
    if (t + 1 < nt) {
      stage_store();
      __syncthreads();
    }
  }

  // ---- epilogue
  if (kDrop && Sp <= kMaxStagedTiles * 64) {
    for (int t = 0; t < nt; ++t)
      dmask[((int64_t)bh * Sp + t * 64 + lane) * (Sp >> 5) + (q0w >> 5)] = Wst[t * 256 + w * 64 + lane];
  }
  if (amax_part) {
    // max |context| of this wave's 32 queries (the fp16x3 attention-output GEMM's operand
    // scale, ops/gemm16.py): one partial per wave, rows past S count 0
    const float il = 1.f / l_run;
    float am = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) am = fmaxf(am, fmaxf(fabsf(o0[i] * il), fabsf(o1[i] * il)));
    if (q >= S) am = 0.f;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
    if (lane == 0) amax_part[(((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 4 + w] = am;
  }
  if (q >= S) return;
  const float inv_l = 1.f / l_run;
  float* op = out + ((int64_t)b * S + q) * H + hd * D;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d0 = 8 * g + 4 * h;
    const float4 va =
        make_float4(o0[4 * g] * inv_l, o0[4 * g + 1] * inv_l, o0[4 * g + 2] * inv_l, o0[4 * g + 3] * inv_l);
    const float4 vb =
        make_float4(o1[4 * g] * inv_l, o1[4 * g + 1] * inv_l, o1[4 * g + 2] * inv_l, o1[4 * g + 3] * inv_l);
    *reinterpret_cast<float4*>(op + d0) = va;
    *reinterpret_cast<float4*>(op + 32 + d0) = vb;
  }
  if (h == 0) lse[bh * S + q] = m_run + __logf(l_run);
}


// ============================================================================ backward
// The bf16 kernel's structure (attention_bf16.hip) with every MFMA operand as three bf16
// pieces and six passes per product.  grid (ceil(S/128), nh, B), block 256 = 4 waves; wave w
// owns keys kbase + 32w .. +31 ON THE LANES (their K / V piece fragments in registers) and
// the workgroup sweeps 32-query tiles:
//   S = Qs . K^T, dP = dO . V^T            (32x32x16: A = piece rows of the tile, B = key pieces)
//   P = exp(S + mask - lse), Pd = P drop/keep, dS = P (dP drop/keep - D)     (fp32, in place)
//   dV += Pd^T . dO, dK += dS^T . Qs        (A = pieces of the P / dS accumulators, B = pieces
//                                            of transposed, query-permuted images of dO / Q)
//   dQ  = dS . K over the block's 128 keys  (16x16x32: dS pieces through LDS, K^T pieces)
// D = rowsum(dO * O) in fp32 while staging.  ~134 KiB of LDS: one workgroup per CU, so the
// kernel may use the whole register file (one wave per SIMD).
constexpr int TS = 40;    // transposed 32-query image row stride (bf16)
constexpr int KTS = 136;  // K^T [dim][128 keys] and dS [query][128 keys] row stride (bf16)
constexpr int KT_B = 64 * KTS * 2, DS_B = 32 * KTS * 2, QS_B = 32 * RS * 2, QT_B = 64 * TS * 2;
constexpr int BWD_SMEM = 3 * (KT_B + DS_B + 2 * QS_B + 2 * QT_B) + 5 * 32 * 4;

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
#define HX_X6_16(ACC, A, B) \
  do {                                    \
    ACC = mfma16(A[0], B[0], ACC);        \
    ACC = mfma16(A[0], B[1], ACC);        \
    ACC = mfma16(A[1], B[0], ACC);        \
    ACC = mfma16(A[0], B[2], ACC);        \
    ACC = mfma16(A[1], B[1], ACC);        \
    ACC = mfma16(A[2], B[0], ACC);        \
  } while (0)

// rows r0, r1 (consecutive image positions) x 4 dims -> 4 words of a transposed image
__device__ __forceinline__ void put_t4(uint16_t* img, int stride, int dim0, int pos, uint2 r0, uint2 r1) {
  uint32_t* p = reinterpret_cast<uint32_t*>(img + dim0 * stride + pos);
  const int sw = stride / 2;
  p[0] = (r0.x & 0xffffu) | (r1.x << 16);
  p[sw] = (r0.x >> 16) | (r1.x & 0xffff0000u);
  p[2 * sw] = (r0.y & 0xffffu) | (r1.y << 16);
  p[3 * sw] = (r0.y >> 16) | (r1.y & 0xffff0000u);
}
__device__ __forceinline__ void ld8(const float* p, const float* bias, float (&f)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), c = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = c.x; f[5] = c.y; f[6] = c.z; f[7] = c.w;
  if (bias) {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] += bias[j];
  }
}

template <bool kDrop>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void attn_bwd_x6_k(
    const float* __restrict__ qkv, const float* __restrict__ qkv_bias, float* __restrict__ dbias_part,
    const float* __restrict__ maskb, const float* __restrict__ dout, const float* __restrict__ outp,
    const float* __restrict__ lse, const uint32_t* __restrict__ dmask, float* __restrict__ dqkv,
    float* __restrict__ dq_acc, int dq_ld, int S, int nh, float keep, float* __restrict__ amax_part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float am = 0.f;   // max |dQKV| of this block's stores (one key block per head only: fp16x3 operand scale)
  uint16_t* Kt = reinterpret_cast<uint16_t*>(smem);                       // [3][64][KTS]
  uint16_t* dSs = reinterpret_cast<uint16_t*>(smem + 3 * KT_B);           // [3][32][KTS]
  uint16_t* Qs = reinterpret_cast<uint16_t*>(smem + 3 * (KT_B + DS_B));   // [3][32][RS]
  uint16_t* dOs = Qs + 3 * 32 * RS;                                       // [3][32][RS]
  uint16_t* Qt = dOs + 3 * 32 * RS;                                       // [3][64][TS]
  uint16_t* dOt = Qt + 3 * 64 * TS;                                       // [3][64][TS]
  float* Ls = reinterpret_cast<float*>(dOt + 3 * 64 * TS);                // [32] lse
  float* Ds = Ls + 32;                                                    // [32][4 waves] D partials

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.z, hd = blockIdx.y;
  const int H = nh * D, H3 = 3 * H;
  const int kbase = blockIdx.x * 128;
  const bool single = gridDim.x == 1;
  const int64_t bh = (int64_t)b * nh + hd;
  const float scale = 0.125f, inv_keep = 1.f / keep;
  const int Sp = (S + 127) & ~127;
  const int nwords = Sp >> 5;
  const float* base = qkv + (int64_t)b * S * H3 + hd * D;
  const float* qbias = qkv_bias ? qkv_bias + hd * D : nullptr;
  const float* kbias = qkv_bias ? qkv_bias + H + hd * D : nullptr;
  const float* vbias = qkv_bias ? qkv_bias + 2 * H + hd * D : nullptr;

  // ---- K^T pieces of the 128 keys (natural key order) for dQ: 64 key pairs x 16 dim quads
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = tid + 256 * i, kp = u & 63, dq = u >> 6;   // lanes over key pairs: conflict-free put_t4
    const int k0 = kbase + 2 * kp < S ? kbase + 2 * kp : S - 1;
    const int k1 = kbase + 2 * kp + 1 < S ? kbase + 2 * kp + 1 : S - 1;
    const float4 a = *reinterpret_cast<const float4*>(base + (int64_t)k0 * H3 + H + 4 * dq);
    const float4 c = *reinterpret_cast<const float4*>(base + (int64_t)k1 * H3 + H + 4 * dq);
    float fa[4] = {a.x, a.y, a.z, a.w}, fc[4] = {c.x, c.y, c.z, c.w};
    if (kbias) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        fa[j] += kbias[4 * dq + j];
        fc[j] += kbias[4 * dq + j];
      }
    }
    uint2 pa[3], pc[3];
    split4(fa, pa);
    split4(fc, pc);
#pragma unroll
    for (int p = 0; p < 3; ++p) put_t4(Kt + p * 64 * KTS, KTS, 4 * dq, 2 * kp, pa[p], pc[p]);
  }
  // ---- this lane's key: K and V piece fragments (B operands of S and dP), dims 16ks + 8h .. +7
  const int mykey = kbase + w * 32 + l32;
  const int mykc = mykey < S ? mykey : S - 1;
  bf16x8 kf[4][3], vf[4][3];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int c = 16 * ks + 8 * h;
    float f[8];
    ld8(base + (int64_t)mykc * H3 + H + c, kbias ? kbias + c : nullptr, f);
    split8(f, kf[ks][0], kf[ks][1], kf[ks][2]);
    ld8(base + (int64_t)mykc * H3 + 2 * H + c, vbias ? vbias + c : nullptr, f);
    split8(f, vf[ks][0], vf[ks][1], vf[ks][2]);
  }
  const float mk = mykey < S ? maskb[(int64_t)b * S + mykey] : -INFINITY;

  const float* dout_b = dout + (int64_t)b * S * H + hd * D;
  const float* out_b = outp + (int64_t)b * S * H + hd * D;
  float* dqkv_b = dqkv + (int64_t)b * S * H3 + hd * D;
  float* dqa_b = dq_acc ? dq_acc + (int64_t)b * S * dq_ld + hd * D : nullptr;
  const float* lse_bh = lse + bh * S;
  const uint32_t* dmask_bh = kDrop ? dmask + bh * Sp * nwords : nullptr;
  const int moff = mykey * nwords;

  // staging unit of this thread: query pair (2sqp, 2sqp+1) x dims 4sdq .. 4sdq+3; lanes run
  // over the query pairs so the transposed-image stores (put_t4) hit 64 distinct banks
  const int sqp = tid & 15, sdq = tid >> 4;
  float4 pq[2], pd[2], po[2];
  float pl = 0.f;
  uint32_t pm = 0;
  auto ld_tile = [&](int qt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int qr = qt + 2 * sqp + i;
      const int r = qr < S ? qr : S - 1;
      pq[i] = *reinterpret_cast<const float4*>(base + (int64_t)r * H3 + 4 * sdq);
      pd[i] = *reinterpret_cast<const float4*>(dout_b + (int64_t)r * H + 4 * sdq);
      po[i] = *reinterpret_cast<const float4*>(out_b + (int64_t)r * H + 4 * sdq);
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

  // split the prefetched tile into the piece images (+ bias, 1/8 on Q), D = rowsum(dO * O), lse
  auto stage = [&](int qt) {
    float q0[4] = {pq[0].x, pq[0].y, pq[0].z, pq[0].w}, q1[4] = {pq[1].x, pq[1].y, pq[1].z, pq[1].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float bj = qbias ? qbias[4 * sdq + j] : 0.f;
      q0[j] = (q0[j] + bj) * scale;
      q1[j] = (q1[j] + bj) * scale;
    }
    float d0[4] = {pd[0].x, pd[0].y, pd[0].z, pd[0].w}, d1[4] = {pd[1].x, pd[1].y, pd[1].z, pd[1].w};
    uint2 q0p[3], q1p[3], d0p[3], d1p[3];
    split4(q0, q0p);
    split4(q1, q1p);
    split4(d0, d0p);
    split4(d1, d1p);
    const int pos = vpos(2 * sqp);
    // Q / dO image rows q with q2 ^ q3 ^ q4 = 1 hold their 16-B chunks pair-swapped (chunk ^ 1):
    // the staging stores drop from 4-way to 2-way bank conflicts (the minimum for this thread
    // map) and the 16-B fragment reads stay conflict-free (searched over all XOR swizzles of
    // the row bits under the guide's ds_write_b64 / ds_read_b128 lane groups)
    const int qcol = 8 * ((sdq >> 1) ^ (((sqp >> 1) ^ (sqp >> 2) ^ (sqp >> 3)) & 1)) + 4 * (sdq & 1);
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      *reinterpret_cast<uint2*>(&Qs[p * 32 * RS + (2 * sqp) * RS + qcol]) = q0p[p];
      *reinterpret_cast<uint2*>(&Qs[p * 32 * RS + (2 * sqp + 1) * RS + qcol]) = q1p[p];
      *reinterpret_cast<uint2*>(&dOs[p * 32 * RS + (2 * sqp) * RS + qcol]) = d0p[p];
      *reinterpret_cast<uint2*>(&dOs[p * 32 * RS + (2 * sqp + 1) * RS + qcol]) = d1p[p];
      put_t4(Qt + p * 64 * TS, TS, 4 * sdq, pos, q0p[p], q1p[p]);
      put_t4(dOt + p * 64 * TS, TS, 4 * sdq, pos, d0p[p], d1p[p]);
    }
    float e0 = pd[0].x * po[0].x + pd[0].y * po[0].y + pd[0].z * po[0].z + pd[0].w * po[0].w;
    float e1 = pd[1].x * po[1].x + pd[1].y * po[1].y + pd[1].z * po[1].z + pd[1].w * po[1].w;
    // this wave's 16 dims (lanes 16 apart), then one partial per wave: Ds[query][wave]
    e0 += __shfl_xor(e0, 16, 64);
    e1 += __shfl_xor(e1, 16, 64);
    e0 += __shfl_xor(e0, 32, 64);
    e1 += __shfl_xor(e1, 32, 64);
    if (lane < 16) {
      Ds[(2 * sqp) * 4 + w] = e0;
      Ds[(2 * sqp + 1) * 4 + w] = e1;
    }
    if (tid < 32) Ls[tid] = qt + tid < S ? pl : INFINITY;   // rows past S: P = 0
  };
  // P, Pd, dS in place for accumulator rows r, r + 1 (queries crow(r), crow(r) + 1); the dS
  // pieces also go to LDS ([query][key]) for dQ
  auto pds = [&](f32x16& sa, f32x16& dpa, uint32_t mword, int r) {
    float ds[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int qr = crow(r + i, h);
      const float p = __expf(sa[r + i] + mk - Ls[qr]);
      float keepf = 1.f;
      if (kDrop) keepf = ((mword >> qr) & 1) ? inv_keep : 0.f;
      sa[r + i] = p * keepf;
      const float4 dq4 = *reinterpret_cast<const float4*>(&Ds[4 * qr]);
      ds[i] = p * (dpa[r + i] * keepf - ((dq4.x + dq4.y) + (dq4.z + dq4.w)));
      dpa[r + i] = ds[i];
    }
    uint32_t pc[3];
    split2(ds[0], ds[1], pc);
    const int o = crow(r, h) * KTS + w * 32 + l32;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      dSs[p * 32 * KTS + o] = (uint16_t)pc[p];
      dSs[p * 32 * KTS + o + KTS] = (uint16_t)(pc[p] >> 16);
    }
  };
  // dV += Pd^T . dO, dK += dS^T . Qs over accumulator half HALF (k-slots = its query rows)
  auto load_img = [&](const uint16_t* img, int half, bf16x8 (&t0)[3], bf16x8 (&t1)[3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      t0[p] = *reinterpret_cast<const bf16x8*>(&img[p * 64 * TS + l32 * TS + 8 * h + 16 * half]);
      t1[p] = *reinterpret_cast<const bf16x8*>(&img[p * 64 * TS + (32 + l32) * TS + 8 * h + 16 * half]);
    }
  };
  // dQ = dS . K over the block's 128 keys (16x16x32 tiles)
  auto dq_mfma = [&](f32x4& qa0, f32x4& qa1) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 a[3], b0[3], b1[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        a[p] = *reinterpret_cast<const bf16x8*>(&dSs[p * 32 * KTS + (qh * 16 + r16) * KTS + 32 * ks + 8 * kg]);
        b0[p] = *reinterpret_cast<const bf16x8*>(&Kt[p * 64 * KTS + (32 * dp2 + r16) * KTS + 32 * ks + 8 * kg]);
        b1[p] = *reinterpret_cast<const bf16x8*>(&Kt[p * 64 * KTS + (32 * dp2 + 16 + r16) * KTS + 32 * ks + 8 * kg]);
      }
      HX_X6_16(qa0, a, b0);
      HX_X6_16(qa1, a, b1);
    }
  };

  stage(0);
  uint32_t mnext = pm;
  for (int qt = 0; qt < S; qt += 32) {
    // tile qt is staged; every wave is done with the previous tile's dS
    __syncthreads();
    const uint32_t mword = mnext;
    const bool more = qt + 32 < S;
    if (more) ld_tile(qt + 32);   // in flight during this tile's math

    // ---- S = Qs . K^T, dP = dO . V^T (queries on accumulator rows, keys on lanes)
    f32x16 sa = {0}, dpa = {0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 qa[3], da[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int qc = 8 * ((2 * ks + h) ^ (((l32 >> 2) ^ (l32 >> 3) ^ (l32 >> 4)) & 1));   // stores' swizzle
        qa[p] = *reinterpret_cast<const bf16x8*>(&Qs[p * 32 * RS + l32 * RS + qc]);
        da[p] = *reinterpret_cast<const bf16x8*>(&dOs[p * 32 * RS + l32 * RS + qc]);
      }
      HX_X6(sa, qa, kf[ks]);
      HX_X6(dpa, da, vf[ks]);
    }
#pragma unroll
    for (int r = 0; r < 8; r += 2) pds(sa, dpa, mword, r);
    {   // accumulator half 0: dV / dK MFMAs, rows 8..15's P / dS in their shadow
      bf16x8 a[3], c[3], t0[3], t1[3];
      split_acc<0>(sa, a);
      split_acc<0>(dpa, c);
      load_img(dOt, 0, t0, t1);
      HX_X6(dv0, a, t0);
      pds(sa, dpa, mword, 8);
      HX_X6(dv1, a, t1);
      pds(sa, dpa, mword, 10);
      load_img(Qt, 0, t0, t1);
      HX_X6(dk0, c, t0);
      pds(sa, dpa, mword, 12);
      HX_X6(dk1, c, t1);
      pds(sa, dpa, mword, 14);
    }
    {   // accumulator half 1
      bf16x8 a[3], c[3], t0[3], t1[3];
      split_acc<8>(sa, a);
      split_acc<8>(dpa, c);
      load_img(dOt, 1, t0, t1);
      HX_X6(dv0, a, t0);
      HX_X6(dv1, a, t1);
      load_img(Qt, 1, t0, t1);
      HX_X6(dk0, c, t0);
      HX_X6(dk1, c, t1);
    }
    // every wave's dS columns are in LDS; the piece images of tile qt are free
    __syncthreads();
    f32x4 qa0 = {0.f, 0.f, 0.f, 0.f}, qa1 = {0.f, 0.f, 0.f, 0.f};
    if (more) {   // next tile's staging in the dQ MFMAs' shadow
      dq_mfma(qa0, qa1);
      stage(qt + 32);
      mnext = pm;
    } else {
      dq_mfma(qa0, qa1);
    }
    const int q0 = qt + qh * 16 + 4 * kg;
    if (dbias_part) {   // rows past S hold exact zeros (their P, hence dS, is 0)
      cq0 += (qa0[0] + qa0[1]) + (qa0[2] + qa0[3]);
      cq1 += (qa1[0] + qa1[1]) + (qa1[2] + qa1[3]);
    }
    const int dcol = 32 * dp2 + r16;
    if (single) {
      float* dq = dqkv_b + (int64_t)q0 * H3 + dcol;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (q0 + r >= S) continue;
        dq[r * H3] = qa0[r] * scale;
        dq[r * H3 + 16] = qa1[r] * scale;
        am = fmaxf(am, fmaxf(fabsf(qa0[r] * scale), fabsf(qa1[r] * scale)));
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
  if (dbias_part) {
    // QKV-bias gradient = column sums of dQ, dK, dV: one row of 3H partials per
    // (batch, key block), folded into the bias-grad slots afterwards (attention.hip)
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
    float* red = reinterpret_cast<float*>(dSs);   // [4 waves][3][64] floats
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
  {
    // ---- epilogue: dK (accumulated against pre-scaled Q: already scaled), dV
    float* dk = dqkv + (int64_t)b * S * H3 + H + hd * D;
    float* dvp = dqkv + (int64_t)b * S * H3 + 2 * H + hd * D;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kbase + w * 32 + crow(r, h);
      if (key >= S) continue;
      dk[(int64_t)key * H3 + l32] = dk0[r];
      dk[(int64_t)key * H3 + 32 + l32] = dk1[r];
      dvp[(int64_t)key * H3 + l32] = dv0[r];
      dvp[(int64_t)key * H3 + 32 + l32] = dv1[r];
      am = fmaxf(am, fmaxf(fmaxf(fabsf(dk0[r]), fabsf(dk1[r])), fmaxf(fabsf(dv0[r]), fabsf(dv1[r]))));
    }
    if (amax_part && single) {
      __shared__ float red_am[4];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
      if (lane == 0) red_am[w] = am;
      __syncthreads();
      if (tid == 0)
        amax_part[(int64_t)blockIdx.z * gridDim.y + blockIdx.y] =
            fmaxf(fmaxf(red_am[0], red_am[1]), fmaxf(red_am[2], red_am[3]));
    }
  }
}

#undef HX_X6_16
#undef HX_X6

}  // namespace

void hx_attn_fwd_x6(const float* qkv, const float* bias, const float* maskb, float* out, float* lse,
                    uint32_t* dmask, int B, int S, int nh, float keep, const uint64_t* seed, uint64_t stream,
                    hipStream_t s, float* amax_part) {
  dim3 grid((S + 127) / 128, nh, B);
  if (keep < 1.f)
    attn_fwd_x6_k<true><<<grid, 256, 0, s>>>(qkv, bias, maskb, out, lse, dmask, S, nh, keep, seed, stream, amax_part);
  else
    attn_fwd_x6_k<false><<<grid, 256, 0, s>>>(qkv, bias, maskb, out, lse, dmask, S, nh, keep, seed, stream, amax_part);
}

void hx_attn_bwd_x6(const float* qkv, const float* bias, float* dbias_part, const float* maskb, const float* dout,
                    const float* out, const float* lse, const uint32_t* dmask, float* dqkv, float* dq_acc, int dq_ld,
                    int B, int S, int nh, float keep, hipStream_t s, float* amax_part) {
  dim3 grid((S + 127) / 128, nh, B);
  static bool attr = false;
  if (!attr) {   // > 64 KiB of dynamic LDS needs an explicit opt-in (gfx950: 160 KiB per CU)
    const void* k[2] = {reinterpret_cast<const void*>(&attn_bwd_x6_k<true>),
                        reinterpret_cast<const void*>(&attn_bwd_x6_k<false>)};
    for (const void* f : k) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, BWD_SMEM);
    attr = true;
  }
  if (keep < 1.f)
    attn_bwd_x6_k<true><<<grid, 256, BWD_SMEM, s>>>(qkv, bias, dbias_part, maskb, dout, out, lse, dmask, dqkv, dq_acc,
                                                    dq_ld, S, nh, keep, amax_part);
  else
    attn_bwd_x6_k<false><<<grid, 256, BWD_SMEM, s>>>(qkv, bias, dbias_part, maskb, dout, out, lse, dmask, dqkv, dq_acc,
                                                     dq_ld, S, nh, keep, amax_part);
}
