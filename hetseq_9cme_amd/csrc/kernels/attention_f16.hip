// fp32 attention on the fp16 matrix cores (--fp32-gemm fp16x3): backward and forward.
//
// Same math and I/O as the other attention backward kernels (reference
// hetseq/bert_modeling.py:351-377 differentiated): packed fp32 [B, S, 3H] QKV (+ the
// projection bias), fp32 context gradient, context, per-query logsumexp and the transposed dropout
// bitmask in; fp32 dQKV (+ QKV-bias gradient partials, + max |dQKV| partials) out.
//
// Every product runs as three fp16 MFMA passes over scaled two-piece operands (the GEMMs' fp16x3
// class, hx_gemm.h): x = 2^-E (h0 + h1), h0 = fp16(2^E x), h1 = fp16(2^E x - h0), the product
// a.b = a0 b0 + a0 b1 + a1 b0 -- half the MFMA passes of a three-piece bf16 split (the round-4
// x6 kernels, deleted in round 5), two LDS images per operand instead of three.  The scale exponents are powers of two chosen so
// the largest magnitude of an operand lands below 2^15:
//   K, V      one exponent per workgroup (its 128 keys), fixed for the kernel;
//   Q, dO     one running exponent per workgroup: each 32-query tile's max |x| is reduced over the
//             workgroup before the tile is split; the exponent follows the tiles down at once and up
//             when a tile lies more than 2^12 below it (next_exp) -- the dK and dV accumulators
//             (which sum over query tiles) are rescaled by the exact power of two when it moves;
//   Pd        fixed: P <= 1, so Pd <= 1 / keep;
//   dS (dK)   one running exponent per wave (its 32 keys), from the wave's max |dS| of each tile,
//             again with an exact rescale of the wave's dK accumulator when it moves;
//   dS (dQ)   one exponent per tile over the workgroup's 128 keys: dS goes through LDS as fp32 and
//             is split after the barrier that publishes every wave's max.
// Unscaling is exact (ldexp) and happens on the fp32 results: S and dP per tile, dQ per tile, dK
// and dV once in the epilogue.
//
// Structure (the x6 kernel's): grid (ceil(S/128), nh, B), block 256 = 4 waves; wave w owns keys
// kbase + 32w .. +31 ON THE LANES (K / V piece fragments in registers) and the workgroup sweeps
// 32-query tiles:
//   S = Qs . K^T, dP = dO . V^T            (32x32x16: A = piece rows of the tile, B = key pieces)
//   P = exp(S + mask - lse), Pd = P drop/keep, dS = P (dP drop/keep - D)     (fp32, in place)
//   dV += Pd^T . dO, dK += dS^T . Qs        (A = pieces of the P / dS accumulators, B = pieces
//                                            of transposed, query-permuted images of dO / Q)
//   dQ  = dS . K over the block's 128 keys  (16x16x32: dS from LDS split per tile, K^T pieces)
// D = rowsum(dO * O) in fp32 while staging.
#include "hx_launch.h"
#include "hx_vec.h"
#include "hx_attn.h"
#include "hx_gemm.h"

namespace {

using hx::attn::crow;
using hx::attn::f32x16;
using hx::g::f16_scale_exp;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int D = 64;
constexpr int RS = 72;    // [query][dim] image row stride (halves): conflict-free 16-B fragment reads
// fp32 dS [query][128 keys]: 144-float rows, the two 4-float halves of each 8-float unit swapped
// on rows with bit 2 set -- conflict-free dQ fragment reads and dS stores (tools/probe/
// lds_conflicts.py models them with the lane groups of MI355X_MICROARCH.md §LDS; the previous
// unswizzled 132-float rows cost 4 extra cycles per ds_read_b128).  Row bit 2 is a lane constant at
// every access (h at the stores, r16 at the reads), so the addresses keep additive constants.
constexpr int DSF = 144;
constexpr int DS_B = 32 * DSF * 4, QS_B = 32 * RS * 2;
constexpr int NSC = 16;   // per-tile scalars: max |Q|, max |dO|, max |dS| per wave (+ spare)
constexpr int KRS = 72;   // K image [128 keys][64 dims] row stride (halves)
constexpr int KI_B = 128 * KRS * 2;
// 73 KiB: two workgroups (two waves per SIMD) per CU
constexpr int BWD_SMEM = 2 * KI_B + DS_B + 2 * (2 * QS_B) + (32 + 128 + NSC) * 4;
constexpr int kNoScale = 120;   // exponent of an operand seen only as zeros so far (no constraint)

__device__ __forceinline__ f32x16 mfma(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// (a0, b0), (a0, b1), (a1, b0)
#define HX_X3(ACC, A, B)          \
  do {                            \
    ACC = mfma(A[0], B[0], ACC);  \
    ACC = mfma(A[0], B[1], ACC);  \
    ACC = mfma(A[1], B[0], ACC);  \
  } while (0)
#define HX_X3_16(ACC, A, B)         \
  do {                              \
    ACC = mfma16(A[0], B[0], ACC);  \
    ACC = mfma16(A[0], B[1], ACC);  \
    ACC = mfma16(A[1], B[0], ACC);  \
  } while (0)

// exponent for an operand whose max |x| so far is m (zeros: no constraint)
__device__ __forceinline__ int run_exp(float m) { return m > 0.f ? f16_scale_exp(m) : kNoScale; }

// Running exponent of a tiled operand whose accumulators are rescaled exactly when it moves: the
// next tile (max |x| = m) lowers it at once, but raises it only when the tile lies more than
// 2^kRaise below it -- a value down to 2^-17 of the scaled range keeps both pieces normal (22 bits),
// so tiles within 2^kRaise need no rescale -- and never above lo + kSpan, lo the smallest exponent
// seen (accumulators built at lo hold <= 2^43 at S <= 8192: 2^(43 + 2 kSpan) stays finite for the dK
// accumulator, whose exponent is the sum of two).  Zero tiles leave it alone.  Rows far below
// earlier, larger rows (a decreasing ramp) thus keep the 22 bits of their own exponent.
constexpr int kRaise = 12, kSpan = 36;
__device__ __forceinline__ int next_exp(int cur, float m, int& lo) {
  if (!(m > 0.f)) return cur;
  const int t = f16_scale_exp(m);
  const int e = t < cur ? t : t > cur + kRaise ? min(t, lo + kSpan) : cur;
  lo = min(lo, e);
  return e;
}

// 8 fp32 values * s -> two fp16 pieces
__device__ __forceinline__ void sp8(const f32x8 x, float s, f16x8 (&p)[2]) {
  const f32x8 y = x * s;
  p[0] = __builtin_convertvector(y, f16x8);
  p[1] = __builtin_convertvector(y - __builtin_convertvector(p[0], f32x8), f16x8);
}
// 4 fp32 values * s -> two pieces of 4 halves (two words each)
__device__ __forceinline__ void sp4(const float (&x)[4], float s, uint2 (&p)[2]) {
  const f32x4 y = f32x4{x[0], x[1], x[2], x[3]} * s;
  const f16x4 h0 = __builtin_convertvector(y, f16x4);
  const f16x4 h1 = __builtin_convertvector(y - __builtin_convertvector(h0, f32x4), f16x4);
  p[0] = __builtin_bit_cast(uint2, h0);
  p[1] = __builtin_bit_cast(uint2, h1);
}
template <int O>
__device__ __forceinline__ f32x8 acc8(const f32x16& s) {
  return f32x8{s[O], s[O + 1], s[O + 2], s[O + 3], s[O + 4], s[O + 5], s[O + 6], s[O + 7]};
}

// key k (0..63 of a 64-position group) -> its column in a transposed, permuted image
// (attention_bf16.hip): the accumulator's row order, so P / dS pieces feed the MFMA A operand
__device__ __forceinline__ int vpos(int k) {
  const int kk = k & 15;
  return (k & ~15) + 8 * ((kk >> 2) & 1) + (kk & 3) + 4 * (kk >> 3);
}
__device__ __forceinline__ f32x8 ld8(const float* p, const float* bias) {
  const float4 a = *reinterpret_cast<const float4*>(p), c = *reinterpret_cast<const float4*>(p + 4);
  f32x8 f = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
  if (bias) {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] += bias[j];
  }
  return f;
}
__device__ __forceinline__ float amax8(const f32x8 f) {
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(f[j]));
  return m;
}
// max over the wave, in every lane: DPP within each row of 16 lanes (quad xor 1, xor 2, half-row
// mirror, row mirror), then the four row maxima through readlane -- no LDS round trip
template <int CTRL>
__device__ __forceinline__ float dmax(float v) {
  return fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false)));
}
__device__ __forceinline__ float wave_max(float m) {
  m = dmax<0xB1>(m);    // quad_perm [1, 0, 3, 2]
  m = dmax<0x4E>(m);    // quad_perm [2, 3, 0, 1]
  m = dmax<0x141>(m);   // row_half_mirror
  m = dmax<0x140>(m);   // row_mirror
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m), 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}
// v *= 2^e, every element (exact unless the result leaves the normal range)
__device__ __forceinline__ void rescale(f32x16& v, int e) {
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = ldexpf(v[r], e);
}
// the same behind a wave-uniform branch that stays a branch (taken on the few tiles whose
// exponent moves): the empty asm keeps the compiler from if-converting it into unconditional
// ldexps and accumulator copies on every tile
__device__ __forceinline__ void rescale2_if(bool c, f32x16& a, f32x16& b, int e) {
  if (c) {
    asm volatile("" ::: "memory");
    rescale(a, e);
    rescale(b, e);
  }
}

// (block, head, batch) of this workgroup, XCD-aware: the hardware deals consecutive workgroups
// round-robin over the 8 XCDs, so the grid is walked so that the key (query) blocks of one head --
// which read the same query (key) rows, and add into the same dQ rows -- run on the same XCD and
// share its L2
struct Blk {
  int x, hd, b;
};
__device__ __forceinline__ Blk xcd_block() {
  const int n = gridDim.x * gridDim.y * gridDim.z;
  int id = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  if ((n & 7) == 0) id = (id & 7) * (n >> 3) + (id >> 3);
  Blk k;
  k.x = id % gridDim.x;
  id /= gridDim.x;
  k.hd = id % gridDim.y;
  k.b = id / gridDim.y;
  return k;
}

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

// B operand (8 consecutive k = image rows r0 .. r0 + 7, one column per lane) of a row-major fp16
// image through two ds_read_b64_tr_b16: per 16-lane group, lane 4q + p addresses row q (+4),
// columns c0 + 4p .. +3, and lane i receives column c0 + i of the four rows (T10)
__device__ __forceinline__ f16x8 tr8(const uint16_t* img, int stride, int r0, int c0, int i) {
  const uint16_t* a = img + (r0 + (i >> 2)) * stride + c0 + 4 * (i & 3);
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a));
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a + 4 * stride));
  const v4i16 v[2] = {lo, hi};
  return *reinterpret_cast<const f16x8*>(v);
}

template <bool kDrop>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_bwd_f16_k(
    const float* __restrict__ qkv, const float* __restrict__ qkv_bias, float* __restrict__ dbias_part,
    const float* __restrict__ maskb, const float* __restrict__ dout, const float* __restrict__ outp,
    const float* __restrict__ lse, const uint32_t* __restrict__ dmask, float* __restrict__ dqkv,
    float* __restrict__ dq_acc, int dq_ld, int S, int nh, float keep, float* __restrict__ amax_part,
    float* __restrict__ colmax_part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // one row-major image per operand, read both ways: K [key][dim] as the B operand of S (rows) and
  // of dQ (transposed reads); Q / dO [vpos(query)][dim] as the A operand of S / dP (rows) and the
  // B operand of dK / dV (transposed reads of 8 consecutive rows = the accumulator's k order)
  uint16_t* Ki = reinterpret_cast<uint16_t*>(smem);                      // [2][128][KRS]
  float* dSf = reinterpret_cast<float*>(smem + 2 * KI_B);                // [32][DSF] fp32
  uint16_t* Qs = reinterpret_cast<uint16_t*>(smem + 2 * KI_B + DS_B);    // [2][32][RS]
  uint16_t* dOs = Qs + 2 * 32 * RS;                                      // [2][32][RS]
  float* Ls = reinterpret_cast<float*>(smem + 2 * KI_B + DS_B + 4 * QS_B);   // [32] lse
  float* Ds = Ls + 32;                                                   // [32] D = rowsum(dO * O)
  float* Sc = Ds + 128;                                                  // per-tile scalars
  float* ScQ = Sc, *ScD = Sc + 4, *ScS = Sc + 8;                         // [4 waves] each

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const Blk blk = xcd_block();
  const int b = blk.b, hd = blk.hd;
  const int H = nh * D, H3 = 3 * H;
  const int kbase = blk.x * 128;
  const bool single = gridDim.x == 1;
  const int64_t bh = (int64_t)b * nh + hd;
  const float scale = 0.125f, inv_keep = 1.f / keep;
  const int Sp = (S + 127) & ~127;
  const int nwords = Sp >> 5;
  const float* base = qkv + (int64_t)b * S * H3 + hd * D;
  const float* qbias = qkv_bias ? qkv_bias + hd * D : nullptr;
  const float* kbias = qkv_bias ? qkv_bias + H + hd * D : nullptr;
  const float* vbias = qkv_bias ? qkv_bias + 2 * H + hd * D : nullptr;
  // max |dQ|, |dK|, |dV| of each of the head's rows, for the QKV GEMMs' per-row operand scale
  // (amax_part[row][head]; ops/gemm16.py takes the max over the heads).  Several key blocks
  // (S > 128): this block's key rows' dK / dV only -- dQ is summed over the blocks by atomics, its
  // maxima come from one pass over the dQ third (ops/flash_attention.py)
  __shared__ unsigned rmx_s[128];
  const bool want_am = amax_part != nullptr;
  if (want_am && tid < 128) rmx_s[tid] = 0u;
  // ... and max |dQ| / |dK| / |dV| of each of its columns -> colmax_part[b][key block][3H] (the QKV
  // weight gradient's per-column scale; several key blocks: the dQ section stays 0)
  const bool want_cm = colmax_part != nullptr;
  float cqm0 = 0.f, cqm1 = 0.f;   // running column maxima of this lane's two dQ columns
  const int mykey = kbase + w * 32 + l32;
  const int mykc = mykey < S ? mykey : S - 1;

  const float* dout_b = dout + (int64_t)b * S * H + hd * D;
  const float* out_b = outp + (int64_t)b * S * H + hd * D;
  float* dqkv_b = dqkv + (int64_t)b * S * H3 + hd * D;
  float* dqa_b = dq_acc ? dq_acc + (int64_t)b * S * dq_ld + hd * D : nullptr;
  const float* lse_bh = lse + bh * S;
  const uint32_t* dmask_bh = kDrop ? dmask + bh * Sp * nwords : nullptr;
  const int moff = mykey * nwords;

  // staging unit of this thread: query pair (2sqp, 2sqp+1) x dims 4sdq .. 4sdq+3 -- the 16 lanes of
  // a group share the query pair, so each image store of the group fills one row (conflict-free:
  // with the lanes on 16 rows a ds_write_b64 took 4x its cycles) and D = rowsum(dO * O) completes
  // inside the group
  const int sqp = tid >> 4, sdq = tid & 15;
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
  // ---- the block's K rows (4 x 8 dims per thread, for the K image) and this lane's V fragments
  // (dims 16ks + 8h .. +7), then the first query tile's loads (both in flight together), then the
  // block's max |K|, |V|
  f32x8 kx[4], vx[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = tid + 256 * i, key = kbase + (u >> 3), c8 = (u & 7) * 8;
    kx[i] = ld8(base + (int64_t)(key < S ? key : S - 1) * H3 + H + c8, kbias ? kbias + c8 : nullptr);
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int c = 16 * ks + 8 * h;
    vx[ks] = ld8(base + (int64_t)mykc * H3 + 2 * H + c, vbias ? vbias + c : nullptr);
  }
  ld_tile(0);
  float mkx = 0.f, mvx = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) mkx = fmaxf(mkx, amax8(kx[i]));
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) mvx = fmaxf(mvx, amax8(vx[ks]));
  mkx = wave_max(mkx);
  mvx = wave_max(mvx);
  if (lane == 0) {
    ScQ[w] = mkx;
    ScD[w] = mvx;
  }
  const float mk = mykey < S ? maskb[(int64_t)b * S + mykey] : -INFINITY;

  // (q + bias) / 8 of the prefetched tile (the head's Q bias from LDS, staged once)
  __shared__ __attribute__((aligned(16))) float Qb[64];
  if (tid < 64) Qb[tid] = qbias ? qbias[tid] : 0.f;   // published by the barrier after ld_tile(0)
  auto qvals = [&](float (&q0)[4], float (&q1)[4]) {
    const float a[8] = {pq[0].x, pq[0].y, pq[0].z, pq[0].w, pq[1].x, pq[1].y, pq[1].z, pq[1].w};
    const float4 bq = *reinterpret_cast<const float4*>(&Qb[4 * sdq]);
    const float bb[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      q0[j] = (a[j] + bb[j]) * scale;
      q1[j] = (a[4 + j] + bb[j]) * scale;
    }
  };
  // the prefetched tile's max |Q|, |dO| -> this wave's slots
  auto tile_max = [&]() {
    float q0[4], q1[4];
    qvals(q0, q1);
    float mq = 0.f, md = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) mq = fmaxf(mq, fmaxf(fabsf(q0[j]), fabsf(q1[j])));
    md = fmaxf(fmaxf(fmaxf(fabsf(pd[0].x), fabsf(pd[0].y)), fmaxf(fabsf(pd[0].z), fabsf(pd[0].w))),
               fmaxf(fmaxf(fabsf(pd[1].x), fabsf(pd[1].y)), fmaxf(fabsf(pd[1].z), fabsf(pd[1].w))));
    mq = wave_max(mq);
    md = wave_max(md);
    if (lane == 0) {
      ScQ[w] = mq;
      ScD[w] = md;
    }
  };
  auto max4 = [&](const float* p) { return fmaxf(fmaxf(p[0], p[1]), fmaxf(p[2], p[3])); };

  __syncthreads();   // block max |K|, |V| published
  const int ek = f16_scale_exp(max4(ScQ)), ev = f16_scale_exp(max4(ScD));
  const float sk = ldexpf(1.f, ek), sv = ldexpf(1.f, ev);
  // V's piece fragments in registers (B operands of dP); K's pieces into the image
  f16x8 vf[4][2];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) sp8(vx[ks], sv, vf[ks]);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = tid + 256 * i, row = u >> 3, c8 = (u & 7) * 8;
    f16x8 p2[2];
    sp8(kx[i], sk, p2);
    *reinterpret_cast<f16x8*>(&Ki[row * KRS + c8]) = p2[0];
    *reinterpret_cast<f16x8*>(&Ki[128 * KRS + row * KRS + c8]) = p2[1];
  }
  __syncthreads();   // every wave has read the K / V maxima
  tile_max();
  __syncthreads();
  int eq = run_exp(max4(ScQ)), ed = run_exp(max4(ScD));   // running exponents of the Q / dO images

  // dQ tiles of this wave (16x16x32 layout): queries 16qh .., dims 32dp2 .. and 32dp2 + 16 ..
  const int qh = w & 1, dp2 = w >> 1;
  const int vq = vpos(l32);   // image row of query l32 (A operand row of S / dP)
  const int r16 = lane & 15, kg = lane >> 4;

  // accumulators and the exponents they are held at: dv = dV 2^(ep + dv_e), dk = dK 2^(dk_e)
  f32x16 dv0 = {0}, dv1 = {0}, dk0 = {0}, dk1 = {0};
  const int ep = f16_scale_exp(inv_keep);   // Pd <= 1 / keep
  const float keep_s = ldexpf(inv_keep, ep), one_s = ldexpf(1.f, ep);
  int dv_e = ed, es = kNoScale, dk_e = eq + kNoScale;
  int eq_lo = eq, ed_lo = ed, es_lo = kNoScale;   // the smallest exponents seen (next_exp)
  float cq0 = 0.f, cq1 = 0.f;

  // split the prefetched tile into the piece images (+ bias, 1/8 on Q) at the running exponents,
  // D = rowsum(dO * O), lse
  auto stage = [&](int qt) {
    float q0[4], q1[4];
    qvals(q0, q1);
    const float d0[4] = {pd[0].x, pd[0].y, pd[0].z, pd[0].w}, d1[4] = {pd[1].x, pd[1].y, pd[1].z, pd[1].w};
    const float sq = ldexpf(1.f, eq), sd = ldexpf(1.f, ed);
    uint2 q0p[2], q1p[2], d0p[2], d1p[2];
    sp4(q0, sq, q0p);
    sp4(q1, sq, q1p);
    sp4(d0, sd, d0p);
    sp4(d1, sd, d1p);
    // rows in the accumulator's k order (vpos): 8 consecutive rows = one k slice of dK / dV
    const int r0 = vpos(2 * sqp), col = 4 * sdq;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      *reinterpret_cast<uint2*>(&Qs[p * 32 * RS + r0 * RS + col]) = q0p[p];
      *reinterpret_cast<uint2*>(&Qs[p * 32 * RS + (r0 + 1) * RS + col]) = q1p[p];
      *reinterpret_cast<uint2*>(&dOs[p * 32 * RS + r0 * RS + col]) = d0p[p];
      *reinterpret_cast<uint2*>(&dOs[p * 32 * RS + (r0 + 1) * RS + col]) = d1p[p];
    }
    float e0 = pd[0].x * po[0].x + pd[0].y * po[0].y + pd[0].z * po[0].z + pd[0].w * po[0].w;
    float e1 = pd[1].x * po[1].x + pd[1].y * po[1].y + pd[1].z * po[1].z + pd[1].w * po[1].w;
    // the 64 dims of the query pair sit on the 16 lanes of the group
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      e0 += __shfl_xor(e0, o, 64);
      e1 += __shfl_xor(e1, o, 64);
    }
    if (sdq == 0) {
      Ds[2 * sqp] = e0;
      Ds[2 * sqp + 1] = e1;
    }
    if (tid < 32) Ls[tid] = qt + tid < S ? pl : INFINITY;   // rows past S: P = 0
  };
  // dims l32 (t0) and 32 + l32 (t1) of image rows 16 half + 8h .. +7, transposed
  const int gcol = 16 * ((lane >> 4) & 1), li = lane & 15;

  stage(0);
  uint32_t mnext = pm;
  for (int qt = 0; qt < S; qt += 32) {
    // tile qt is staged at exponents (eq, ed); every wave is done with the previous tile's dS
    __syncthreads();
    const uint32_t mword = mnext;
    const bool more = qt + 32 < S;
    if (more) ld_tile(qt + 32);   // in flight during this tile's math

    // ---- S = Qs . K^T, dP = dO . V^T (queries on accumulator rows, keys on lanes)
    f32x16 sa = {0}, dpa = {0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      f16x8 qa[2], da[2], kf[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int off = p * 32 * RS + vq * RS + 16 * ks + 8 * h;
        qa[p] = *reinterpret_cast<const f16x8*>(&Qs[off]);
        da[p] = *reinterpret_cast<const f16x8*>(&dOs[off]);
        kf[p] = *reinterpret_cast<const f16x8*>(&Ki[p * 128 * KRS + (w * 32 + l32) * KRS + 16 * ks + 8 * h]);
      }
      HX_X3(sa, qa, kf);
      HX_X3(dpa, da, vf[ks]);
    }
    rescale2_if(ed != dv_e, dv0, dv1, ed - dv_e);   // the dO images' exponent dropped: bring dV along
    dv_e = ed;
    // ---- P, Pd (at 2^ep), dS in place; the wave's max |dS|
    const float fs = ldexpf(1.f, -(eq + ek)), fd = ldexpf(1.f, -(ed + ev));
    float smax = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qr = crow(r, h);
      const float p = __expf(fmaf(sa[r], fs, mk) - Ls[qr]);
      float keepf = 1.f, keeps = one_s;
      if (kDrop) {
        const bool kb = (mword >> qr) & 1;
        keepf = kb ? inv_keep : 0.f;
        keeps = kb ? keep_s : 0.f;
      }
      sa[r] = p * keeps;
      const float ds = p * (dpa[r] * fd * keepf - Ds[qr]);
      dpa[r] = ds;
      smax = fmaxf(smax, fabsf(ds));
      dSf[qr * DSF + w * 32 + (l32 ^ (4 * h))] = ds;   // row bit 2 of crow(r, h) is h
    }
    smax = wave_max(smax);
    if (lane == 0) ScS[w] = smax;
    {   // the wave's dS exponent (running, decreasing) and the dK accumulator's
      const int es_new = next_exp(es, smax, es_lo);
      rescale2_if(eq + es_new != dk_e, dk0, dk1, eq + es_new - dk_e);
      dk_e = eq + es_new;
      es = es_new;
    }
    const float ss = ldexpf(1.f, es);
    // ---- dV += Pd^T . dO, dK += dS^T . Qs over the two accumulator halves (k-slots = query rows)
    // one operand pair live at a time (fewer VGPRs at the loop's peak: no spills in the loop)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f16x8 a[2], t[2];
      sp8(half ? acc8<8>(sa) : acc8<0>(sa), 1.f, a);
#pragma unroll
      for (int p = 0; p < 2; ++p) t[p] = tr8(dOs + p * 32 * RS, RS, 16 * half + 8 * h, gcol, li);
      HX_X3(dv0, a, t);
#pragma unroll
      for (int p = 0; p < 2; ++p) t[p] = tr8(dOs + p * 32 * RS, RS, 16 * half + 8 * h, 32 + gcol, li);
      HX_X3(dv1, a, t);
    }
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f16x8 c[2], t[2];
      sp8(half ? acc8<8>(dpa) : acc8<0>(dpa), ss, c);
#pragma unroll
      for (int p = 0; p < 2; ++p) t[p] = tr8(Qs + p * 32 * RS, RS, 16 * half + 8 * h, gcol, li);
      HX_X3(dk0, c, t);
#pragma unroll
      for (int p = 0; p < 2; ++p) t[p] = tr8(Qs + p * 32 * RS, RS, 16 * half + 8 * h, 32 + gcol, li);
      HX_X3(dk1, c, t);
    }
    if (more) tile_max();   // the next tile's max |Q|, |dO| (its loads have landed by now)
    // every wave's dS and maxima are in LDS; the piece images of tile qt are free
    __syncthreads();
    const int et = run_exp(max4(ScS));   // this tile's dS exponent over the 128 keys
    const float st = ldexpf(1.f, et);
    if (more) {
      eq = next_exp(eq, max4(ScQ), eq_lo);
      ed = next_exp(ed, max4(ScD), ed_lo);
    }
    // ---- dQ = dS . K over the block's 128 keys (16x16x32 tiles); dq_sw: this lane row's half swap
    const int dq_sw = 4 * ((r16 >> 2) & 1);
    f32x4 qa0 = {0.f, 0.f, 0.f, 0.f}, qa1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const float* src = &dSf[(qh * 16 + r16) * DSF + 32 * ks + 8 * kg];
      const float4 x0 = *reinterpret_cast<const float4*>(src + dq_sw),
                   x1 = *reinterpret_cast<const float4*>(src + 4 - dq_sw);
      f16x8 a[2], b0[2], b1[2];
      sp8(f32x8{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w}, st, a);
#pragma unroll
      for (int p = 0; p < 2; ++p) {   // K^T fragments: dims 32dp2 + r16 (+ 16), keys 32ks + 8kg .. +7
        b0[p] = tr8(Ki + p * 128 * KRS, KRS, 32 * ks + 8 * kg, 32 * dp2, r16);
        b1[p] = tr8(Ki + p * 128 * KRS, KRS, 32 * ks + 8 * kg, 32 * dp2 + 16, r16);
      }
      HX_X3_16(qa0, a, b0);
      HX_X3_16(qa1, a, b1);
    }
    if (more) {   // next tile's staging in the dQ MFMAs' shadow
      stage(qt + 32);
      mnext = pm;
    }
    const int eqo = -(et + ek);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      qa0[r] = ldexpf(qa0[r], eqo) * scale;
      qa1[r] = ldexpf(qa1[r], eqo) * scale;
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
        dq[r * H3] = qa0[r];
        dq[r * H3 + 16] = qa1[r];
      }
      if (want_cm) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (q0 + r < S) {
            cqm0 = fmaxf(cqm0, fabsf(qa0[r]));
            cqm1 = fmaxf(cqm1, fabsf(qa1[r]));
          }
      }
      if (want_am) {   // row q0 + r: its 32 columns of this wave over the 16 lanes of the group
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float m = fmaxf(fabsf(qa0[r]), fabsf(qa1[r]));
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
          if (r16 == 0 && q0 + r < S) atomicMax(&rmx_s[q0 + r], __float_as_uint(m));
        }
      }
    } else {
      float* dq = dqa_b + (int64_t)q0 * dq_ld + dcol;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (q0 + r >= S) continue;
        atomicAdd(dq + r * dq_ld, qa0[r]);
        atomicAdd(dq + r * dq_ld + 16, qa1[r]);
      }
    }
  }
  // ---- undo the accumulators' scales: dK (against pre-scaled Q: already scaled by 1/8), dV
  rescale(dk0, -dk_e);
  rescale(dk1, -dk_e);
  rescale(dv0, -(ep + dv_e));
  rescale(dv1, -(ep + dv_e));
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
    __syncthreads();   // every wave is done with dSf
    float* red = dSf;   // [4 waves][3][64] floats
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
      dbias_part[((int64_t)b * gridDim.x + blk.x) * H3 + part * H + hd * D + c] = v;
    }
  }
  {
    // ---- epilogue: dK, dV
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
    }
    if (want_am) {
      // key rows: the 64 dK and 64 dV columns of a row sit on the 32 lanes of a half-wave.
      // Transposing max-reduction: at lane masks 16 .. 2 a lane keeps the half of its row values
      // its lane bit selects and takes the partner's other half, then one more exchange (mask 1):
      // 16 shuffles instead of 16 x 5; lanes 2k, 2k + 1 end with row value k
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = fmaxf(fmaxf(fabsf(dk0[r]), fabsf(dk1[r])), fmaxf(fabsf(dv0[r]), fabsf(dv1[r])));
#pragma unroll
      for (int m = 16, n = 16; m >= 2; m >>= 1, n >>= 1) {
        const bool up = (l32 & m) != 0;
#pragma unroll
        for (int j = 0; j < n / 2; ++j) {
          const float keepv = up ? v[j + n / 2] : v[j], sendv = up ? v[j] : v[j + n / 2];
          v[j] = fmaxf(keepv, __shfl_xor(sendv, m, 64));
        }
      }
      v[0] = fmaxf(v[0], __shfl_xor(v[0], 1, 64));
      {
        const int key = kbase + w * 32 + crow(l32 >> 1, h);
        if ((l32 & 1) == 0 && key < S) atomicMax(&rmx_s[key - kbase], __float_as_uint(v[0]));
      }
      __syncthreads();
      if (tid < 128 && kbase + tid < S)
        amax_part[((int64_t)b * S + kbase + tid) * nh + hd] = __uint_as_float(rmx_s[tid]);
    }
    if (want_cm) {
      __shared__ float cmx_s[4][3][64];
      // dQ: lane (r16, kg) of wave (qh, dp2) holds columns 32 dp2 + r16 (+ 16) over rows 4 kg + r
      cqm0 = fmaxf(cqm0, __shfl_xor(cqm0, 16, 64));
      cqm0 = fmaxf(cqm0, __shfl_xor(cqm0, 32, 64));
      cqm1 = fmaxf(cqm1, __shfl_xor(cqm1, 16, 64));
      cqm1 = fmaxf(cqm1, __shfl_xor(cqm1, 32, 64));
      // dK / dV: lane (l32, h) holds columns l32 and 32 + l32 of the wave's key rows crow(r, h)
      float mk0 = 0.f, mk1 = 0.f, mv0 = 0.f, mv1 = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (kbase + w * 32 + crow(r, h) >= S) continue;
        mk0 = fmaxf(mk0, fabsf(dk0[r])); mk1 = fmaxf(mk1, fabsf(dk1[r]));
        mv0 = fmaxf(mv0, fabsf(dv0[r])); mv1 = fmaxf(mv1, fabsf(dv1[r]));
      }
      mk0 = fmaxf(mk0, __shfl_xor(mk0, 32, 64)); mk1 = fmaxf(mk1, __shfl_xor(mk1, 32, 64));
      mv0 = fmaxf(mv0, __shfl_xor(mv0, 32, 64)); mv1 = fmaxf(mv1, __shfl_xor(mv1, 32, 64));
      if (lane < 16) {   // this wave's dQ columns; the other query half's wave fills the same slots
        cmx_s[w][0][32 * dp2 + lane] = cqm0;
        cmx_s[w][0][32 * dp2 + 16 + lane] = cqm1;
      }
      if (lane < 32) {
        cmx_s[w][1][l32] = mk0; cmx_s[w][1][32 + l32] = mk1;
        cmx_s[w][2][l32] = mv0; cmx_s[w][2][32 + l32] = mv1;
      }
      __syncthreads();
      if (tid < 192) {
        const int sec = tid >> 6, c = tid & 63;
        float m;
        if (sec == 0) {   // waves (0,1) own dQ columns 0..31 (dp2 = 0), waves (2,3) 32..63
          const int wa = c < 32 ? 0 : 2;
          m = fmaxf(cmx_s[wa][0][c], cmx_s[wa + 1][0][c]);
        } else {
          m = fmaxf(fmaxf(cmx_s[0][sec][c], cmx_s[1][sec][c]), fmaxf(cmx_s[2][sec][c], cmx_s[3][sec][c]));
        }
        colmax_part[((int64_t)b * gridDim.x + blk.x) * 3 * H + sec * H + hd * D + c] = m;
      }
    }
  }
}

// ============================================================================ forward
// Two fp16 pieces and three passes per product:
// one workgroup = 4 waves x 32 queries ON THE LANES, 64-key tiles, keys on the accumulator rows
// (S^T = K . Q^T with Q's piece fragments in VGPRs), K staged as piece images [key][dim], V as
// transposed piece images [dim][vpos(key)] so O^T += V^T . P^T takes P's pieces straight from the
// accumulator.  Exponents: Q one per wave (fixed); K and V one per 64-key tile, from the tile's
// max |x| reduced over the workgroup before it is split (S is unscaled per tile; the tile-to-tile
// change of V's exponent rides in the online-softmax rescale of the O accumulator); P <= 1 / keep
// fixed.  Single-buffered images (37 KiB: two workgroups per CU), the next tile's fp32 loads in
// flight in registers during the current tile's math.
template <bool kDrop>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_fwd_f16_k(
    const float* __restrict__ qkv, const float* __restrict__ qkv_bias, const float* __restrict__ maskb,
    float* __restrict__ out, float* __restrict__ lse, uint32_t* __restrict__ dmask, int S, int nh, float keep,
    const uint64_t* __restrict__ seedp, uint64_t stream, float* __restrict__ amax_part,
    float* __restrict__ colmax_part) {
  const uint64_t seed = *seedp;   // per-update Philox key, device-resident (graph-safe)
  __shared__ __attribute__((aligned(16))) uint16_t Ks[2][64 * RS];   // [piece][key][dim]
  __shared__ __attribute__((aligned(16))) uint16_t Vt[2][64 * RS];   // [piece][dim][vpos(key)]
  __shared__ float Ms[64];
  __shared__ float Mx[8];                                             // per-wave max |K|, |V|
  __shared__ __attribute__((aligned(16))) float Bkv[128];             // the K | V bias of this head
  constexpr int kMaxStagedTiles = 8;   // S <= 512: mask words staged, stored after the loop
  __shared__ uint32_t Wst[kDrop ? kMaxStagedTiles * 256 : 1];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const Blk blk = xcd_block();
  const int b = blk.b, hd = blk.hd;
  const int H = nh * D, H3 = 3 * H;
  const int q = blk.x * 128 + w * 32 + l32;
  const int qc = q < S ? q : S - 1;            // rows past S: clamped loads, no stores
  const int Sp = (S + 127) & ~127;
  const int q0w = blk.x * 128 + w * 32;
  const uint32_t t16 = (uint32_t)(keep * 65536.f + 0.5f);
  const float inv_keep = 1.f / keep;
  const float* base = qkv + (int64_t)b * S * H3 + hd * D;
  const int64_t bh = (int64_t)b * nh + hd;
  const float* kbias = qkv_bias ? qkv_bias + H + hd * D : nullptr;
  const float* vbias = qkv_bias ? qkv_bias + 2 * H + hd * D : nullptr;

  // Q pieces: lane (query, half h), fragment ks = dims 16ks + 8h .. +7, scaled by 1/8 (exact) and
  // by the wave's exponent -- the fp32 loads first, the first K / V tile's loads next (below), so
  // both latencies overlap; the max / split waits only for Q
  f16x8 qf[4][2];
  int eq;
  f32x8 qx[4];
  {
    const float* qp = base + (int64_t)qc * H3 + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qx[ks] = ld8(qp + 16 * ks, nullptr);
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
  // the thread's K bias (its 8 columns are the same for both rows it stages) and V bias (4 dims of
  // each of its two key pairs), in registers for the whole kernel (loaded from LDS below)
  float4 kb[2], vb[2];
  auto add4 = [](float4& a, const float4& b) { a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w; };
  // the loaded tile + bias, in place (once per tile, before its max and its split)
  auto add_bias = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      add4(kr[i][0], kb[0]);
      add4(kr[i][1], kb[1]);
      add4(vr[i][0], vb[i]);
      add4(vr[i][1], vb[i]);
    }
  };
  auto kvals = [&](int i, f32x8& f) {
    f = f32x8{kr[i][0].x, kr[i][0].y, kr[i][0].z, kr[i][0].w, kr[i][1].x, kr[i][1].y, kr[i][1].z, kr[i][1].w};
  };
  auto vvals = [&](int i, float (&v0)[4], float (&v1)[4]) {
    const float a[8] = {vr[i][0].x, vr[i][0].y, vr[i][0].z, vr[i][0].w, vr[i][1].x, vr[i][1].y, vr[i][1].z, vr[i][1].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v0[j] = a[j];
      v1[j] = a[4 + j];
    }
  };
  // the loaded tile's max |K|, |V| -> this wave's slots (read after the next barrier)
  auto tile_max = [&]() {
    float mk = 0.f, mv = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f32x8 f;
      kvals(i, f);
      mk = fmaxf(mk, amax8(f));
      float v0[4], v1[4];
      vvals(i, v0, v1);
#pragma unroll
      for (int j = 0; j < 4; ++j) mv = fmaxf(mv, fmaxf(fabsf(v0[j]), fabsf(v1[j])));
    }
    mk = wave_max(mk);
    mv = wave_max(mv);
    if (lane == 0) {
      Mx[w] = mk;
      Mx[4 + w] = mv;
    }
  };
  auto stage_store = [&](float sk, float sv) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i, row = e >> 3, c8 = (e & 7) * 8;
      f32x8 f;
      kvals(i, f);
      f16x8 p[2];
      sp8(f, sk, p);
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) *reinterpret_cast<f16x8*>(&Ks[pc][row * RS + c8]) = p[pc];
      const int kp2 = e & 31, dq = e >> 5;
      float v0[4], v1[4];
      vvals(i, v0, v1);
      uint2 a0[2], a1[2];
      sp4(v0, sv, a0);   // key 2kp2, dims 4dq .. +3
      sp4(v1, sv, a1);   // key 2kp2 + 1
      constexpr int RW = RS / 2;   // row stride in 32-bit words
      const int pos = vpos(2 * kp2) >> 1;
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) {
        uint32_t* vt = reinterpret_cast<uint32_t*>(Vt[pc]);
        vt[(4 * dq + 0) * RW + pos] = (a0[pc].x & 0xffffu) | (a1[pc].x << 16);
        vt[(4 * dq + 1) * RW + pos] = (a0[pc].x >> 16) | (a1[pc].x & 0xffff0000u);
        vt[(4 * dq + 2) * RW + pos] = (a0[pc].y & 0xffffu) | (a1[pc].y << 16);
        vt[(4 * dq + 3) * RW + pos] = (a0[pc].y >> 16) | (a1[pc].y & 0xffff0000u);
      }
    }
    if (tid < 64) Ms[tid] = mr;
  };
  auto max4 = [&](const float* p) { return fmaxf(fmaxf(p[0], p[1]), fmaxf(p[2], p[3])); };

  f32x16 o0 = {0}, o1 = {0};
  float m_run = -INFINITY, l_run = 0.f;
  const int ep = f16_scale_exp(inv_keep);   // P' <= 1 / keep
  const float ps = ldexpf(1.f, ep);
  int ek, ev, ev_o = 0;                     // the tile's K / V exponents; o holds O 2^(ep + ev_o)
  const int nt = (S + 63) >> 6;
  stage_load(0);   // in flight with the Q loads
  {
    float m = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (qkv_bias) {
        const float* qb = qkv_bias + hd * D + 16 * ks + 8 * h;
#pragma unroll
        for (int j = 0; j < 8; ++j) qx[ks][j] += qb[j];
      }
      qx[ks] = qx[ks] * 0.125f;
      m = fmaxf(m, amax8(qx[ks]));
    }
    eq = f16_scale_exp(wave_max(m));
    const float sq = ldexpf(1.f, eq);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) sp8(qx[ks], sq, qf[ks]);
  }
  // the head's K and V bias, once per workgroup (the staging adds them at every tile: from LDS,
  // not 12 dependent global loads per tile and thread)
  if (tid < 128) Bkv[tid] = qkv_bias ? (tid < 64 ? kbias[tid] : vbias[tid - 64]) : 0.f;
  __syncthreads();
  kb[0] = *reinterpret_cast<const float4*>(&Bkv[(tid & 7) * 8]);
  kb[1] = *reinterpret_cast<const float4*>(&Bkv[(tid & 7) * 8 + 4]);
#pragma unroll
  for (int i = 0; i < 2; ++i) vb[i] = *reinterpret_cast<const float4*>(&Bkv[64 + 4 * ((tid + 256 * i) >> 5)]);
  add_bias();
  tile_max();
  __syncthreads();
  ek = f16_scale_exp(max4(Mx));
  ev = f16_scale_exp(max4(Mx + 4));
  ev_o = ev;
  stage_store(ldexpf(1.f, ek), ldexpf(1.f, ev));
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
    // ---- S^T = K . Q^T, two 32-key blocks, three piece passes each
    f32x16 s0 = {0}, s1 = {0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      f16x8 ka[2], kb[2];
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) {
        ka[pc] = *reinterpret_cast<const f16x8*>(&Ks[pc][l32 * RS + 16 * ks + 8 * h]);
        kb[pc] = *reinterpret_cast<const f16x8*>(&Ks[pc][(32 + l32) * RS + 16 * ks + 8 * h]);
      }
      HX_X3(s0, ka, qf[ks]);
      HX_X3(s1, kb, qf[ks]);
    }
    // unscale, + mask, running max, exp, row sum (the fp32 kernel's formulation)
    const float fs = ldexpf(1.f, -(ek + eq));
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s0[r] = fmaf(s0[r], fs, Ms[crow(r, h)]);
      s1[r] = fmaf(s1[r], fs, Ms[32 + crow(r, h)]);
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
    // the online-softmax rescale of O, with the move to this tile's V exponent folded in
    const float oa = ldexpf(alpha, ev - ev_o);
    ev_o = ev;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      o0[r] *= oa;
      o1[r] *= oa;
    }
    if (kDrop) {
      uint32_t myword = 0;
      hx::attn::drop_step<0>(s0, s1, keepbits, inv_keep, myword);
      if (Sp <= kMaxStagedTiles * 64)
        Wst[t * 256 + w * 64 + lane] = myword;
      else
        dmask[((int64_t)bh * Sp + kt + lane) * (Sp >> 5) + (q0w >> 5)] = myword;
    }
    // ---- O^T += V^T . P^T : P's pieces from the accumulator, V^T rows from the piece images
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f16x8 pp[2];
      if (g == 0) sp8(acc8<0>(s0), ps, pp);
      else if (g == 1) sp8(acc8<8>(s0), ps, pp);
      else if (g == 2) sp8(acc8<0>(s1), ps, pp);
      else sp8(acc8<8>(s1), ps, pp);
      f16x8 va[2], vb[2];
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) {
        va[pc] = *reinterpret_cast<const f16x8*>(&Vt[pc][l32 * RS + 16 * g + 8 * h]);
        vb[pc] = *reinterpret_cast<const f16x8*>(&Vt[pc][(32 + l32) * RS + 16 * g + 8 * h]);
      }
      HX_X3(o0, va, pp);
      HX_X3(o1, vb, pp);
    }
    if (t + 1 < nt) {
      add_bias();
      tile_max();                // the next tile's max |K|, |V| (its loads have landed)
      __syncthreads();           // every wave is done with this tile's images; maxima published
      ek = f16_scale_exp(max4(Mx));
      ev = f16_scale_exp(max4(Mx + 4));
      stage_store(ldexpf(1.f, ek), ldexpf(1.f, ev));
      __syncthreads();
    }
  }

  // ---- epilogue
  if (kDrop && Sp <= kMaxStagedTiles * 64) {
    for (int t = 0; t < nt; ++t)
      dmask[((int64_t)bh * Sp + t * 64 + lane) * (Sp >> 5) + (q0w >> 5)] = Wst[t * 256 + w * 64 + lane];
  }
  const float inv_l = ldexpf(1.f / l_run, -(ep + ev_o));
  if (amax_part) {
    // max |context| of each query row over this head's 64 columns (lanes l and l + 32 hold its two
    // halves) -> amax_part[row][head]: the attention-output GEMM's per-row operand scale
    // (ops/gemm16.py takes the max over the nh heads of a row)
    float am = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) am = fmaxf(am, fmaxf(fabsf(o0[i] * inv_l), fabsf(o1[i] * inv_l)));
    am = fmaxf(am, __shfl_xor(am, 32, 64));
    if (q < S && h == 0) amax_part[((int64_t)b * S + q) * nh + hd] = am;
  }
  if (colmax_part) {
    // max |context| of each of the head's 64 columns over this block's 128 queries ->
    // colmax_part[b * query blocks + block][column]: the attention-output weight gradient's
    // per-column scale.  A column's 32 queries of a wave are the 32 lanes of a half.
    __shared__ float cmx_s[4][64];
    // transposing max-reduction over the 32 queries of a half-wave: at each level (lane masks 16 ..
    // 1) a lane keeps the half of its values its lane bit selects and takes the partner's other
    // half; after 31 shuffles (not 32 x 5) lane l32 holds the max of value l32 over the half
    float v[32];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      v[i] = q < S ? fabsf(o0[i] * inv_l) : 0.f;
      v[16 + i] = q < S ? fabsf(o1[i] * inv_l) : 0.f;
    }
#pragma unroll
    for (int m = 16, n = 32; m >= 1; m >>= 1, n >>= 1) {
      const bool up = (l32 & m) != 0;
#pragma unroll
      for (int j = 0; j < n / 2; ++j) {
        const float keepv = up ? v[j + n / 2] : v[j], sendv = up ? v[j] : v[j + n / 2];
        v[j] = fmaxf(keepv, __shfl_xor(sendv, m, 64));
      }
    }
    {
      const int k = l32 & 15;   // value l32: o0 (l32 < 16) or o1 (l32 >= 16) register k
      const int d = 8 * (k >> 2) + 4 * h + (k & 3);
      cmx_s[w][(l32 < 16 ? 0 : 32) + d] = v[0];
    }
    __syncthreads();
    if (tid < 64)
      colmax_part[((int64_t)b * gridDim.x + blk.x) * H + hd * D + tid] =
          fmaxf(fmaxf(cmx_s[0][tid], cmx_s[1][tid]), fmaxf(cmx_s[2][tid], cmx_s[3][tid]));
  }
  if (q >= S) return;
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

#undef HX_X3_16
#undef HX_X3

}  // namespace

void hx_attn_fwd_f16(const float* qkv, const float* bias, const float* maskb, float* out, float* lse,
                     uint32_t* dmask, int B, int S, int nh, float keep, const uint64_t* seed, uint64_t stream,
                     hipStream_t s, float* amax_part, float* colmax_part) {
  dim3 grid((S + 127) / 128, nh, B);
  if (keep < 1.f)
    attn_fwd_f16_k<true><<<grid, 256, 0, s>>>(qkv, bias, maskb, out, lse, dmask, S, nh, keep, seed, stream, amax_part,
                                              colmax_part);
  else
    attn_fwd_f16_k<false><<<grid, 256, 0, s>>>(qkv, bias, maskb, out, lse, dmask, S, nh, keep, seed, stream,
                                               amax_part, colmax_part);
}

void hx_attn_bwd_f16(const float* qkv, const float* bias, float* dbias_part, const float* maskb, const float* dout,
                     const float* out, const float* lse, const uint32_t* dmask, float* dqkv, float* dq_acc, int dq_ld,
                     int B, int S, int nh, float keep, hipStream_t s, float* amax_part, float* colmax_part) {
  dim3 grid((S + 127) / 128, nh, B);
  static bool attr = false;
  if (!attr) {   // > 64 KiB of dynamic LDS needs an explicit opt-in (gfx950: 160 KiB per CU)
    const void* k[2] = {reinterpret_cast<const void*>(&attn_bwd_f16_k<true>),
                        reinterpret_cast<const void*>(&attn_bwd_f16_k<false>)};
    for (const void* f : k) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, BWD_SMEM);
    attr = true;
  }
  if (keep < 1.f)
    attn_bwd_f16_k<true><<<grid, 256, BWD_SMEM, s>>>(qkv, bias, dbias_part, maskb, dout, out, lse, dmask, dqkv, dq_acc,
                                                     dq_ld, S, nh, keep, amax_part, colmax_part);
  else
    attn_bwd_f16_k<false><<<grid, 256, BWD_SMEM, s>>>(qkv, bias, dbias_part, maskb, dout, out, lse, dmask, dqkv,
                                                      dq_acc, dq_ld, S, nh, keep, amax_part, colmax_part);
}
