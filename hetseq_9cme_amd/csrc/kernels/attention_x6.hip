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

// x -> three bf16 pieces (x0 + x1 + x2 = x to 2^-26 relative)
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
  f32x8 v = {x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]};
  p0 = __builtin_convertvector(v, bf16x8);
  v -= __builtin_convertvector(p0, f32x8);
  p1 = __builtin_convertvector(v, bf16x8);
  v -= __builtin_convertvector(p1, f32x8);
  p2 = __builtin_convertvector(v, bf16x8);
}
template <int O>
__device__ __forceinline__ void split_acc(const f32x16& s, bf16x8 (&p)[3]) {
  const float x[8] = {s[O], s[O + 1], s[O + 2], s[O + 3], s[O + 4], s[O + 5], s[O + 6], s[O + 7]};
  split8(x, p[0], p[1], p[2]);
}
// one fp32 value -> its three pieces as raw bf16 bits
__device__ __forceinline__ void split1(float x, uint32_t& a, uint32_t& b, uint32_t& c) {
  const uint16_t q0 = hx::f2bf(x);
  x -= hx::bf2f(q0);
  const uint16_t q1 = hx::f2bf(x);
  x -= hx::bf2f(q1);
  a = q0;
  b = q1;
  c = hx::f2bf(x);
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
    const uint64_t* __restrict__ seedp, uint64_t stream) {
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
      const int dq = e & 15, kp2 = e >> 4;
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
      const int dq = e & 15, kp2 = e >> 4;
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
        uint32_t a0, a1, a2, b0, b1, b2;
        split1(v0[j], a0, a1, a2);
        split1(v1[j], b0, b1, b2);
        const int off = (4 * dq + j) * RW + (vpos(2 * kp2) >> 1);
        reinterpret_cast<uint32_t*>(Vt[0])[off] = a0 | (b0 << 16);
        reinterpret_cast<uint32_t*>(Vt[1])[off] = a1 | (b1 << 16);
        reinterpret_cast<uint32_t*>(Vt[2])[off] = a2 | (b2 << 16);
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
  if (q >= S) return;
  const float inv_l = 1.f / l_run;
  float* op = out + ((int64_t)b * S + q) * H + hd * D;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d0 = 8 * g + 4 * h;
    *reinterpret_cast<float4*>(op + d0) =
        make_float4(o0[4 * g] * inv_l, o0[4 * g + 1] * inv_l, o0[4 * g + 2] * inv_l, o0[4 * g + 3] * inv_l);
    *reinterpret_cast<float4*>(op + 32 + d0) =
        make_float4(o1[4 * g] * inv_l, o1[4 * g + 1] * inv_l, o1[4 * g + 2] * inv_l, o1[4 * g + 3] * inv_l);
  }
  if (h == 0) lse[bh * S + q] = m_run + __logf(l_run);
}

#undef HX_X6

}  // namespace

void hx_attn_fwd_x6(const float* qkv, const float* bias, const float* maskb, float* out, float* lse,
                    uint32_t* dmask, int B, int S, int nh, float keep, const uint64_t* seed, uint64_t stream,
                    hipStream_t s) {
  dim3 grid((S + 127) / 128, nh, B);
  if (keep < 1.f)
    attn_fwd_x6_k<true><<<grid, 256, 0, s>>>(qkv, bias, maskb, out, lse, dmask, S, nh, keep, seed, stream);
  else
    attn_fwd_x6_k<false><<<grid, 256, 0, s>>>(qkv, bias, maskb, out, lse, dmask, S, nh, keep, seed, stream);
}
