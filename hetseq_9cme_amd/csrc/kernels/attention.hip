// Fused scaled-dot-product attention forward / backward for BERT on gfx950
// (exact-fp32 MFMA: v_mfma_f32_32x32x2_f32, 64 FLOP/clk/SIMD, no TF32 shortcut).
//
// Reference (hetseq/bert_modeling.py:351-377): Q.K^T batched GEMM,
// /sqrt(d), + additive mask (1-m)*-10000, softmax, dropout(p=0.1) on the probs,
// probs.V, head permutes + .contiguous() copies -- [B, nh, S, S] fp32 scores and
// probs materialised (25 MB / 403 MB per layer at S=128/512, B=32) and ~10 kernels.
// Here one kernel per direction, no S x S tensor in HBM:
//
//  * reads Q/K/V straight from the packed [B, S, 3H] QKV-projection output
//    (head h = columns h*64..h*64+63 of each third) and writes the context in
//    [B, S, H] layout -- no permute copies (K05 removed);
//  * forward ("swapped" orientation): each wave owns 32 queries ON THE LANES, keys
//    in the accumulator REGISTERS: S^T = K.Q^T (A = K from LDS, B = Q held in 32
//    VGPRs), so each query's softmax row lives in one lane pair (l, l^32) -- row
//    max/sum are register reductions + one cross-half shuffle; then O^T += V^T.P^T
//    consumes the probability accumulator directly as the MFMA B operand (no LDS
//    round trip, no transpose);
//  * online softmax over 64-key tiles, per-query logsumexp saved for backward;
//  * dropout mask = Philox4x32-10(seed, stream, (bh*S + q)*S + key) generated ONCE
//    in forward (1 call per 4 keys) and stored as a bitmask [B, nh, S, S/32] u32
//    (1 bit / prob, 3 MB per layer at B=128,S=128) which backward reads;
//  * backward: a workgroup owns 128 keys (4 waves x 32, keys ON THE LANES) and
//    sweeps 32-query tiles: recomputes S, P = exp(S - lse), dP = dO.V^T,
//    dS = P*(dP*mask/keep - D), and accumulates dV += Pd^T.dO and dK += dS^T.Q in
//    registers (accumulator used directly as the A operand); dQ = dS.K needs keys
//    as the reduction index, so dS takes one trip through LDS, the 4 waves' dQ
//    partials are summed in LDS and written with one fp32 atomic per element per
//    workgroup (S/128 adds per element; a plain overwrite-free sum at S=128).
//
// LDS images use a 68-float row stride so the 16-B ds_read_b128 lane groups of the
// [row = lane][32 contiguous dims] operand reads hit 16 distinct 16-B slots.
#include "hx_launch.h"
#include "hx_vec.h"
#include "hx_reduce.h"
#include "hx_attn.h"

namespace {

using hx::attn::f32x16;

constexpr int D = 64;      // head dim (BERT-base/large)
constexpr int LDK = 68;    // padded LDS row stride (floats)

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
using hx::attn::crow;
using hx::attn::drop_step;

// ============================================================================ forward
// grid (S/128, nh, B), block 256 = 4 waves x 32 queries.
template <typename T, bool kDrop>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void attn_fwd_k(const T* __restrict__ qkv, const float* __restrict__ qkv_bias,
                                                const float* __restrict__ maskb,
                                                T* __restrict__ out, float* __restrict__ lse,
                                                uint32_t* __restrict__ dmask, int S, int nh, float keep,
                                                const uint64_t* __restrict__ seedp, uint64_t stream) {
  const uint64_t seed = *seedp;   // per-update Philox key, device-resident (graph-safe)
  __shared__ __attribute__((aligned(16))) float Ks[64 * LDK];
  __shared__ __attribute__((aligned(16))) float Vs[64 * LDK];
  __shared__ float Ms[64];
  // dropout words of this workgroup, written out after the key loop: a global store
  // inside the loop would hold every later s_waitcnt vmcnt (stores count in vmcnt)
  constexpr int kMaxStagedTiles = 8;   // S <= 512: all of BERT's positions
  __shared__ uint32_t Wst[kDrop ? kMaxStagedTiles * 256 : 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.z, hd = blockIdx.y;
  const int H = nh * D, H3 = 3 * H;
  const int q = blockIdx.x * 128 + w * 32 + l32;
  const int qc = q < S ? q : S - 1;            // rows past S: clamped loads, no stores
  const int Sp = (S + 127) & ~127;             // mask-word / RNG row pitch
  const int q0w = blockIdx.x * 128 + w * 32;    // first query of this wave (bitmask word)
  const uint32_t t16 = (uint32_t)(keep * 65536.f + 0.5f);
  const T* base = qkv + (int64_t)b * S * H3;
  const float scale = 0.125f;  // 1/sqrt(64): exact power of two

  // Q row slice held in registers: qr[s] = Q[q][h*32 + s] * scale
  float qr[32];
  {
    const T* qp = base + (int64_t)qc * H3 + hd * D + h * 32;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float4 v = hx::load4(qp + 4 * i);
      if (qkv_bias) v = add4(v, *reinterpret_cast<const float4*>(qkv_bias + hd * D + h * 32 + 4 * i));
      qr[4 * i] = v.x * scale;
      qr[4 * i + 1] = v.y * scale;
      qr[4 * i + 2] = v.z * scale;
      qr[4 * i + 3] = v.w * scale;
    }
  }
  f32x16 o0 = {0}, o1 = {0};
  float m_run = -INFINITY, l_run = 0.f;
  const float inv_keep = 1.f / keep;
  const int64_t bh = (int64_t)b * nh + hd;

  for (int kt = 0; kt < S; kt += 64) {
    // ---- stage K, V tile (64 keys x 64 dims) + mask into LDS (keys past S: -inf)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + i * 256;         // float4 index in the 64x16 tile
      const int row = e >> 4, c4 = (e & 15) * 4;
      const int kr = kt + row < S ? kt + row : S - 1;
      const T* src = base + (int64_t)kr * H3 + hd * D + c4;
      float4 kv = hx::load4(src + H), vv = hx::load4(src + 2 * H);
      if (qkv_bias) {
        kv = add4(kv, *reinterpret_cast<const float4*>(qkv_bias + H + hd * D + c4));
        vv = add4(vv, *reinterpret_cast<const float4*>(qkv_bias + 2 * H + hd * D + c4));
      }
      *reinterpret_cast<float4*>(&Ks[row * LDK + c4]) = kv;
      *reinterpret_cast<float4*>(&Vs[row * LDK + c4]) = vv;
    }
    if (tid < 64) Ms[tid] = kt + tid < S ? maskb[(int64_t)b * S + kt + tid] : -INFINITY;
    __syncthreads();

    // dropout decisions first: the Philox chain (dependent integer multiplies) has no
    // input from this tile's math, so issuing it here lets it overlap the MFMAs below
    uint32_t kb[4] = {0u, 0u, 0u, 0u};
    if (kDrop) {
      const uint64_t cbase = hx::attn::drop_counter(bh, S, q, Sp, kt, h);
#pragma unroll
      for (int j = 0; j < 4; ++j) kb[j] = hx::keep8(seed, stream, cbase + j, t16);
    }
    // ---- S^T = K . Q^T for two 32-key sub-blocks; keys in registers, queries on lanes
    f32x16 s0 = {0}, s1 = {0};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 ka = *reinterpret_cast<const float4*>(&Ks[l32 * LDK + h * 32 + 4 * i]);
      const float4 kb = *reinterpret_cast<const float4*>(&Ks[(32 + l32) * LDK + h * 32 + 4 * i]);
      s0 = mfma(ka.x, qr[4 * i], s0);
      s1 = mfma(kb.x, qr[4 * i], s1);
      s0 = mfma(ka.y, qr[4 * i + 1], s0);
      s1 = mfma(kb.y, qr[4 * i + 1], s1);
      s0 = mfma(ka.z, qr[4 * i + 2], s0);
      s1 = mfma(kb.z, qr[4 * i + 2], s1);
      s0 = mfma(ka.w, qr[4 * i + 3], s0);
      s1 = mfma(kb.w, qr[4 * i + 3], s1);
    }
    // + mask, tile max
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
      // decisions kb[] were drawn before the MFMAs (4 Philox calls x 8 16-bit
      // decisions; counter = (query, tile, lane half, call) -- any bijection works,
      // backward reads the stored bits); transposed bitmask [key][query word]
      uint32_t myword = 0;
      drop_step<0>(s0, s1, kb, inv_keep, myword);
      if (Sp <= kMaxStagedTiles * 64)
        Wst[(kt >> 6) * 256 + w * 64 + lane] = myword;
      else
        dmask[((int64_t)bh * Sp + kt + lane) * (Sp >> 5) + (q0w >> 5)] = myword;
    }
    // ---- O^T += V^T . P^T   (A = V^T from LDS, B = P accumulator register)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = crow(r, h);
      const float va0 = Vs[key * LDK + l32], va1 = Vs[key * LDK + 32 + l32];
      const float vb0 = Vs[(32 + key) * LDK + l32], vb1 = Vs[(32 + key) * LDK + 32 + l32];
      o0 = mfma(va0, s0[r], o0);
      o1 = mfma(va1, s0[r], o1);
      o0 = mfma(vb0, s1[r], o0);
      o1 = mfma(vb1, s1[r], o1);
    }
    __syncthreads();
  }
  // ---- epilogue: O = O^T^T / l ; lane owns query q, registers hold 4-contiguous dims
  if (kDrop && Sp <= kMaxStagedTiles * 64) {
    // (each wave reads back only its own words: no barrier needed)
    const int nt = (S + 63) >> 6;
    for (int t = 0; t < nt; ++t)
      dmask[((int64_t)bh * Sp + t * 64 + lane) * (Sp >> 5) + (q0w >> 5)] = Wst[t * 256 + w * 64 + lane];
  }
  if (q >= S) return;
  const float inv_l = 1.f / l_run;
  T* op = out + ((int64_t)b * S + q) * H + hd * D;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d0 = 8 * g + 4 * h;
    hx::store4(op + d0,
               make_float4(o0[4 * g] * inv_l, o0[4 * g + 1] * inv_l, o0[4 * g + 2] * inv_l, o0[4 * g + 3] * inv_l));
    hx::store4(op + 32 + d0,
               make_float4(o1[4 * g] * inv_l, o1[4 * g + 1] * inv_l, o1[4 * g + 2] * inv_l, o1[4 * g + 3] * inv_l));
  }
  if (h == 0) lse[bh * S + q] = m_run + __logf(l_run);
}

// ============================================================================ backward
// grid (S/128, nh, B), block 256 = 4 waves; wave w owns keys kbase + w*32 .. +31 (ON THE LANES).
// Sized for TWO workgroups per CU (LDS <= 80 KiB, <= 256 VGPRs): V lives in registers
// (each lane: its key's 32 dims of its half), only K (both MFMA layouts need it), the
// current 32-query tile of Q / dO and the tile's dS go through LDS.  Per 32-query tile:
//   S = Q.K^T, dP = dO.V^T                       (32x32x2, queries rows / keys lanes)
//   P = exp(S + mask - lse), dS = P*(dP*drop/keep - D)
//   dV += Pd^T.dO, dK += dS^T.Q                  (accumulators as the A operand)
//   dQ = dS.K over all 128 keys                  (16x16x4: each wave owns 2 of the 8
//                                                 16x16 output tiles -> no cross-wave sum)
// D = rowsum(dO * O) is computed while staging the tile (no separate pass), and the next
// tile's Q / dO / O / lse / dropout words are prefetched into registers during compute.
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int LDSS = 132;   // dS row stride ([32 q][128 keys])

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <typename T, bool kDrop>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_bwd_k(const T* __restrict__ qkv, const float* __restrict__ qkv_bias,
                                                float* __restrict__ dbias_part, const float* __restrict__ maskb,
                                                const T* __restrict__ dout, const T* __restrict__ outp,
                                                const float* __restrict__ lse, const uint32_t* __restrict__ dmask,
                                                T* __restrict__ dqkv, float* __restrict__ dq_acc, int dq_ld,
                                                int S, int nh, float keep) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ks = smem;                      // [128][LDK]
  float* Qs = Ks + 128 * LDK;            // [32][LDK]  (pre-scaled Q tile)
  float* dOs = Qs + 32 * LDK;            // [32][LDK]
  float* dSs = dOs + 32 * LDK;           // [32][LDSS]
  float* Ls = dSs + 32 * LDSS;           // [32] lse
  float* Ds = Ls + 32;                   // [32] D

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.z, hd = blockIdx.y;
  const int H = nh * D, H3 = 3 * H;
  const int kbase = blockIdx.x * 128;
  const bool single = gridDim.x == 1;          // one workgroup sees every key: dQ is final
  const T* base = qkv + (int64_t)b * S * H3;
  const int64_t bh = (int64_t)b * nh + hd;
  const float scale = 0.125f, inv_keep = 1.f / keep;
  const int Sp = (S + 127) & ~127;
  const int nwords = Sp >> 5;                   // query words per key row of the bitmask

  // ---- K of this block's 128 keys -> LDS; V of this lane's key / dim-half -> registers
  // (keys past S: clamped loads, -inf mask -> P = 0, never stored)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = tid + i * 256;
    const int row = e >> 4, c4 = (e & 15) * 4;
    const int kr = kbase + row < S ? kbase + row : S - 1;
    float4 kv = hx::load4(base + (int64_t)kr * H3 + H + hd * D + c4);
    if (qkv_bias) kv = add4(kv, *reinterpret_cast<const float4*>(qkv_bias + H + hd * D + c4));
    *reinterpret_cast<float4*>(&Ks[row * LDK + c4]) = kv;
  }
  const int mykey = kbase + w * 32 + l32;     // key on this lane
  const int mykc = mykey < S ? mykey : S - 1;
  float vr[32];
  {
    const T* vp = base + (int64_t)mykc * H3 + 2 * H + hd * D + h * 32;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float4 v = hx::load4(vp + 4 * i);
      if (qkv_bias) v = add4(v, *reinterpret_cast<const float4*>(qkv_bias + 2 * H + hd * D + h * 32 + 4 * i));
      vr[4 * i] = v.x; vr[4 * i + 1] = v.y; vr[4 * i + 2] = v.z; vr[4 * i + 3] = v.w;
    }
  }
  const float mk = mykey < S ? maskb[(int64_t)b * S + mykey] : -INFINITY;
  const float* Kw = Ks + (w * 32) * LDK;      // this wave's keys

  T* dqkv_b = dqkv + (int64_t)b * S * H3 + hd * D;
  // multi-block (S > 128): dQ partial sums are added atomically into an fp32 buffer
  // (dqkv itself when T = float, a separate [B, S, H] scratch for bf16)
  float* dqa_b = dq_acc ? dq_acc + (int64_t)b * S * dq_ld + hd * D : nullptr;
  // staging map of a 32x64 tile: thread -> rows (tid>>4) and 16 + (tid>>4), float4 column c4
  const int srow = tid >> 4, sc4 = (tid & 15) * 4;
  // Per-(b, head) bases are wave-uniform (SGPRs); per-lane offsets within one
  // sequence fit 32 bits.  Keeping the per-lane addresses 32-bit keeps this kernel
  // under 256 VGPRs without spills -- a spilled address is reloaded from scratch,
  // and scratch loads count in vmcnt: the reload's wait would drain the prefetch.
  const T* dout_b = dout + (int64_t)b * S * H + hd * D;
  const T* out_b = outp + (int64_t)b * S * H + hd * D;
  const T* qkv_bh = base + hd * D;
  const float* lse_bh = lse + bh * S;
  // dropout bits of (this lane's key, the 32 queries of a tile): ONE word
  const uint32_t* dmask_bh = kDrop ? dmask + (int64_t)bh * Sp * nwords : nullptr;
  const int moff = mykey * nwords;
  auto ld_tile = [&](int qt, float4 (&qn)[2], float4 (&dn)[2], float& xn, uint32_t& mn) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int qr = qt + srow + 16 * i;
      const int r = qr < S ? qr : S - 1;
      qn[i] = hx::load4(qkv_bh + r * H3 + sc4);
      dn[i] = hx::load4(dout_b + r * H + sc4);
    }
    // unconditional (clamped) loads: a branch around a load makes the compiler's
    // vmcnt tracking fall back to vmcnt(0), which would wait out the whole prefetch
    const int lq = qt + (tid & 31);
    xn = lse_bh[lq < S ? lq : S - 1];
    if (kDrop) mn = dmask_bh[moff + (qt >> 5)];
  };
  float4 qn[2], dn[2];
  float xn = 0.f;
  uint32_t mn = 0;
  ld_tile(0, qn, dn, xn, mn);

  // dQ tiles of this wave (16x16x4 layout): queries qh*16.., dims 16*dqa.. and 16*(dqa+1)..
  const int qh = w & 1, dqa = 2 * (w >> 1);
  const int r16 = lane & 15, k4 = lane >> 4;

  f32x16 dv0 = {0}, dv1 = {0}, dk0 = {0}, dk1 = {0};
  float cq0 = 0.f, cq1 = 0.f;   // this lane's share of the dQ column sums (bias gradient)

  for (int qt = 0; qt < S; qt += 32) {
    __syncthreads();  // previous tile's LDS buffers are free
    float4 on[2];   // O rows for D = rowsum(dO * O): loaded here (not prefetched) to stay in 256 VGPRs
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int qr = qt + srow + 16 * i;
      on[i] = hx::load4(out_b + (qr < S ? qr : S - 1) * H + sc4);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float4 qv = qn[i];
      if (qkv_bias) qv = add4(qv, *reinterpret_cast<const float4*>(qkv_bias + hd * D + sc4));
      qv.x *= scale; qv.y *= scale; qv.z *= scale; qv.w *= scale;
      *reinterpret_cast<float4*>(&Qs[(srow + 16 * i) * LDK + sc4]) = qv;
      *reinterpret_cast<float4*>(&dOs[(srow + 16 * i) * LDK + sc4]) = dn[i];
      float d = dn[i].x * on[i].x + dn[i].y * on[i].y + dn[i].z * on[i].z + dn[i].w * on[i].w;
      d += __shfl_xor(d, 1, 64);
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 4, 64);
      d += __shfl_xor(d, 8, 64);
      if ((tid & 15) == 0) Ds[srow + 16 * i] = d;
    }
    if (tid < 32) Ls[tid] = qt + tid < S ? xn : INFINITY;   // rows past S: P = 0
    const uint32_t mword = mn;
    if (qt + 32 < S) ld_tile(qt + 32, qn, dn, xn, mn);   // in flight during this tile's math
    __syncthreads();

    // ---- S = Qs . K^T (queries rows, keys on lanes); dP = dO . V^T
    f32x16 sa = {0}, dp = {0};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 qa = *reinterpret_cast<const float4*>(&Qs[l32 * LDK + h * 32 + 4 * i]);
      const float4 ka = *reinterpret_cast<const float4*>(&Kw[l32 * LDK + h * 32 + 4 * i]);
      const float4 da = *reinterpret_cast<const float4*>(&dOs[l32 * LDK + h * 32 + 4 * i]);
      sa = mfma(qa.x, ka.x, sa);
      dp = mfma(da.x, vr[4 * i], dp);
      sa = mfma(qa.y, ka.y, sa);
      dp = mfma(da.y, vr[4 * i + 1], dp);
      sa = mfma(qa.z, ka.z, sa);
      dp = mfma(da.z, vr[4 * i + 2], dp);
      sa = mfma(qa.w, ka.w, sa);
      dp = mfma(da.w, vr[4 * i + 3], dp);
      if (i & 1) __builtin_amdgcn_sched_barrier(0);
    }
    // P = exp(S + mask - lse) ; Pd = P*drop/keep ; dS = P * (dP*drop/keep - D)   (in place)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qr_ = crow(r, h);
      const float p = __expf(sa[r] + mk - Ls[qr_]);
      float keepf = 1.f;
      if (kDrop) keepf = ((mword >> qr_) & 1) ? inv_keep : 0.f;
      sa[r] = p * keepf;
      dp[r] = p * (dp[r] * keepf - Ds[qr_]);
      dSs[qr_ * LDSS + w * 32 + l32] = dp[r];
      if ((r & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
    // ---- dV += Pd^T . dO ; dK += dS^T . Qs   (accumulators as A operand, step r <-> register r)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qr_ = crow(r, h);
      const float d0 = dOs[qr_ * LDK + l32], d1 = dOs[qr_ * LDK + 32 + l32];
      const float q0 = Qs[qr_ * LDK + l32], q1 = Qs[qr_ * LDK + 32 + l32];
      dv0 = mfma(sa[r], d0, dv0);
      dv1 = mfma(sa[r], d1, dv1);
      dk0 = mfma(dp[r], q0, dk0);
      dk1 = mfma(dp[r], q1, dk1);
      if ((r & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // every wave's dS columns are in LDS
    __builtin_amdgcn_sched_barrier(0);
    // ---- dQ = dS . K over the block's 128 keys: two 16x16 tiles per wave
    f32x4 qa0 = {0}, qa1 = {0};
#pragma unroll 8
    for (int s = 0; s < 32; ++s) {
      const int key = 4 * s + k4;
      const float a = dSs[(qh * 16 + r16) * LDSS + key];
      qa0 = mfma16(a, Ks[key * LDK + dqa * 16 + r16], qa0);
      qa1 = mfma16(a, Ks[key * LDK + dqa * 16 + 16 + r16], qa1);
      if ((s & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
    const int q0 = qt + qh * 16 + 4 * k4;
    if (dbias_part) {   // rows past S hold exact zeros (their P, hence dS, is 0)
      cq0 += (qa0[0] + qa0[1]) + (qa0[2] + qa0[3]);
      cq1 += (qa1[0] + qa1[1]) + (qa1[2] + qa1[3]);
    }
    if (single) {
      T* dq = dqkv_b + q0 * H3 + dqa * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (q0 + r >= S) continue;
        hx::io<T>::st(dq + r * H3, qa0[r] * scale);
        hx::io<T>::st(dq + r * H3 + 16, qa1[r] * scale);
      }
    } else {
      float* dq = dqa_b + q0 * dq_ld + dqa * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (q0 + r >= S) continue;
        atomicAdd(dq + r * dq_ld, qa0[r] * scale);
        atomicAdd(dq + r * dq_ld + 16, qa1[r] * scale);
      }
    }
  }
  // ---- epilogue: dK (accumulated against pre-scaled Q -> already scaled), dV
  T* dk = dqkv + (int64_t)b * S * H3 + H + hd * D;
  T* dvp = dqkv + (int64_t)b * S * H3 + 2 * H + hd * D;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int key = kbase + w * 32 + crow(r, h);
    if (key >= S) continue;
    hx::io<T>::st(dk + (int64_t)key * H3 + l32, dk0[r]);
    hx::io<T>::st(dk + (int64_t)key * H3 + 32 + l32, dk1[r]);
    hx::io<T>::st(dvp + (int64_t)key * H3 + l32, dv0[r]);
    hx::io<T>::st(dvp + (int64_t)key * H3 + 32 + l32, dv1[r]);
  }
  if (dbias_part) {
    // QKV-bias gradient = column sums of dQ, dK, dV.  Per workgroup: dK / dV over
    // its 128 keys (accumulator rows), dQ over every query for its key block (the
    // per-key-block dQ partials add up to dQ).  One row of 3H partials per
    // (batch, key block); a fold kernel sums the rows into the bias-grad slots.
    float sk0 = 0.f, sk1 = 0.f, sv0 = 0.f, sv1 = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sk0 += dk0[r]; sk1 += dk1[r]; sv0 += dv0[r]; sv1 += dv1[r];
    }
    sk0 += __shfl_xor(sk0, 32, 64); sk1 += __shfl_xor(sk1, 32, 64);
    sv0 += __shfl_xor(sv0, 32, 64); sv1 += __shfl_xor(sv1, 32, 64);
    cq0 += __shfl_xor(cq0, 16, 64); cq0 += __shfl_xor(cq0, 32, 64);
    cq1 += __shfl_xor(cq1, 16, 64); cq1 += __shfl_xor(cq1, 32, 64);
    cq0 *= scale;   // dQ = scale * dS.K (the accumulators are pre-scale)
    cq1 *= scale;
    __syncthreads();                          // every wave is done with dSs
    float* red = dSs;                         // [4 waves][3][64]
    if (lane < 32) {
      red[(w * 3 + 1) * 64 + l32] = sk0; red[(w * 3 + 1) * 64 + 32 + l32] = sk1;
      red[(w * 3 + 2) * 64 + l32] = sv0; red[(w * 3 + 2) * 64 + 32 + l32] = sv1;
    }
    if (lane < 16) {   // dQ columns dqa*16 + lane and dqa*16 + 16 + lane of this wave's query half
      red[(w * 3) * 64 + dqa * 16 + lane] = cq0;
      red[(w * 3) * 64 + dqa * 16 + 16 + lane] = cq1;
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

size_t hx_attn_bwd_smem_bytes() {
  return sizeof(float) * (128 * LDK + 2 * 32 * LDK + 32 * LDSS + 64);
}

namespace {

template <typename T>
void attn_fwd_t(const void* qkv, const float* bias, const float* maskb, void* out, float* lse, uint32_t* dmask, int B,
                int S, int nh, float keep, const uint64_t* seed, uint64_t stream, hipStream_t s) {
  dim3 grid((S + 127) / 128, nh, B);
  if (keep < 1.f)
    attn_fwd_k<T, true><<<grid, 256, 0, s>>>((const T*)qkv, bias, maskb, (T*)out, lse, dmask, S, nh, keep, seed,
                                             stream);
  else
    attn_fwd_k<T, false><<<grid, 256, 0, s>>>((const T*)qkv, bias, maskb, (T*)out, lse, dmask, S, nh, keep, seed,
                                              stream);
}

template <typename T>
void attn_bwd_t(const void* qkv, const float* bias, float* dbias_part, const float* maskb, const void* dout,
                const void* out, const float* lse, const uint32_t* dmask, void* dqkv, float* dq_acc, int dq_ld, int B,
                int S, int nh, float keep, hipStream_t s) {
  dim3 grid((S + 127) / 128, nh, B);
  const size_t smem = hx_attn_bwd_smem_bytes();
  static bool attr = false;
  if (!attr) {  // > 64 KiB dynamic LDS needs an explicit opt-in (gfx950 has 160 KiB per CU)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd_k<T, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd_k<T, false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr = true;
  }
  if (keep < 1.f)
    attn_bwd_k<T, true><<<grid, 256, smem, s>>>((const T*)qkv, bias, dbias_part, maskb, (const T*)dout,
                                                (const T*)out, lse, dmask, (T*)dqkv, dq_acc, dq_ld, S, nh, keep);
  else
    attn_bwd_k<T, false><<<grid, 256, smem, s>>>((const T*)qkv, bias, dbias_part, maskb, (const T*)dout,
                                                 (const T*)out, lse, dmask, (T*)dqkv, dq_acc, dq_ld, S, nh, keep);
}

}  // namespace

void hx_attn_fwd(int bf16, const void* qkv, const float* bias, const float* maskb, void* out, float* lse,
                 uint32_t* dmask, int B, int S, int nh, float keep, const uint64_t* seed, uint64_t stream, hipStream_t s) {
  if (bf16) hx_attn_fwd_bf16(qkv, bias, maskb, out, lse, dmask, B, S, nh, keep, seed, stream, s);  // bf16 MFMA
  else attn_fwd_t<float>(qkv, bias, maskb, out, lse, dmask, B, S, nh, keep, seed, stream, s);
}

void hx_attn_bwd(int kind, const void* qkv, const float* bias, float* dbq, float* dbk, float* dbv, float* dbias_part,
                 const float* maskb, const void* dout, const void* out, const float* lse, const uint32_t* dmask,
                 void* dqkv, float* dq_acc, int dq_ld, int B, int S, int nh, float keep, hipStream_t s,
                 float* amax_part, float* colmax_part) {
  if (kind == 1)   // bf16 MFMA (attention_bf16.hip)
    hx_attn_bwd_bf16(qkv, bias, dbias_part, maskb, dout, out, lse, dmask, dqkv, dq_acc, dq_ld, B, S, nh, keep, s);
  else if (kind == 3)   // fp32 on fp16 MFMA, scaled two-piece operands (attention_f16.hip)
    hx_attn_bwd_f16((const float*)qkv, bias, dbias_part, maskb, (const float*)dout, (const float*)out, lse, dmask,
                    (float*)dqkv, dq_acc, dq_ld, B, S, nh, keep, s, amax_part, colmax_part);
  else
    attn_bwd_t<float>(qkv, bias, dbias_part, maskb, dout, out, lse, dmask, dqkv, dq_acc, dq_ld, B, S, nh, keep, s);
  if (dbias_part) {
    // [B * key blocks][3H] partial rows -> dbq | dbk | dbv (H each)
    const int H = nh * D;
    hx::fold_rows(dbias_part, B * ((S + 127) / 128), 3 * (int64_t)H, 3 * H, H, dbq, dbk, dbv, 0, s);
  }
}
