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

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int D = 64;      // head dim (BERT-base/large)
constexpr int LDK = 68;    // padded LDS row stride (floats)

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// accumulator register r of a 32x32 tile, lane half h -> row index
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// ============================================================================ forward
// grid (S/128, nh, B), block 256 = 4 waves x 32 queries.
template <bool kDrop>
__global__ __launch_bounds__(256) void attn_fwd_k(const float* __restrict__ qkv, const float* __restrict__ maskb,
                                                float* __restrict__ out, float* __restrict__ lse,
                                                uint32_t* __restrict__ dmask, int S, int nh, float keep,
                                                uint64_t seed, uint64_t stream) {
  __shared__ __attribute__((aligned(16))) float Ks[64 * LDK];
  __shared__ __attribute__((aligned(16))) float Vs[64 * LDK];
  __shared__ float Ms[64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.z, hd = blockIdx.y;
  const int H = nh * D, H3 = 3 * H;
  const int q = blockIdx.x * 128 + w * 32 + l32;
  const float* base = qkv + (int64_t)b * S * H3;
  const float scale = 0.125f;  // 1/sqrt(64): exact power of two

  // Q row slice held in registers: qr[s] = Q[q][h*32 + s] * scale
  float qr[32];
  {
    const float4* qp = reinterpret_cast<const float4*>(base + (int64_t)q * H3 + hd * D + h * 32);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 v = qp[i];
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
    // ---- stage K, V tile (64 keys x 64 dims) + mask into LDS
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + i * 256;         // float4 index in the 64x16 tile
      const int row = e >> 4, c4 = (e & 15) * 4;
      const float* src = base + (int64_t)(kt + row) * H3 + hd * D + c4;
      *reinterpret_cast<float4*>(&Ks[row * LDK + c4]) = *reinterpret_cast<const float4*>(src + H);
      *reinterpret_cast<float4*>(&Vs[row * LDK + c4]) = *reinterpret_cast<const float4*>(src + 2 * H);
    }
    if (tid < 64) Ms[tid] = maskb[(int64_t)b * S + kt + tid];
    __syncthreads();

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
      // keys of register group g (r = 4g..4g+3): sub-block kb, 8g + 4h + (0..3)
      const int64_t rowbase = (bh * S + q) * S + kt;
      uint32_t bits0 = 0, bits1 = 0;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t k0 = hx::keep4(seed, stream, (uint64_t)(rowbase + 8 * g + 4 * h) >> 2, keep);
        const uint32_t k1 = hx::keep4(seed, stream, (uint64_t)(rowbase + 32 + 8 * g + 4 * h) >> 2, keep);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s0[4 * g + j] = ((k0 >> j) & 1) ? s0[4 * g + j] * inv_keep : 0.f;
          s1[4 * g + j] = ((k1 >> j) & 1) ? s1[4 * g + j] * inv_keep : 0.f;
        }
        bits0 |= k0 << (8 * g + 4 * h);
        bits1 |= k1 << (8 * g + 4 * h);
      }
      bits0 |= __shfl_xor(bits0, 32, 64);
      bits1 |= __shfl_xor(bits1, 32, 64);
      if (h == 0) {
        uint32_t* dm = dmask + (bh * S + q) * (S >> 5) + (kt >> 5);
        dm[0] = bits0;
        dm[1] = bits1;
      }
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

// ============================================================================ backward
// D[bh, q] = sum_d dO[b,q,hd*64+d] * O[b,q,hd*64+d]   (one wave per (b,q), lanes = (hd,d) chunks)
__global__ __launch_bounds__(256) void attn_bwd_dot_k(const float* __restrict__ dout, const float* __restrict__ out,
                                                    float* __restrict__ Dv, int BS, int S, int nh) {
  const int H = nh * D;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= BS) return;
  const int lane = threadIdx.x & 63;
  const int b = (int)(row / S), q = (int)(row % S);
  // each head: 16 lanes x float4
  for (int hd = lane >> 4; hd < nh; hd += 4) {
    const int c = hd * D + (lane & 15) * 4;
    const float4 a = *reinterpret_cast<const float4*>(dout + row * H + c);
    const float4 o = *reinterpret_cast<const float4*>(out + row * H + c);
    float s = a.x * o.x + a.y * o.y + a.z * o.z + a.w * o.w;
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    s += __shfl_xor(s, 8, 64);
    if ((lane & 15) == 0) Dv[((int64_t)b * nh + hd) * S + q] = s;
  }
}

// grid (S/128, nh, B), block 256 = 4 waves; wave w owns keys k0 = blk*128 + w*32 .. +31 (on lanes).
// LDS per q-tile: Q (pre-scaled) and dO tiles, lse, D and the tile's dropout-mask
// words are staged once, so the inner loop issues no global loads.
template <bool kDrop>
__global__ __launch_bounds__(256) void attn_bwd_k(const float* __restrict__ qkv, const float* __restrict__ maskb,
                                                const float* __restrict__ dout, const float* __restrict__ lse,
                                                const float* __restrict__ Dv, const uint32_t* __restrict__ dmask,
                                                float* __restrict__ dqkv, int S, int nh, float keep) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ks = smem;                      // [128][LDK]
  float* Vs = Ks + 128 * LDK;            // [128][LDK]
  float* Qs = Vs + 128 * LDK;            // [32][LDK]  (pre-scaled Q tile)
  float* dOs = Qs + 32 * LDK;            // [32][LDK]
  float* dSs = dOs + 32 * LDK;           // [4 waves][32][33]; reused as dQ partials [4][32][65]? no: separate
  float* dQp = dSs + 4 * 32 * 33;        // [4 waves][32][65]
  float* Ls = dQp + 4 * 32 * 65;         // [32] lse
  float* Ds = Ls + 32;                   // [32] D
  uint32_t* Wm = reinterpret_cast<uint32_t*>(Ds + 32);   // [32 q][4 words] dropout bits of this key block

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.z, hd = blockIdx.y;
  const int H = nh * D, H3 = 3 * H;
  const int kbase = blockIdx.x * 128;
  const bool single = gridDim.x == 1;          // one workgroup sees every key: dQ is final
  const float* base = qkv + (int64_t)b * S * H3;
  const int64_t bh = (int64_t)b * nh + hd;
  const float scale = 0.125f, inv_keep = 1.f / keep;
  const int nwords = S >> 5;

  // ---- stage this block's 128 keys of K and V
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = tid + i * 256;
    const int row = e >> 4, c4 = (e & 15) * 4;
    const float* src = base + (int64_t)(kbase + row) * H3 + hd * D + c4;
    *reinterpret_cast<float4*>(&Ks[row * LDK + c4]) = *reinterpret_cast<const float4*>(src + H);
    *reinterpret_cast<float4*>(&Vs[row * LDK + c4]) = *reinterpret_cast<const float4*>(src + 2 * H);
  }
  const int mykey = kbase + w * 32 + l32;     // key on this lane
  const float mk = maskb[(int64_t)b * S + mykey];
  const float* Kw = Ks + (w * 32) * LDK;      // this wave's keys
  const float* Vw = Vs + (w * 32) * LDK;
  float* dSw = dSs + w * 32 * 33;
  float* dQw = dQp + w * 32 * 65;

  f32x16 dv0 = {0}, dv1 = {0}, dk0 = {0}, dk1 = {0};

  for (int qt = 0; qt < S; qt += 32) {
    __syncthreads();  // previous iteration done with the q-tile buffers
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + i * 256;          // 32 rows x 16 float4
      const int row = e >> 4, c4 = (e & 15) * 4;
      float4 qv = *reinterpret_cast<const float4*>(base + (int64_t)(qt + row) * H3 + hd * D + c4);
      qv.x *= scale; qv.y *= scale; qv.z *= scale; qv.w *= scale;
      *reinterpret_cast<float4*>(&Qs[row * LDK + c4]) = qv;
      *reinterpret_cast<float4*>(&dOs[row * LDK + c4]) =
          *reinterpret_cast<const float4*>(dout + ((int64_t)b * S + qt + row) * H + hd * D + c4);
    }
    if (tid < 32) Ls[tid] = lse[bh * S + qt + tid];
    else if (tid < 64) Ds[tid - 32] = Dv[bh * S + qt + tid - 32];
    else if (kDrop && tid < 64 + 128) {
      const int i = tid - 64, row = i >> 2, wd = i & 3;
      Wm[i] = dmask[(bh * S + qt + row) * nwords + (kbase >> 5) + wd];
    }
    __syncthreads();

    // ---- S = Qs . K^T (queries in registers, keys on lanes); dP = dO . V^T
    f32x16 sa = {0}, dp = {0};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 qa = *reinterpret_cast<const float4*>(&Qs[l32 * LDK + h * 32 + 4 * i]);
      const float4 ka = *reinterpret_cast<const float4*>(&Kw[l32 * LDK + h * 32 + 4 * i]);
      const float4 da = *reinterpret_cast<const float4*>(&dOs[l32 * LDK + h * 32 + 4 * i]);
      const float4 va = *reinterpret_cast<const float4*>(&Vw[l32 * LDK + h * 32 + 4 * i]);
      sa = mfma(qa.x, ka.x, sa);
      dp = mfma(da.x, va.x, dp);
      sa = mfma(qa.y, ka.y, sa);
      dp = mfma(da.y, va.y, dp);
      sa = mfma(qa.z, ka.z, sa);
      dp = mfma(da.z, va.z, dp);
      sa = mfma(qa.w, ka.w, sa);
      dp = mfma(da.w, va.w, dp);
    }
    // P = exp(S + mask - lse) ; Pd = P*mask/keep ; dS = P * (dP*mask/keep - D)
    f32x16 pd, ds;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qr_ = crow(r, h);
      const float p = __expf(sa[r] + mk - Ls[qr_]);
      float keepf = 1.f;
      if (kDrop) keepf = ((Wm[qr_ * 4 + w] >> l32) & 1) ? inv_keep : 0.f;
      pd[r] = p * keepf;
      ds[r] = p * (dp[r] * keepf - Ds[qr_]);
    }
    // ---- dV += Pd^T . dO ; dK += dS^T . Qs   (accumulators as A operand, step r <-> register r)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qr_ = crow(r, h);
      const float d0 = dOs[qr_ * LDK + l32], d1 = dOs[qr_ * LDK + 32 + l32];
      const float q0 = Qs[qr_ * LDK + l32], q1 = Qs[qr_ * LDK + 32 + l32];
      dv0 = mfma(pd[r], d0, dv0);
      dv1 = mfma(pd[r], d1, dv1);
      dk0 = mfma(ds[r], q0, dk0);
      dk1 = mfma(ds[r], q1, dk1);
    }
    // ---- dQ = dS . K : dS through LDS ([q][key], row stride 33); own wave only
#pragma unroll
    for (int r = 0; r < 16; ++r) dSw[crow(r, h) * 33 + l32] = ds[r];
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's dS writes landed
    __builtin_amdgcn_wave_barrier();
    f32x16 dq0 = {0}, dq1 = {0};
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int key = 2 * s + h;
      const float a = dSw[l32 * 33 + key];
      dq0 = mfma(a, Kw[key * LDK + l32], dq0);
      dq1 = mfma(a, Kw[key * LDK + 32 + l32], dq1);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dQw[crow(r, h) * 65 + l32] = dq0[r];
      dQw[crow(r, h) * 65 + 32 + l32] = dq1[r];
    }
    __syncthreads();
    // sum the 4 waves' partials; 256 threads x 8 elements of the 32x64 tile
    for (int i = tid; i < 32 * 64; i += 256) {
      const int row = i >> 6, c = i & 63, o = row * 65 + c;
      const float v = ((dQp[o] + dQp[32 * 65 + o]) + (dQp[2 * 32 * 65 + o] + dQp[3 * 32 * 65 + o])) * scale;
      float* dst = dqkv + ((int64_t)b * S + qt + row) * H3 + hd * D + c;
      if (single) *dst = v;
      else atomicAdd(dst, v);
    }
  }
  // ---- epilogue: dK (accumulated against pre-scaled Q -> already scaled), dV
  float* dk = dqkv + (int64_t)b * S * H3 + H + hd * D;
  float* dvp = dqkv + (int64_t)b * S * H3 + 2 * H + hd * D;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int key = kbase + w * 32 + crow(r, h);
    dk[(int64_t)key * H3 + l32] = dk0[r];
    dk[(int64_t)key * H3 + 32 + l32] = dk1[r];
    dvp[(int64_t)key * H3 + l32] = dv0[r];
    dvp[(int64_t)key * H3 + 32 + l32] = dv1[r];
  }
}

}  // namespace

size_t hx_attn_bwd_smem_bytes() {
  return sizeof(float) * (2 * 128 * LDK + 2 * 32 * LDK + 4 * 32 * 33 + 4 * 32 * 65 + 64 + 128);
}

void hx_attn_fwd(const float* qkv, const float* maskb, float* out, float* lse, uint32_t* dmask, int B, int S, int nh,
                 float keep, uint64_t seed, uint64_t stream, hipStream_t s) {
  dim3 grid(S / 128, nh, B);
  if (keep < 1.f)
    attn_fwd_k<true><<<grid, 256, 0, s>>>(qkv, maskb, out, lse, dmask, S, nh, keep, seed, stream);
  else
    attn_fwd_k<false><<<grid, 256, 0, s>>>(qkv, maskb, out, lse, dmask, S, nh, keep, seed, stream);
}

void hx_attn_bwd(const float* qkv, const float* maskb, const float* dout, const float* out, const float* lse,
                 const uint32_t* dmask, float* Dws, float* dqkv, int B, int S, int nh, float keep, hipStream_t s) {
  const int BS = B * S;
  attn_bwd_dot_k<<<(BS + 3) / 4, 256, 0, s>>>(dout, out, Dws, BS, S, nh);
  dim3 grid(S / 128, nh, B);
  const size_t smem = hx_attn_bwd_smem_bytes();
  static bool attr = false;
  if (!attr) {  // > 64 KiB dynamic LDS needs an explicit opt-in (gfx950 has 160 KiB per CU)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd_k<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd_k<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr = true;
  }
  if (keep < 1.f)
    attn_bwd_k<true><<<grid, 256, smem, s>>>(qkv, maskb, dout, lse, Dws, dmask, dqkv, S, nh, keep);
  else
    attn_bwd_k<false><<<grid, 256, smem, s>>>(qkv, maskb, dout, lse, Dws, dmask, dqkv, S, nh, keep);
}
