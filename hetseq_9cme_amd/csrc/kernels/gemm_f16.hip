// fp32 GEMMs on the fp16 matrix cores with THREE passes (--fp32-gemm fp16x3):
//
//   x = 2^-E (h0 + h1),  h0 = fp16(2^E x),  h1 = fp16(2^E x - h0)   (hx_gemm.h: f16_scale_exp)
//   a . b = 2^-(Ea + Eb) (a0 b0 + a0 b1 + a1 b0) + O(2^-22 |a||b|)
//
// Two RNE fp16 pieces hold 22 significant bits of an fp32 value (bf16 pieces hold 8 each, so
// fp32-class bf16 emulation needs three of them and six pair products: --fp32-gemm bf16x6).  fp16
// has 5 exponent bits, so every operand tensor is scaled by a power of two 2^E chosen from its
// largest magnitude (max |x| lands in [2^14, 2^15)): the product of two scaled pieces is exact in
// the fp32 accumulator, and the scales are undone exactly in the epilogue.  Half the matrix-core
// work of bf16x6 at fp32-class accuracy (tests/test_gemm_f16_gpu.py: fp64-referenced errors).
//
// Operands: activations and gradients are read AS fp32 and split in registers here (fp32 = 4 B per
// element; three bf16 pieces were 6), and their scale comes from the max |x| partials written by
// their producer (LayerNorm, attention, this kernel's own epilogues) or by hx_amax_rows.  A
// producer that knows a whole row when it writes it (the forward LayerNorms, ops/gemm16.py
// presplit) may instead hand over the row's two pieces, split at that same scale (AT 2: the same
// 4 B per element, read like B, no split in the k loop; bit-identical).  Weights are split once per forward
// (split_weight_f16_many_k) into the "P2" piece layout: element (r, p, k) at r 2K + (k / 16) 32 +
// p 16 + k % 16, so one 16-deep k step of a row is 64 contiguous bytes holding both pieces.
//
// Kernels (reference sites: hetseq/bert_modeling.py:334-336 Q/K/V, :383 attention output, :409 +
// :166-168 FFN-up with bias_gelu, :419 FFN-down, :538-547 MLM decoder, and their backward):
//  * gemm_f16_k   C[M][N] (+)= A[M][K] . B[N][K]^T  (forward: A = activations, B = weight pieces;
//    data gradient: A = output gradient, B = pieces of W^T).  One workgroup per BM x BN tile,
//    tiles dealt XCD-aware; LDS-DMA (buffer_load ... lds) of fp32 A and fp16 B stages, 16 deep,
//    three stages with the next-next stage's DMA pieces issued between the MFMA passes; each
//    wave reads its A fragment as fp32 (two ds_read_b128), splits it in registers and runs
//    3 x MB x NB v_mfma_f32_32x32x16_f16.  Epilogues after a 4 x 4 DPP quad transpose (16-B
//    stores): C (+)= s acc (+ bias); FFN-up bias + GELU (C = gelu'(u), P = gelu(u) fp32 + its
//    per-tile max |.|); FFN-down data gradient with the GELU backward (P = t fp32, its max |.|,
//    per-wave column partials of t = the FFN-up bias gradient).  Split-K slabs for deep
//    reductions with few tiles (the MLM decoder's data gradient).
//  * wgrad_f16_k  dW[M][N] = dY[T][M]^T . X[T][N] (tokens = reduction): both operands fp32,
//    32 tokens per stage loaded into registers, split, and written as fp16 piece tiles into an
//    XOR-swizzled LDS image read with the transposing ds_read_b64_tr_b16; token-range split-K
//    over the CUs, partial slabs summed by one vectorised pass.
#include <algorithm>
#include <type_traits>

#include "hx_gemm.h"
#include "hx_launch.h"
#include "hx_reduce.h"

namespace {

using namespace hx::g;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

__device__ __forceinline__ f32x16 mfma16(const f16x8& a, const f16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// raw workgroup barrier: no vmcnt / lgkmcnt drain (LDS-DMA and fragment reads stay in flight
// across it; the k loop retires what it needs with counted waits), and a compiler memory fence
__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }

// the two-piece split of two fp32 values (x0, x1) at scale s: h0 = fp16(s x), h1 = fp16(s x - h0),
// both round-to-nearest-even, as two packed halves -- four v_fma_mix instructions (the fma is exact
// before its one rounding), against 12 for cvt / pk_fma / cvt (hx_gemm.h split2)
__device__ __forceinline__ void split_pair_mix(float x0, float x1, float s, uint32_t& h0, uint32_t& h1) {
  asm volatile(
      "v_fma_mixlo_f16 %0, %2, %4, 0 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(h0), "=&v"(h1)
      : "v"(x0), "v"(x1), "v"(s));
}

// the same with one scale per value (the weight gradient's per-column scales)
__device__ __forceinline__ void split_pair_mix2(float x0, float x1, float s0, float s1, uint32_t& h0, uint32_t& h1) {
  asm volatile(
      "v_fma_mixlo_f16 %0, %2, %4, 0 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %3, %5, 0 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %5, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(h0), "=&v"(h1)
      : "v"(x0), "v"(x1), "v"(s0), "v"(s1));
}

struct F16Args {
  const void* A;   // fp32 (AT 0), bf16 (AT 1) or fp16 P2 pieces already split at the row scale (AT 2)
  int64_t lda;
  const float* a_amax;   // A row r's max |x| partials: a_amax[r a_rs + j], j < na (a_rs 0: one set, per tensor)
  int na, a_rs;
  const uint16_t* B;
  int64_t ldb;
  const float* b_amax;   // B row n's (= output column n's) partials, the same way
  int nb, b_rs;
  float* C;
  int64_t ldc;
  int M, N, K, beta;
  const float* bias;
  const float* aux;
  int64_t ldaux;
  float* P;
  int64_t ldp;
  float* colpart;   // EPI 2: per-wave column sums of t, [TM NWM][N]
  float* rowmax;    // EPI 1 / 2: max |P| per (row, N tile), [M][N / BN] (the consumer GEMM's row scale)
  float* colmax;    // EPI 1 / 2: max |P| per (M tile, column), [TM][N] (the weight gradient's column scale)
  int dmode;        // EPI 1: C gets gelu'(u) (1) or u (0); EPI 2: aux holds gelu'(u) (1) or u (0)
  int ks;           // split-K slabs (EPI 0 only): slab z reduces k steps [z, z + 1) K / ks into C + z c_zs
  int64_t c_zs;
};

// max |x| of `rows` operand rows starting at r0 from their partials -> scale tables (2^E, 2^-E);
// rs == 0: one per-tensor bound for every row.  Rows past `valid` get 1.
__device__ __forceinline__ void row_scales(const float* __restrict__ p, int np, int rs, int r0, int rows, int valid,
                                           float* s, float* is, float* red) {
  if (rs == 0) {
    const int E = f16_scale_exp(block_amax(p, np, red));
    for (int t = threadIdx.x; t < rows; t += blockDim.x) {
      if (s) s[t] = ldexpf(1.f, E);
      is[t] = ldexpf(1.f, -E);
    }
    return;
  }
  for (int t = threadIdx.x; t < rows; t += blockDim.x) {
    float m = 0.f;
    if (t < valid) {
      const float* q = p + (int64_t)(r0 + t) * rs;
      for (int j = 0; j < np; ++j) m = fmaxf(m, q[j]);
    }
    const int E = f16_scale_exp(m);
    if (s) s[t] = ldexpf(1.f, E);
    is[t] = ldexpf(1.f, -E);
  }
}

// ---------------------------------------------------------------- the GEMM
// C[M][N] (+)= A[M][K] . B[N][K]^T on a BM x BN tile per workgroup, NW = (BM / WM)(BN / WN) waves.
// k loop, step it (16-deep fp16x3 stage, or 32-deep bf16):
//   * the MFMA passes of stage it run on fragments already in registers (read during step it - 1),
//   * under them: the fragment reads (and, fp16x3, the fp32 -> two-piece split of A) of stage
//     it + 1, and this wave's LDS-DMA pieces of stage it + NS - 1 into the ring slot stage it - 1
//     used (its fragments were consumed in step it - 1, before the previous barrier),
//   * a counted vmcnt that leaves only stage it + NS - 1's pieces in flight (so stage it + 2 has
//     landed: NS = 4 gives every DMA two steps), then ONE raw barrier.
// The barrier opens step it + 1 straight into MFMAs: no wave waits on a fragment read after it.
// DW = 4: only waves 0 .. 3 (one per SIMD: waves w and w + 4 share a SIMD) issue the LDS-DMA pieces,
// the others only read fragments and run MFMAs -- a DMA burst then stalls one wave of a SIMD pair,
// not both (DW = 12: waves 4 .. 7 instead, measured slower)
template <int BM, int BN, int WM, int WN, int EPI, int WGS, int NS, int AT = 0, int OB = 0, int DIL = 1, int DW = 0>
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64, (BM / WM) * (BN / WN) * WGS / 4) void gemm_f16_k(F16Args g) {
  static_assert(AT != 1 || EPI == 0 || EPI == 3 || OB == 1, "bf16 operands: GELU epilogues in bf16");
  static_assert(AT >= 0 && AT <= 2, "operand kind");
  constexpr bool BF = AT == 1;           // --precision bf16 (one pass, no scales)
  static_assert(OB == 0 || AT == 1, "bf16 output with bf16 operands");
  static_assert(NS >= 3 && NS <= 5, "ring depth");
  constexpr int KD = BF ? 32 : 16;       // k elements per stage
  constexpr int AE = BF ? 2 : 4;         // A element bytes (AT 2: a row's two pieces take 4 B per k)
  constexpr int NWM = BM / WM, NWN = BN / WN, NW = NWM * NWN, NT = NW * 64;
  constexpr int MB = WM / 32, NB = WN / 32;
  constexpr int A_BYTES = BM * 64, B_BYTES = BN * 64, STAGE = A_BYTES + B_BYTES;
  constexpr int KA = BM / 16, KB = BN / 16, PTOT = KA + KB;   // 1-KiB DMA pieces per stage
  constexpr int NDW = DW > 0 ? (DW & 7) : NW;                   // waves that issue DMA
  constexpr int DW0 = DW >= 8 ? NW - NDW : 0;                   // the first of them
  static_assert(NDW <= NW && NDW > 0, "DMA waves");
  constexpr int JHI = (PTOT + NDW - 1) / NDW, JLO = PTOT / NDW;
  static_assert(JLO >= 1, "fewer DMA pieces than waves");
  static_assert(BM % 16 == 0 && BN % 16 == 0 && WM % 32 == 0 && WN % 32 == 0, "tile shape");
  static_assert(NT >= BM && NT >= BN, "one thread per table row");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* tsa = reinterpret_cast<float*>(lds + NS * STAGE);   // [BM] 2^Ea of each A row
  float* tia = tsa + BM;                                      // [BM] 2^-Ea
  float* tib = tia + BM;                                      // [BN] 2^-Eb of each B row
  float* red = tib + BN;                                      // [NW] block reductions

  const int TM = (g.M + BM - 1) / BM, TN = g.N / BN, total = TM * TN;
  const int per = (total * g.ks + 7) / 8;
  const int work0 = (blockIdx.x % 8) * per + blockIdx.x / 8;   // tiles dealt XCD by XCD
  if (work0 >= total * g.ks) return;                          // uniform per workgroup
  const int z = work0 / total, work = work0 - z * total;
  const int nt = work % TN, mt = work / TN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nit = g.K / KD / g.ks, it0 = z * nit;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w % NWM, wn = w / NWM, h = lane >> 5, l32 = lane & 31;
  const int wv = __builtin_amdgcn_readfirstlane(w);

  const int mrows = min(BM, g.M - m0);
  const u32x4 ra = rsrc_of((const char*)g.A + (int64_t)m0 * g.lda * AE, (uint32_t)((int64_t)mrows * g.lda * AE));
  const u32x4 rb = rsrc_of(g.B + (int64_t)n0 * g.ldb, (uint32_t)((int64_t)BN * g.ldb * 2));

  // this wave's DMA pieces q = wv + NW j of a stage: [A pieces (16 rows) | B pieces].  Every wave
  // issues JHI pieces (no wave-dependent branch in the k loop): a wave with JLO real pieces aims
  // the last one past every buffer (no memory traffic) into a junk KiB after the tables.
  constexpr int JUNK = NS * STAGE + (2 * BM + BN + NW) * 4;
  uint32_t voff[JHI], dbase[JHI], dslot[JHI];
  {
    int rl, ch;
    img_lane_src(lane, rl, ch);
#pragma unroll
    for (int j = 0; j < JHI; ++j) {
      const int q = wv - DW0 + NDW * j;
      if (q < KA) voff[j] = (uint32_t)(((int64_t)(q * 16 + rl) * g.lda + (16 / AE) * ch) * AE);
      else voff[j] = (uint32_t)(((int64_t)((q - KA) * 16 + rl) * g.ldb + 8 * ch) * 2);
      dbase[j] = q < PTOT ? 1024u * q : (uint32_t)JUNK;
      dslot[j] = q < PTOT ? 1u : 0u;
      if (q >= PTOT) voff[j] = 0x40000000u;   // + any k offset stays past the buffer, never wraps
    }
  }
  const uint32_t lds0 = (uint32_t)(size_t)(lds_void*)lds;
  auto dma_one = [&](int it, int j) {   // piece j of this wave for stage it (64 B of each row per stage)
    if (DW > 0 && (wv < DW0 || wv >= DW0 + NDW)) return;   // wave-uniform: a non-DMA wave
    const uint32_t st = (uint32_t)(it % NS) * STAGE;
    // stages past this slab's end: an offset past every buffer (the load returns zeros, reads nothing)
    const uint32_t ko = it < nit ? (uint32_t)(it0 + it) * 64u : 0x80000000u;
    const int q = wv - DW0 + NDW * j;   // A or B piece: uniform per wave, a select of the descriptor
    dma16(q < KA ? ra : rb, lds0 + dbase[j] + dslot[j] * st, voff[j] + ko);
  };
  auto dma = [&](int it) {   // every piece of stage it into its ring slot
#pragma unroll
    for (int j = 0; j < JHI; ++j) dma_one(it, j);
  };
  // stage it + 2 landed on this wave's side: the youngest NS - 3 stages (it + 3 .. it + NS - 1) may
  // stay in flight
  auto wait_ring = [&]() { dma_wait<(NS - 3) * JHI>(); };

#pragma unroll
  for (int i = 0; i < NS - 1; ++i) dma(i);
  if constexpr (!BF) {
    // operand scales: per row (partials per row) or per tensor (one set of partials)
    row_scales(g.a_amax, g.na, g.a_rs, m0, BM, mrows, AT == 0 ? tsa : nullptr, tia, red);
    row_scales(g.b_amax, g.nb, g.b_rs, n0, BN, BN, nullptr, tib, red);
  }
  // stages 0 and 1 landed (NS = 4: stage 2 may still be in flight)
  wait_ring();   // stages 0 and 1 landed
  __syncthreads();

  f32x16 acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = f32x16{0};

  // fragment byte offsets in a stage (fixed for the k loop)
  int offa[MB], offb[NB];
#pragma unroll
  for (int a = 0; a < MB; ++a) offa[a] = (wm * WM + 32 * a + l32) * 64;
#pragma unroll
  for (int b = 0; b < NB; ++b) offb[b] = A_BYTES + (wn * WN + 32 * b + l32) * 64;
  const int sw = 16 * ((l32 >> 2) & 3);   // chunk swizzle of the lane's rows (img_off)
  auto chunk = [&](int row_off, int ch) { return row_off + ((16 * ch) ^ sw); };

  if constexpr (AT == 2) {
    // A pieces written by their producer at the row scale (LayerNorm forward / backward): the
    // fragments are read like B's and the k step is three MFMA passes and nothing else
    struct Fr {
      f16x8 a0[MB], a1[MB], b0[NB], b1[NB];
    };
    auto read = [&](const char* st, Fr& F) {
#pragma unroll
      for (int a = 0; a < MB; ++a) {
        F.a0[a] = *reinterpret_cast<const f16x8*>(st + chunk(offa[a], h));
        F.a1[a] = *reinterpret_cast<const f16x8*>(st + chunk(offa[a], 2 + h));
      }
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        F.b0[b] = *reinterpret_cast<const f16x8*>(st + chunk(offb[b], h));
        F.b1[b] = *reinterpret_cast<const f16x8*>(st + chunk(offb[b], 2 + h));
      }
    };
    auto pass = [&](const Fr& F, int q) {
#pragma unroll
      for (int i = 0; i < MB * NB; ++i) {
        const int a = i / NB, b = i % NB;
        acc[a][b] = mfma16(q == 2 ? F.a1[a] : F.a0[a], q == 1 ? F.b1[b] : F.b0[b], acc[a][b]);
      }
    };
    auto step = [&](int it, const Fr& Fc, Fr& Fn) {   // branch-free, as the AT 0 step
      read(lds + ((it + 1) % NS) * STAGE, Fn);
      pass(Fc, 0);
#pragma unroll
      for (int i = 0; i < MB * NB; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, (2 * MB + 2 * NB + MB * NB - 1) / (MB * NB), 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      dma(it + NS - 1);
      __builtin_amdgcn_sched_barrier(0);
      pass(Fc, 1);
      pass(Fc, 2);
      __builtin_amdgcn_sched_barrier(0);
      wait_ring();
      raw_barrier();
    };
    Fr F0, F1;
    read(lds, F0);
    for (int it = 0; it < nit; it += 2) {
      step(it, F0, F1);
      if (it + 1 < nit) step(it + 1, F1, F0);
    }
  } else if constexpr (AT == 0) {
    float sa[MB];
#pragma unroll
    for (int a = 0; a < MB; ++a) sa[a] = tsa[wm * WM + 32 * a + l32];
    struct Fr {
      f16x8 a0[MB], a1[MB], b0[NB], b1[NB];
    };
    auto read_a = [&](const char* st, f32x4 (&raw)[MB][2]) {
#pragma unroll
      for (int a = 0; a < MB; ++a) {
        raw[a][0] = *reinterpret_cast<const f32x4*>(st + chunk(offa[a], 2 * h));
        raw[a][1] = *reinterpret_cast<const f32x4*>(st + chunk(offa[a], 2 * h + 1));
      }
    };
    auto read_b = [&](const char* st, Fr& F) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        F.b0[b] = *reinterpret_cast<const f16x8*>(st + chunk(offb[b], h));       // piece 0
        F.b1[b] = *reinterpret_cast<const f16x8*>(st + chunk(offb[b], 2 + h));   // piece 1
      }
    };
    auto split_a = [&](const f32x4 (&raw)[MB][2], Fr& F) {
#pragma unroll
      for (int a = 0; a < MB; ++a) {
        const f32x8 y = f32x8{raw[a][0][0], raw[a][0][1], raw[a][0][2], raw[a][0][3],
                              raw[a][1][0], raw[a][1][1], raw[a][1][2], raw[a][1][3]} * sa[a];
        split2(y, F.a0[a], F.a1[a]);
        // pin the split here: the pieces are used one step later, past the barrier, and LLVM
        // would otherwise sink the VALU into the next step's head (a VALU burst before its MFMAs)
        asm volatile("" ::"v"(F.a0[a]), "v"(F.a1[a]));
      }
    };
    auto mma = [&](const Fr& F, int q, int i) {   // MFMA i (= a NB + b) of pass q
      const int a = i / NB, b = i % NB;
      acc[a][b] = mfma16(q == 2 ? F.a1[a] : F.a0[a], q == 1 ? F.b1[b] : F.b0[b], acc[a][b]);
    };
    auto pass = [&](const Fr& F, int q) {
#pragma unroll
      for (int i = 0; i < MB * NB; ++i) mma(F, q, i);
    };
    // one k step on Fc (stage it) while stage it + 1 is read into Fn -- branch-free: past the
    // end the reads fetch a stale slot (never used) and the DMA is aimed past the buffer (no
    // memory traffic, still counted by vmcnt), so every step has the same waits.  The fragment
    // reads are spread over pass 0; the DMA pieces go as one burst (r5d: interleaving them with
    // MFMAs measured 2-5 % slower); the split of the next A fragments runs as v_fma_mix pairs, one
    // pair after each of the first pass-1 / pass-2 MFMAs (r5g: the packed cvt / pk_fma split cost
    // 17 % of the kernel).
    auto step = [&](int it, const Fr& Fc, Fr& Fn) {
      const char* nx = lds + ((it + 1) % NS) * STAGE;
      f32x4 raw[MB][2];
      read_a(nx, raw);
      read_b(nx, Fn);
      pass(Fc, 0);
#pragma unroll
      for (int i = 0; i < MB * NB; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, (2 * MB + 2 * NB + MB * NB - 1) / (MB * NB), 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      dma(it + NS - 1);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (4 * MB > 2 * MB * NB) {   // small wave tiles (NB = 1): the compiler's split
        pass(Fc, 1);
        split_a(raw, Fn);
        pass(Fc, 2);
      } else {
        uint32_t h0w[MB][4], h1w[MB][4];
#pragma unroll
        for (int i = 0; i < 2 * MB * NB; ++i) {
          mma(Fc, 1 + i / (MB * NB), i % (MB * NB));
          if (i < 4 * MB) {   // (r5i: placing the pairs after the last MFMAs instead measured the same)
            const int a = i / 4, w = i % 4;
            const f32x4& r = raw[a][w >> 1];
            split_pair_mix(r[2 * (w & 1)], r[2 * (w & 1) + 1], sa[a], h0w[a][w], h1w[a][w]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int a = 0; a < MB; ++a) {
          Fn.a0[a] = __builtin_bit_cast(f16x8, u32x4{h0w[a][0], h0w[a][1], h0w[a][2], h0w[a][3]});
          Fn.a1[a] = __builtin_bit_cast(f16x8, u32x4{h1w[a][0], h1w[a][1], h1w[a][2], h1w[a][3]});
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // stage it + 2 landed on this wave's side (stage it + NS - 1 stays in flight), then the
      // barrier publishes it to every wave and frees stage it's slot for the DMA of step it + 1
      wait_ring();
      raw_barrier();
    };
    Fr F0, F1;
    {
      f32x4 raw[MB][2];
      read_a(lds, raw);
      read_b(lds, F0);
      split_a(raw, F0);
    }
    for (int it = 0; it < nit; it += 2) {
      step(it, F0, F1);
      if (it + 1 < nit) step(it + 1, F1, F0);
    }
  } else {
    // --precision bf16: two 16-deep k halves per 32-deep stage, one MFMA pass each
    struct Fr {
      bf16x8v a[2][MB], b[2][NB];
    };
    auto read = [&](const char* st, Fr& F) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int a = 0; a < MB; ++a) F.a[ks][a] = *reinterpret_cast<const bf16x8v*>(st + chunk(offa[a], 2 * ks + h));
#pragma unroll
        for (int b = 0; b < NB; ++b) F.b[ks][b] = *reinterpret_cast<const bf16x8v*>(st + chunk(offb[b], 2 * ks + h));
      }
    };
    auto mma = [&](const Fr& F, int ks, int i) {
      const int a = i / NB, b = i % NB;
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F.a[ks][a], F.b[ks][b], acc[a][b], 0, 0, 0);
    };
    auto pass = [&](const Fr& F, int ks) {
#pragma unroll
      for (int i = 0; i < MB * NB; ++i) mma(F, ks, i);
    };
    auto step = [&](int it, const Fr& Fc, Fr& Fn) {   // branch-free, as the fp16x3 step
      read(lds + ((it + 1) % NS) * STAGE, Fn);
      pass(Fc, 0);
#pragma unroll
      for (int i = 0; i < MB * NB; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, (4 * MB + 4 * NB + MB * NB - 1) / (MB * NB), 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      constexpr int NI = DIL == 1 ? (JHI < MB * NB ? JHI : MB * NB) : 0;
#pragma unroll
      for (int j = 0; j < NI; ++j) {   // one DMA piece after each of the first MFMAs (fp16x3 step)
        mma(Fc, 1, j);
        dma_one(it + NS - 1, j);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int j = NI; j < JHI; ++j) dma_one(it + NS - 1, j);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = NI; i < MB * NB; ++i) mma(Fc, 1, i);
      __builtin_amdgcn_sched_barrier(0);
      wait_ring();
      raw_barrier();
    };
    Fr F0, F1;
    read(lds, F0);
    for (int it = 0; it < nit; it += 2) {
      step(it, F0, F1);
      if (it + 1 < nit) step(it + 1, F1, F0);
    }
  }
  // every wave is past its last fragment read before the ring is reused below
  __syncthreads();

  // output store cache policy: the GELU epilogues' two outputs (2 x 201 MB at the FFN shapes) go
  // non-temporal -- r5m: FFN up 326 -> 305 us, FFN-down dgrad 294 -> 285 us; the plain / beta
  // epilogues' outputs are read by the next kernel at once and stay cached (r5z: non-temporal
  // there too measured the same, sc0 sc1 no better)
  constexpr int SP = (EPI == 1 || EPI == 2) ? 2 : 0;
  // ---- epilogue: quad transpose, then lane (l32 & 3) owns row 8 gq + 4 h + (l32 & 3) of each
  // 32 x 32 block and its columns (l32 & ~3) .. + 3; stores past M dropped by the descriptor
  const int mrow = wm * WM + 4 * h + (l32 & 3), ncol = wn * WN + (l32 & ~3);
  const hx::Buf cbuf(g.C + z * g.c_zs + (int64_t)m0 * g.ldc + n0, (uint32_t)((int64_t)mrows * g.ldc * 4));
  auto coff = [&](int a, int b, int gq) { return (uint32_t)((mrow + 32 * a + 8 * gq) * g.ldc + ncol + 32 * b) * 4; };
  float ibc[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i) ibc[b][i] = BF ? 1.f : tib[ncol + 32 * b + i];
  auto tr = [&](int a, int b, int gq, float (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = acc[a][b][4 * gq + i];
    transpose4(v, lane);
    if constexpr (!BF) {
      const float ir = tia[mrow + 32 * a + 8 * gq];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = v[i] * ir * ibc[b][i];
    }
  };
  float bias[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g.bias) t = *reinterpret_cast<const float4*>(g.bias + n0 + ncol + 32 * b);
    bias[b][0] = t.x; bias[b][1] = t.y; bias[b][2] = t.z; bias[b][3] = t.w;
  }
  if constexpr (OB == 1 && (EPI == 0 || EPI == 3)) {
    // bf16 output [M][ldc]: 4 consecutive columns of a row per lane -> one 8-B store
    const hx::Buf obuf(reinterpret_cast<uint16_t*>(g.C) + (int64_t)m0 * g.ldc + n0, (uint32_t)((int64_t)mrows * g.ldc * 2));
#pragma unroll
    for (int a = 0; a < MB; ++a) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          float v[4];
          tr(a, b, gq, v);
          const uint32_t off = (uint32_t)((mrow + 32 * a + 8 * gq) * g.ldc + ncol + 32 * b) * 2;
          float o[4] = {v[0] + bias[b][0], v[1] + bias[b][1], v[2] + bias[b][2], v[3] + bias[b][3]};
          if constexpr (EPI == 3) {
            const u32x2 c = __builtin_amdgcn_raw_buffer_load_b64(obuf.r, off, 0, 0);
            o[0] += hx::bf2f((uint16_t)(c[0] & 0xffff));
            o[1] += hx::bf2f((uint16_t)(c[0] >> 16));
            o[2] += hx::bf2f((uint16_t)(c[1] & 0xffff));
            o[3] += hx::bf2f((uint16_t)(c[1] >> 16));
          }
          const uint2 pk = make_uint2(hx::f2bf(o[0]) | ((uint32_t)hx::f2bf(o[1]) << 16),
                                      hx::f2bf(o[2]) | ((uint32_t)hx::f2bf(o[3]) << 16));
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, pk), obuf.r, off, 0, SP);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  } else if constexpr (EPI == 0 || EPI == 3) {
#pragma unroll
    for (int a = 0; a < MB; ++a) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          float v[4];
          tr(a, b, gq, v);
          f32x4 o = {v[0] + bias[b][0], v[1] + bias[b][1], v[2] + bias[b][2], v[3] + bias[b][3]};
          if constexpr (EPI == 3)
            o += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(cbuf.r, coff(a, b, gq), 0, 0));
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), cbuf.r, coff(a, b, gq), 0, SP);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    // GELU epilogues; OB: C / P / aux in bf16 (--precision bf16: 8-B accesses of 4 columns)
    constexpr int OE = OB ? 2 : 4;
    const hx::Buf pbuf((const char*)g.P + ((int64_t)m0 * g.ldp + n0) * OE, (uint32_t)((int64_t)mrows * g.ldp * OE));
    const hx::Buf xbuf(EPI == 2 ? (const char*)g.aux + ((int64_t)m0 * g.ldaux + n0) * OE : (const char*)g.C,
                       (uint32_t)((int64_t)mrows * g.ldaux * OE));
    const hx::Buf obuf((const char*)g.C + ((int64_t)m0 * g.ldc + n0) * OE, (uint32_t)((int64_t)mrows * g.ldc * OE));
    auto poff = [&](int a, int b, int gq) { return (uint32_t)((mrow + 32 * a + 8 * gq) * g.ldp + ncol + 32 * b) * OE; };
    auto st4 = [&](const hx::Buf& bf, uint32_t off, f32x4 v) {
      if constexpr (OB == 1) {
        const uint2 pk = make_uint2(hx::f2bf(v[0]) | ((uint32_t)hx::f2bf(v[1]) << 16),
                                    hx::f2bf(v[2]) | ((uint32_t)hx::f2bf(v[3]) << 16));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, pk), bf.r, off, 0, SP);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), bf.r, off, 0, SP);
      }
    };
    float csum[NB][4], cmx[NB][4], rmx[MB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) csum[b][i] = cmx[b][i] = 0.f;
#pragma unroll
    for (int a = 0; a < MB; ++a)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) rmx[a][gq] = 0.f;
#pragma unroll
    for (int a = 0; a < MB; ++a) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        f32x4 u[4];
        if constexpr (EPI == 2) {
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            const uint32_t off = (uint32_t)((mrow + 32 * a + 8 * gq) * g.ldaux + ncol + 32 * b) * OE;
            if constexpr (OB == 1) {
              const u32x2 c = __builtin_amdgcn_raw_buffer_load_b64(xbuf.r, off, 0, 0);
              u[gq] = f32x4{hx::bf2f((uint16_t)(c[0] & 0xffff)), hx::bf2f((uint16_t)(c[0] >> 16)),
                            hx::bf2f((uint16_t)(c[1] & 0xffff)), hx::bf2f((uint16_t)(c[1] >> 16))};
            } else {
              u[gq] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xbuf.r, off, 0, 0));
            }
          }
        }
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          float v[4];
          tr(a, b, gq, v);
          const bool in = mrow + 32 * a + 8 * gq < mrows;
          f32x4 o;
          if constexpr (EPI == 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] += bias[b][i];
            f32x4 c;
            if (g.dmode) {
              // gelu(u) and gelu'(u) from ONE erf (hx::gelu_f / hx::gelu_grad_f bit for bit)
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const float e = erff(v[i] * (1.0f / 1.41421f));
                c[i] = 0.5f * (1.0f + e) + hx::gelu_pdf_f(v[i]);
                o[i] = v[i] * 0.5f * (1.0f + e);
              }
            } else {
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                c[i] = v[i];
                o[i] = hx::gelu_f(v[i]);
              }
            }
            st4(obuf, coff(a, b, gq) / 4 * OE, c);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              o[i] = g.dmode ? v[i] * u[gq][i] : v[i] * hx::gelu_grad_f(u[gq][i] + bias[b][i]);
              csum[b][i] += in ? o[i] : 0.f;
            }
          }
          if (in) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float m = fabsf(o[i]);
              rmx[a][gq] = fmaxf(rmx[a][gq], m);
              cmx[b][i] = fmaxf(cmx[b][i], m);
            }
          }
          st4(pbuf, poff(a, b, gq), o);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // column sums (EPI 2) and column maxima: over the 4 rows of a quad and the two 32-lane
    // halves; lanes (l32 & 3) == 0, h == 0 then hold this wave's 4-column values
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float m = cmx[b][i];
        m = fmaxf(m, qx1(m));
        m = fmaxf(m, qx2(m));
        cmx[b][i] = fmaxf(m, __shfl_xor(m, 32, 64));
        if constexpr (EPI == 2) {
          float t = csum[b][i];
          t += qx1(t);
          t += qx2(t);
          csum[b][i] = t + __shfl_xor(t, 32, 64);
        }
      }
    // row maxima: over the 8 lanes of a row's 4-column groups
#pragma unroll
    for (int a = 0; a < MB; ++a)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        float m = rmx[a][gq];
        m = fmaxf(m, __shfl_xor(m, 4, 64));
        m = fmaxf(m, __shfl_xor(m, 8, 64));
        rmx[a][gq] = fmaxf(m, __shfl_xor(m, 16, 64));
      }
    if constexpr (EPI == 2) {
      if (g.colpart && (l32 & 3) == 0 && h == 0) {
        float* row = g.colpart + (int64_t)(mt * NWM + wm) * g.N + n0 + wn * WN;
#pragma unroll
        for (int b = 0; b < NB; ++b)
          *reinterpret_cast<float4*>(row + 32 * b + l32) = make_float4(csum[b][0], csum[b][1], csum[b][2], csum[b][3]);
      }
    }
    // across the waves sharing rows (NWN) / columns (NWM), through the (free) ring
    float* rx = reinterpret_cast<float*>(lds);   // [NWN][BM]
    float* cx = rx + NWN * BM;                    // [NWM][BN]
    if (l32 < 4) {
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) rx[wn * BM + mrow + 32 * a + 8 * gq] = rmx[a][gq];
    }
    if ((l32 & 3) == 0 && h == 0) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) cx[wm * BN + ncol + 32 * b + i] = cmx[b][i];
    }
    __syncthreads();
    if (g.rowmax && tid < mrows) {
      float m = rx[tid];
#pragma unroll
      for (int j = 1; j < NWN; ++j) m = fmaxf(m, rx[j * BM + tid]);
      g.rowmax[(int64_t)(m0 + tid) * TN + nt] = m;
    }
    if (g.colmax && tid < BN) {
      float m = cx[tid];
#pragma unroll
      for (int j = 1; j < NWM; ++j) m = fmaxf(m, cx[j * BN + tid]);
      g.colmax[(int64_t)mt * g.N + n0 + tid] = m;
    }
  }
}

// ---------------------------------------------------------------- configurations
// cfg 0: 256 x 192, 8 waves of 32 x 192, one workgroup per CU, 4-stage ring
// cfg 1: 256 x 192, 8 waves (4 x 2) of 64 x 96, one workgroup per CU, 4-stage ring -- M >= 8192
// cfg 2: 128 x 96, 4 waves of 32 x 96, two workgroups per CU, 4-stage ring        -- M < 8192
// cfg 3: 64 x 64, 4 waves (2 x 2) of 32 x 32, 4-stage ring                          -- tiny M
// cfg 4: 128 x 192, 4 waves (2 x 2) of 64 x 96, two workgroups per CU, 3-stage ring
// cfg 5: 256 x 256, 8 waves (4 x 2) of 64 x 128, one workgroup per CU, 4-stage ring
// cfg 6: cfg 1 with the bf16 variant's DMA pieces issued as one burst (the fp16x3 step always
//        bursts them: interleaving measured 2-5 % slower, r5d); a 5-stage ring measured no gain (r5c)
constexpr int kCfgs = 7;
int cfg_bm(int c) { return c <= 1 || c >= 5 ? 256 : c == 2 || c == 4 ? 128 : 64; }
int cfg_bn(int c) { return c == 5 ? 256 : c <= 1 || c == 4 || c >= 6 ? 192 : c == 2 ? 96 : 64; }
int cfg_nwm(int c) { return c == 0 ? 8 : c == 1 || c >= 5 ? 4 : c == 2 ? 4 : 2; }

template <int BM, int BN, int WM, int WN, int EPI, int WGS, int NS, int AT = 0, int OB = 0, int DIL = 1, int DW = 0>
void launch_one(const F16Args& a, hipStream_t s) {
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  const int total = ((a.M + BM - 1) / BM) * (a.N / BN) * a.ks;
  const int per = (total + 7) / 8;
  const size_t smem = (size_t)NS * (BM + BN) * 64 + (2 * BM + BN + NT / 64) * 4 + 1024;   // + junk DMA KiB
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_f16_k<BM, BN, WM, WN, EPI, WGS, NS, AT, OB, DIL, DW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr = true;
  }
  gemm_f16_k<BM, BN, WM, WN, EPI, WGS, NS, AT, OB, DIL, DW><<<8 * per, NT, smem, s>>>(a);
}

// which waves of the large fp16x3 tile issue its LDS-DMA: 4 (default) waves 0 .. 3, one per SIMD --
// the headline step 35.54-35.66 vs 35.77-35.81 ms with every wave issuing, 9 alternated pairs on two
// boxes, 8 of them faster (profiles/r6u_gemm_dma_waves_ab.txt; the kernels alone measure equal);
// waves 4 .. 7 instead measured 35.94-36.02.  HX_GEMM_DMA_WAVES=0: every wave (read per call)
int dma_waves() {
  const char* e = getenv("HX_GEMM_DMA_WAVES");
  return e ? atoi(e) : 4;
}

template <int EPI, int AT = 0, int OB = 0>
void launch_cfg(int cfg, const F16Args& a, hipStream_t s) {
  if constexpr (AT != 1) {
    if (cfg == 1 && dma_waves() == 4) {
      launch_one<256, 192, 64, 96, EPI, 1, 4, AT, OB, 1, 4>(a, s);
      return;
    }
  }
  if (cfg == 0) launch_one<256, 192, 32, 192, EPI, 1, 4, AT, OB>(a, s);
  else if (cfg == 1) launch_one<256, 192, 64, 96, EPI, 1, 4, AT, OB>(a, s);
  else if (cfg == 6) launch_one<256, 192, 64, 96, EPI, 1, 4, AT, OB, 0>(a, s);
  else if (cfg == 2) launch_one<128, 96, 32, 96, EPI, 2, 4, AT, OB>(a, s);
  else if (cfg == 4) launch_one<128, 192, 64, 96, EPI, 2, 3, AT, OB>(a, s);
  else if (cfg == 5) launch_one<256, 256, 64, 128, EPI, 1, 4, AT, OB>(a, s);
  else launch_one<64, 64, 32, 32, EPI, 2, 4, AT, OB>(a, s);
}

// ---------------------------------------------------------------- weight gradient (tokens = reduction)
// LDS image of a [16 tokens][W columns] fp16 tile: 8-row x 32-column subtiles of 512 B, XOR-swizzled
// 16-B chunks, odd subtiles with the rows of each pair swapped (conflict-free 16-B stores and
// transposed ds_read_b64_tr_b16 reads)
template <int W>
__device__ __forceinline__ int toff(int row, int ch) {
  return (row >> 3) * (16 * W) + 512 * (ch >> 2) + 64 * ((row & 7) ^ ((ch >> 2) & 1)) +
         16 * ((ch & 3) ^ ((row >> 2) & 3));
}
template <int W>
__device__ __forceinline__ void tr_base(int lane, int (&lo)[2], int (&hi)[2]) {
  const int gq = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = 8 * (gq >> 1) + q, ch = 2 * (gq & 1) + (p >> 1);
  lo[0] = toff<W>(row, ch) + 8 * (p & 1);
  hi[0] = toff<W>(row + 4, ch) + 8 * (p & 1);
  lo[1] = toff<W>(row, ch + 4) - 512 + 8 * (p & 1);
  hi[1] = toff<W>(row + 4, ch + 4) - 512 + 8 * (p & 1);
}
// the k-major fragment (8 consecutive tokens of column c0 + lane & 31) of a [16][W] tile
template <int W>
__device__ __forceinline__ f16x8 tfrag(const char* tile, const int (&lo)[2], const int (&hi)[2], int c0, int odd) {
  const int d = (c0 >> 5) * 512;
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(tile + lo[odd] + d));
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(tile + hi[odd] + d));
  const v4i16 v[2] = {a, b};
  return *reinterpret_cast<const f16x8*>(v);
}

// column scale tables of a weight-gradient operand (ColScale, hx_launch.h)
__device__ __forceinline__ void col_scales(const HxColScale& c, int c0, int cols, float* s, float* is, float* red) {
  if (c.g == nullptr && c.cs == 0) {
    const int E = f16_scale_exp(block_amax(c.p, c.np, red));
    for (int t = threadIdx.x; t < cols; t += blockDim.x) {
      s[t] = ldexpf(1.f, E);
      is[t] = ldexpf(1.f, -E);
    }
    return;
  }
  for (int t = threadIdx.x; t < cols; t += blockDim.x) {
    float m = 0.f;
    if (c.g) {
      m = (fabsf(c.g[c0 + t]) * c.z + fabsf(c.b[c0 + t])) * c.mul;
    } else {
      for (int j = 0; j < c.np; ++j) m = fmaxf(m, c.p[(int64_t)j * c.cs + c0 + t]);
    }
    const int E = f16_scale_exp(m);
    s[t] = ldexpf(1.f, E);
    is[t] = ldexpf(1.f, -E);
  }
}

template <int BM, int BN, int WM, int WN, int BKT = 32>
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64) void wgrad_f16_k(const float* __restrict__ A, int lda,
                                                                         const HxColScale ca,
                                                                         const float* __restrict__ B, int ldb,
                                                                         const HxColScale cb,
                                                                         float* __restrict__ out, int M, int N, int T,
                                                                         int kchunk, int nsplit, int mvalid) {
  constexpr int NWM = BM / WM, NW = NWM * (BN / WN), NT = NW * 64;
  constexpr int MB = WM / 32, NB = WN / 32;
  // BKT tokens per stage: BKT / 16 MFMA substeps per barrier.  32 (r5): half the barriers and
  // post-barrier fragment reads per MFMA of 16, measured the same (r5ag, repeated A/B: QKV 185 /
  // 185, FFN 234 / 233 us) -- neither bounds this kernel; the vector-memory path and the clock do
  constexpr int NSUB = BKT / 16;
  constexpr int CA = BKT * BM / 8 / NT, CB = BKT * BN / 8 / NT;   // 8-column chunks per thread
  static_assert(CA >= 1 && CB >= 1 && BKT * BM / 8 % NT == 0 && BKT * BN / 8 % NT == 0, "tile / thread mismatch");
  static_assert(WM % 64 == 0 && WN % 64 == 0, "subtile parity of fragment a is a & 1");
  constexpr int A_T = BKT * BM * 2, B_T = BKT * BN * 2;   // one fp16 piece tile [32 tokens][cols]
  constexpr int A_S = 16 * BM * 2, B_S = 16 * BN * 2;    // a 16-token substep's offset (toff rows 16..31)
  constexpr int STAGE = 2 * (A_T + B_T);
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // per-column scales of the two operands (dY's columns = dW's rows, X's columns = dW's columns)
  float* tsa = reinterpret_cast<float*>(lds + 2 * STAGE);
  float* tia = tsa + BM;
  float* tsb = tia + BM;
  float* tib = tsb + BN;
  float* red = tib + BN;

  const int total = (M / BM) * (N / BN) * nsplit;
  const int per = (total + 7) / 8;
  const int work = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (work >= total) return;   // uniform per workgroup
  const int TM = M / BM, TN = N / BN;
  const bool mord = M < N;   // output-row tiles fastest when there are fewer of them
  const int nt = mord ? (work / TM) % TN : work % TN;
  const int mt = mord ? work % TM : (work / TN) % TM;
  const int sp = work / (TN * TM);
  const int m0 = mt * BM, n0 = nt * BN;
  const int t0 = sp * kchunk, t1 = min(T, t0 + kchunk);
  const int nit = (t1 - t0 + BKT - 1) / BKT;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w % NWM, wn = w / NWM;

  col_scales(ca, m0, BM, tsa, tia, red);
  col_scales(cb, n0, BN, tsb, tib, red);
  __syncthreads();

  const hx::Buf abuf(A + (int64_t)t0 * lda, (uint32_t)((int64_t)(t1 - t0) * lda * 4));
  const hx::Buf bbuf(B + (int64_t)t0 * ldb, (uint32_t)((int64_t)(t1 - t0) * ldb * 4));
  uint32_t va[CA], vb[CB];
  int sa_[CA], sb_[CB];
  const float* cs[CA + CB];   // the chunks' 8 column scales (LDS tables; read at split time)
#pragma unroll
  for (int i = 0; i < CA; ++i) {
    const int e = tid + i * NT, row = e / (BM / 8), c = e % (BM / 8);
    va[i] = (uint32_t)(row * lda + m0 + 8 * c) * 4;
    sa_[i] = toff<BM>(row, c);
    cs[i] = tsa + 8 * c;
  }
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    const int e = tid + i * NT, row = e / (BN / 8), c = e % (BN / 8);
    vb[i] = (uint32_t)(row * ldb + n0 + 8 * c) * 4;
    sb_[i] = toff<BN>(row, c);
    cs[CA + i] = tsb + 8 * c;
  }
  int alo[2], ahi[2], blo[2], bhi[2];
  tr_base<BM>(lane, alo, ahi);
  tr_base<BN>(lane, blo, bhi);

  // ONE register stage: the fp32 tiles of stage it + 2 are loaded right after stage it + 1's
  // split (in step it's second substep), so a load has a full step of MFMA work to land; past the
  // slab's end the loads are aimed past the buffer (zeros, no memory traffic)
  struct Regs {
    f32x4 v[CA + CB][2];   // chunks: CA of dY, then CB of X
  };
  auto load = [&](int it, Regs& r) {
    const bool in = it < nit;
    const uint32_t soa = in ? (uint32_t)it * BKT * lda * 4 : 0x80000000u;
    const uint32_t sob = in ? (uint32_t)it * BKT * ldb * 4 : 0x80000000u;
#pragma unroll
    for (int i = 0; i < CA; ++i)
#pragma unroll
      for (int k = 0; k < 2; ++k)
        r.v[i][k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(abuf.r, va[i] + 16 * k, soa, 0));
#pragma unroll
    for (int i = 0; i < CB; ++i)
#pragma unroll
      for (int k = 0; k < 2; ++k)
        r.v[CA + i][k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(bbuf.r, vb[i] + 16 * k, sob, 0));
  };
  // the split of one 8-column chunk (c < CA: of dY, else of X) as four v_fma_mix pairs, and its
  // two LDS piece writes
  constexpr int NCH = CA + CB;
  auto scales = [&](int c, f32x4 (&sc)[2]) {
    sc[0] = *reinterpret_cast<const f32x4*>(cs[c]);
    sc[1] = *reinterpret_cast<const f32x4*>(cs[c] + 4);
  };
  auto split_pair = [&](const Regs& r, int c, int p, const f32x4 (&sc)[2], uint32_t (&h0)[4], uint32_t (&h1)[4]) {
    const f32x4& v = r.v[c][p >> 1];
    const int e = 2 * (p & 1);
    split_pair_mix2(v[e], v[e + 1], sc[p >> 1][e], sc[p >> 1][e + 1], h0[p], h1[p]);
  };
  auto write_chunk = [&](int buf, int c, const uint32_t (&h0)[4], const uint32_t (&h1)[4]) {
    char* st = lds + buf * STAGE;
    const u32x4 v0 = {h0[0], h0[1], h0[2], h0[3]}, v1 = {h1[0], h1[1], h1[2], h1[3]};
    if (c < CA) {
      *reinterpret_cast<u32x4*>(st + sa_[c]) = v0;
      *reinterpret_cast<u32x4*>(st + A_T + sa_[c]) = v1;
    } else {
      *reinterpret_cast<u32x4*>(st + 2 * A_T + sb_[c - CA]) = v0;
      *reinterpret_cast<u32x4*>(st + 2 * A_T + B_T + sb_[c - CA]) = v1;
    }
  };
  auto store_all = [&](int buf, const Regs& r) {   // (the prologue's stage 0)
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      f32x4 sc[2];
      scales(c, sc);
      uint32_t h0[4], h1[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) split_pair(r, c, p, sc, h0, h1);
      write_chunk(buf, c, h0, h1);
    }
  };

  f32x16 acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = f32x16{0};

  struct Fr {
    f16x8 a0[MB], b0[NB], b1[NB];   // a0[a] holds piece 1 of A rows a during pass 2
  };
  // fragments of substep s of a stage; the second A pieces (a1, pass 2 only) are read one by one
  // after the last pass-1 MFMA on the first piece of the same rows, into its registers
  auto read = [&](int buf, Fr& F, int s) {
    const char* st = lds + buf * STAGE;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      F.b0[b] = tfrag<BN>(st + 2 * A_T + s * B_S, blo, bhi, wn * WN + 32 * b, b & 1);
      F.b1[b] = tfrag<BN>(st + 2 * A_T + B_T + s * B_S, blo, bhi, wn * WN + 32 * b, b & 1);
    }
#pragma unroll
    for (int a = 0; a < MB; ++a) F.a0[a] = tfrag<BM>(st + s * A_S, alo, ahi, wm * WM + 32 * a, a & 1);
  };
  auto read_a1 = [&](int buf, Fr& F, int a, int s) {
    F.a0[a] = tfrag<BM>(lds + buf * STAGE + A_T + s * A_S, alo, ahi, wm * WM + 32 * a, a & 1);
  };
  constexpr int NMF = 3 * MB * NB;   // MFMAs per substep
  constexpr int G0 = NSUB * NMF - 4 * NCH;   // the step's MFMA after which the first split pair goes
  static_assert(G0 >= 0, "one split pair per MFMA");
  auto mma = [&](const Fr& F, int i) {   // MFMA i: pass q = i / (MB NB)
    const int q = i / (MB * NB), a = (i % (MB * NB)) / NB, b = i % NB;
    acc[a][b] = mfma16(F.a0[a], q == 1 ? F.b1[b] : F.b0[b], acc[a][b]);
  };

  // step it (32 tokens, two 16-token substeps): each substep's fragments, then its MFMAs; the
  // split of stage it + 1 (loaded a step ago) rides pair by pair behind the step's last MFMAs and
  // goes into the other buffer (last read before the previous barrier), then stage it + 2's loads
  // are issued into the freed registers (a full step to land); one barrier per step
  Regs rr;
  load(0, rr);
  store_all(0, rr);
  load(1, rr);
  __syncthreads();
  for (int it = 0; it < nit; ++it) {
    const int cur = it & 1;
    f32x4 sc[2];
    uint32_t h0[4], h1[4];
#pragma unroll
    for (int s = 0; s < NSUB; ++s) {
      Fr F;
      read(cur, F, s);
#pragma unroll
      for (int i = 0; i < NMF; ++i) {
        mma(F, i);
        if (i / (MB * NB) == 1 && i % NB == NB - 1) read_a1(cur, F, (i % (MB * NB)) / NB, s);
        const int g = s * NMF + i;
        if (g >= G0) {
          const int k = g - G0;
          if (k % 4 == 0) scales(k / 4, sc);
          split_pair(rr, k / 4, k % 4, sc, h0, h1);
          if (k % 4 == 3) write_chunk(cur ^ 1, k / 4, h0, h1);
        }
        if (g == NSUB * NMF - 1) load(it + 2, rr);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __syncthreads();
  }

  float* o = out + (nsplit > 1 ? (int64_t)sp * M * N : 0);
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int n = n0 + wn * WN + 32 * b + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WM + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < mvalid) o[(int64_t)m * N + n] = acc[a][b][r] * tia[m - m0] * tib[n - n0];   // rows past mvalid: padding
      }
    }
}

__global__ __launch_bounds__(256) void slab_sum_k(const float4* __restrict__ ws, float4* __restrict__ out, int64_t n4,
                                                  int64_t slab4, int nsplit) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 s = ws[i];
    for (int k = 1; k < nsplit; ++k) {
      const float4 v = ws[(int64_t)k * slab4 + i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    out[i] = s;
  }
}

template <int BM, int BN, int WM, int WN, int BKT = 32>
void wgrad_launch(const float* A, int lda, const HxColScale& ca, const float* B, int ldb, const HxColScale& cb,
                  float* out, float* ws, int M, int N, int T, int nsplit, int mvalid, hipStream_t s) {
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  const int kchunk = ((T + nsplit - 1) / nsplit + BKT - 1) / BKT * BKT;
  nsplit = (T + kchunk - 1) / kchunk;
  const int total = (M / BM) * (N / BN) * nsplit;
  const int per = (total + 7) / 8;
  const size_t smem = (size_t)2 * 2 * BKT * (BM + BN) * 2 + (2 * BM + 2 * BN + NT / 64) * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_f16_k<BM, BN, WM, WN, BKT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr = true;
  }
  wgrad_f16_k<BM, BN, WM, WN, BKT><<<8 * per, NT, smem, s>>>(A, lda, ca, B, ldb, cb, nsplit > 1 ? ws : out, M, N, T,
                                                        kchunk, nsplit, nsplit > 1 ? M : mvalid);
  if (nsplit > 1) {
    const int64_t n4 = (int64_t)mvalid * N / 4, slab4 = (int64_t)M * N / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
    slab_sum_k<<<blocks, 256, 0, s>>>(reinterpret_cast<const float4*>(ws), reinterpret_cast<float4*>(out), n4, slab4,
                                      nsplit);
  }
}

// ---------------------------------------------------------------- weight gradient, add-tid staging
// The same product as wgrad_f16_k on the 256 x 256 tile, with the piece tiles written to LDS by
// ds_write_addtid_b32 (lane l -> dword l of a 256-B block: 128 B/clk/CU) instead of ds_write_b128
// (~79 B/clk/CU, MI355X_MICROARCH.md §LDS): the piece stores were the largest non-MFMA cost of the
// k loop (profiles/r6g_gemm_wgrad_split_probe.md: -14..-19 % without them).
// Per 16-token stage, each of the 8 waves loads 8 (token row, 128-column block) units of ONE
// operand: lane l takes the two columns 2 ((l + 16 r) & 63) of the block (a b64 load; 512 B per
// wave-load, permuted inside the row), splits the pair at its column scales and stores one dword
// per piece at slot l.  Image per (stage, piece, operand): [16 rows][2 blocks][64 slots x 4 B],
// slot l of row r holding column pair (l + 16 r) & 63: the rotation by 16 pairs per row puts the
// four rows of a transposed 16-lane read (ds_read_b64_tr_b16: lane 4q + p reads row q, columns
// 4p .. 4p + 3) on four disjoint 16-bank ranges -- conflict-free reads, and every store is one
// contiguous 256-B block.  Layout: stage 32 KiB, piece 16 KiB, operand 8 KiB, row 512 B, block
// 256 B (64 KiB double-buffered: every store address is M0 (< 16 KiB) + a 16-bit immediate).
// Loads run two stages ahead in a two-set register ring.
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}
// one ds_write_addtid_b32 of dword h to LDS byte address U + C (U wave-uniform, at most UMAX; C a
// compile-time constant): M0[15:0] + a 16-bit immediate, split so that both fit
template <int C, int UMAX>
__device__ __forceinline__ void st_tid(uint32_t u, uint32_t h) {
  constexpr int IMM = C > 65535 ? C - 65535 : 0;   // into M0; the immediate is C - IMM
  static_assert(C - IMM <= 65535 && IMM + UMAX <= 65535, "add-tid address range");
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tds_write_addtid_b32 %1 offset:%3\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(h), "s"(u + (uint32_t)IMM), "i"(C - IMM)
               : "memory");
}

template <int BKT>
__global__ __launch_bounds__(512) void wgrad_f16_tid_k(const float* __restrict__ A, int lda, const HxColScale ca,
                                                        const float* __restrict__ B, int ldb, const HxColScale cb,
                                                        float* __restrict__ out, int M, int N, int T, int kchunk,
                                                        int nsplit, int mvalid) {
  static_assert(BKT == 16 || BKT == 32, "16- or 32-token stages");
  constexpr int BM = 256, BN = 256, WM = 128, WN = 64, NWM = 2, MB = 4, NB = 2;
  constexpr int NU = BKT / 2, NSUB = BKT / 16;      // staging units per wave, 16-token substeps
  constexpr int NSET = BKT == 16 ? 2 : 1;           // register sets: loads run NSET stages ahead
  constexpr int OPB = BKT * 512, PCE = 2 * OPB, STG = 2 * PCE;   // image strides (bytes)
  constexpr int UMAX = OPB + 512 + 256;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* tsa = reinterpret_cast<float*>(lds + 2 * STG);
  float* tia = tsa + BM;
  float* tsb = tia + BM;
  float* tib = tsb + BN;
  float* red = tib + BN;

  const int total = (M / BM) * (N / BN) * nsplit;
  const int per = (total + 7) / 8;
  const int work = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (work >= total) return;   // uniform per workgroup
  const int TM = M / BM, TN = N / BN;
  const bool mord = M < N;
  const int nt = mord ? (work / TM) % TN : work % TN;
  const int mt = mord ? work % TM : (work / TN) % TM;
  const int sp = work / (TN * TM);
  const int m0 = mt * BM, n0 = nt * BN;
  const int t0 = sp * kchunk, t1 = min(T, t0 + kchunk);
  const int nit = (t1 - t0 + BKT - 1) / BKT;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w % NWM, wn = w / NWM;
  const int wv = __builtin_amdgcn_readfirstlane(w);

  col_scales(ca, m0, BM, tsa, tia, red);
  col_scales(cb, n0, BN, tsb, tib, red);
  __syncthreads();

  // ---- this wave's staging units: operand op, column block blk, token rows par + 2 i (i < NU)
  const int op = wv & 1, blk = (wv >> 1) & 1, par = wv >> 2;
  const float* src = op ? B : A;
  const int ld = op ? ldb : lda;
  const hx::Buf buf(src + (int64_t)t0 * ld, (uint32_t)((int64_t)(t1 - t0) * ld * 4));
  const float* tsc = op ? tsb : tsa;
  const int pe = (lane + 16 * par) & 63, po = (lane + 16 * (par + 2)) & 63;   // column pairs (even / odd i)
  const int ce = 128 * blk + 2 * pe, co = 128 * blk + 2 * po;
  const uint32_t ve = (uint32_t)((op ? n0 : m0) + ce) * 4, vo = (uint32_t)((op ? n0 : m0) + co) * 4;
  const float se0 = tsc[ce], se1 = tsc[ce + 1], so0 = tsc[co], so1 = tsc[co + 1];
  const uint32_t lds0 = (uint32_t)(size_t)(lds_void*)lds;
  const uint32_t mu = __builtin_amdgcn_readfirstlane(lds0 + op * OPB + par * 512 + blk * 256);
  const uint32_t row_b = (uint32_t)ld * 4u;

  typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
  struct Regs {
    u32x2v v[NU];
  };
  auto load_one = [&](int it, Regs& r, int i) {
    const bool in = it < nit;
    const uint32_t so = in ? (uint32_t)(it * BKT + par + 2 * i) * row_b : 0x80000000u;
    r.v[i] = __builtin_amdgcn_raw_buffer_load_b64(buf.r, (i & 1) ? vo : ve, so, 0);
  };
  auto load = [&](int it, Regs& r) {
#pragma unroll
    for (int i = 0; i < NU; ++i) load_one(it, r, i);
  };
  // unit i of a register set -> its two piece dwords into stage buffer S (compile-time)
  auto store_one = [&](const Regs& r, auto S, auto I) {
    constexpr int s = decltype(S)::value, i = decltype(I)::value;
    uint32_t h0, h1;
    const float x0 = __uint_as_float(r.v[i].x), x1 = __uint_as_float(r.v[i].y);
    if constexpr ((i & 1) != 0) split_pair_mix2(x0, x1, so0, so1, h0, h1);
    else split_pair_mix2(x0, x1, se0, se1, h0, h1);
    st_tid<s * STG + i * 1024, UMAX>(mu, h0);
    st_tid<s * STG + PCE + i * 1024, UMAX>(mu, h1);
  };

  // transposed fragment offsets (bytes within an operand image): lane (gq, q, p) reads row
  // 8 (gq >> 1) + q (+ 4: the hi read), column pairs (c0 & 127) / 2 + 8 (gq & 1) + 2 p
  const int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int lrow = 8 * (gq >> 1) + q;
  int offa[MB], offb[NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
    offa[a] = lrow * 512 + wm * 256 + 4 * ((16 * a + 8 * (gq & 1) + 2 * p - 16 * q) & 63);
#pragma unroll
  for (int b = 0; b < NB; ++b)
    offb[b] = lrow * 512 + (wn >> 1) * 256 + 4 * ((32 * (wn & 1) + 16 * b + 8 * (gq & 1) + 2 * p - 16 * q) & 63);
  auto frag = [&](int off) {
    const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(lds + off));
    const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(lds + off + 2048));
    const v4i16 v[2] = {a, b};
    return *reinterpret_cast<const f16x8*>(v);
  };

  f32x16 acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = f32x16{0};

  struct Fr {
    f16x8 a0[MB], b0[NB], b1[NB];   // a0[a] holds piece 1 of A rows a during pass 2
  };
  constexpr int NMF = 3 * MB * NB;
  auto mma = [&](const Fr& F, int i) {
    const int qq = i / (MB * NB), a = (i % (MB * NB)) / NB, b = i % NB;
    acc[a][b] = mfma16(F.a0[a], qq == 1 ? F.b1[b] : F.b0[b], acc[a][b]);
  };
  // one BKT-token step on stage buffer S: per 16-token substep, fragments and 24 MFMAs; under them
  // the split + stores of the next stage (register set (S ^ 1) % NSET) into buffer S ^ 1, eight units
  // per substep, each unit's register refilled NSET stages ahead right after its split; one barrier
  Regs R[NSET];
  auto step = [&](int it, auto S) {
    constexpr int s = decltype(S)::value, rs = (s ^ 1) % NSET;
    const int base = s * STG;
    static_for<0, NSUB>([&](auto SS) {
      constexpr int ss = decltype(SS)::value;
      const int sb = base + ss * 8192;
      Fr F;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        F.b0[b] = frag(sb + OPB + offb[b]);
        F.b1[b] = frag(sb + PCE + OPB + offb[b]);
      }
#pragma unroll
      for (int a = 0; a < MB; ++a) F.a0[a] = frag(sb + offa[a]);
      static_for<0, NMF>([&](auto I) {
        constexpr int i = decltype(I)::value;
        mma(F, i);
        if constexpr (i / (MB * NB) == 1 && i % NB == NB - 1) {
          constexpr int a = (i % (MB * NB)) / NB;
          F.a0[a] = frag(sb + PCE + offa[a]);
        }
        if constexpr (i % 3 == 2) {   // units 8 ss + 0 .. 7 after MFMAs 2, 5, .., 23
          constexpr int u = 8 * ss + i / 3;
          store_one(R[rs], std::integral_constant<int, s ^ 1>{}, std::integral_constant<int, u>{});
          load_one(it + 1 + NSET, R[rs], u);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    });
    // the add-tid stores come from asm: the compiler does not count them, so retire them here,
    // before the barrier that publishes the stage
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
  };

  load(0, R[0]);
  if constexpr (NSET == 2) load(1, R[1]);
  static_for<0, NU>([&](auto I) {
    store_one(R[0], std::integral_constant<int, 0>{}, I);
    load_one(NSET, R[0], decltype(I)::value);
  });
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  for (int it = 0; it < nit; it += 2) {
    step(it, std::integral_constant<int, 0>{});
    if (it + 1 < nit) step(it + 1, std::integral_constant<int, 1>{});
  }

  float* o = out + (nsplit > 1 ? (int64_t)sp * M * N : 0);
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int n = n0 + wn * WN + 32 * b + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WM + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < mvalid) o[(int64_t)m * N + n] = acc[a][b][r] * tia[m - m0] * tib[n - n0];
      }
    }
}

template <int BKT>
void wgrad_tid_launch(const float* A, int lda, const HxColScale& ca, const float* B, int ldb, const HxColScale& cb,
                      float* out, float* ws, int M, int N, int T, int nsplit, int mvalid, hipStream_t s) {
  // the token splits of wgrad_launch<.., 32> (32-token granularity): the same slabs, the same sums
  const int kchunk = ((T + nsplit - 1) / nsplit + 31) / 32 * 32;
  nsplit = (T + kchunk - 1) / kchunk;
  const int total = (M / 256) * (N / 256) * nsplit;
  const int per = (total + 7) / 8;
  const size_t smem = (size_t)2 * 4 * BKT * 512 + (4 * 256 + 8) * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_f16_tid_k<BKT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr = true;
  }
  wgrad_f16_tid_k<BKT><<<8 * per, 512, smem, s>>>(A, lda, ca, B, ldb, cb, nsplit > 1 ? ws : out, M, N, T, kchunk,
                                                  nsplit, nsplit > 1 ? M : mvalid);
  if (nsplit > 1) {
    const int64_t n4 = (int64_t)mvalid * N / 4, slab4 = (int64_t)M * N / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
    slab_sum_k<<<blocks, 256, 0, s>>>(reinterpret_cast<const float4*>(ws), reinterpret_cast<float4*>(out), n4, slab4,
                                      nsplit);
  }
}

// ---------------------------------------------------------------- max |x| per row, weight pieces
// max |x| of every row of a [rows][cols] fp32 matrix (row stride ld, cols % 4 == 0): one wave per
// row (the per-row operand scale of the fp16x3 GEMMs, when no producer wrote it)
__global__ __launch_bounds__(256) void amax_rows_k(const float* __restrict__ x, int64_t rows, int cols, int64_t ld,
                                                   float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float4* p = reinterpret_cast<const float4*>(x + r * ld);
  float m = 0.f;
  for (int c = lane; c < cols / 4; c += 64) {
    const float4 v = p[c];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0) out[r] = m;
}

// row and column maxima of every weight of a batch, one 64 x 64 tile per workgroup: atomic max
// (non-negative floats order as their bit patterns) into rmax[n] / cmax[k], zeroed beforehand
__global__ __launch_bounds__(256) void amax_weights_k(HxWeightBatch d, float* __restrict__ rc) {
  __shared__ float cm[4][64];
  const int blk = blockIdx.x;
  int i = 0;
  while (i + 1 < d.n && blk >= d.start[i + 1]) ++i;   // uniform per workgroup
  const int N = d.N[i], K = d.K[i];
  const int tk = K / 64, loc = blk - d.start[i];
  const int k0 = (loc % tk) * 64, n0 = (loc / tk) * 64;
  const float* W = d.W[i];
  const int nv = d.nv[i] ? d.nv[i] : N;
  float* rmax = rc + d.roff[i];
  float* cmax = rmax + N;
  const int t = threadIdx.x, c4 = (t & 15) * 4;
  float col[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r4 = 0; r4 < 4; ++r4) {
    const int r = (t >> 4) + 16 * r4;
    const float4 v = n0 + r < nv ? *reinterpret_cast<const float4*>(W + (int64_t)(n0 + r) * K + k0 + c4)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
    const float a[4] = {fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w)};
    float m = fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3]));
#pragma unroll
    for (int j = 0; j < 4; ++j) col[j] = fmaxf(col[j], a[j]);
    // the 16 lanes of a row (t & 15) are consecutive lanes of one wave
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((t & 15) == 0) atomicMax(reinterpret_cast<unsigned*>(rmax + n0 + r), __float_as_uint(m));
  }
  // columns: over the 4 row groups of a wave (lanes t, t + 16, t + 32, t + 48), then the 4 waves
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    col[j] = fmaxf(col[j], __shfl_xor(col[j], 16, 64));
    col[j] = fmaxf(col[j], __shfl_xor(col[j], 32, 64));
  }
  if ((t & 63) < 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) cm[t >> 6][c4 + j] = col[j];
  }
  __syncthreads();
  if (t < 64) {
    const float m = fmaxf(fmaxf(cm[0][t], cm[1][t]), fmaxf(cm[2][t], cm[3][t]));
    atomicMax(reinterpret_cast<unsigned*>(cmax + k0 + t), __float_as_uint(m));
  }
}

// element offset of (row, piece p, column c) in the P2 layout [rows][C / 16][2][16]
__device__ __forceinline__ int64_t p2_off(int64_t row, int p, int c, int C) {
  return row * 2 * C + (c >> 4) * 32 + p * 16 + (c & 15);
}

// both P2 piece layouts of every weight of a batch, one 64 x 64 tile per workgroup:
//   wf[n] = pieces of W[n][:] scaled by row n's 2^E (forward B operand, rows = output columns),
//   wt[k] = pieces of W[:][k] scaled by column k's 2^E (data gradient B operand)
__global__ __launch_bounds__(256) void split_weight_f16_k(HxWeightBatch d, const float* __restrict__ rc) {
  __shared__ uint16_t tile[2][64][66];
  const int blk = blockIdx.x;
  int i = 0;
  while (i + 1 < d.n && blk >= d.start[i + 1]) ++i;   // uniform per workgroup
  const int N = d.N[i], K = d.K[i];
  const int tk = K / 64, loc = blk - d.start[i];
  const int k0 = (loc % tk) * 64, n0 = (loc / tk) * 64;
  const float* W = d.W[i];
  const int nv = d.nv[i] ? d.nv[i] : N;
  const float* rmax = rc + d.roff[i];
  const float* cmax = rmax + N;
  const int t = threadIdx.x, c4 = (t & 15) * 4;
  float cs[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) cs[j] = ldexpf(1.f, f16_scale_exp(cmax[k0 + c4 + j]));
#pragma unroll
  for (int r4 = 0; r4 < 4; ++r4) {
    const int r = (t >> 4) + 16 * r4;
    const float rs = ldexpf(1.f, f16_scale_exp(rmax[n0 + r]));
    const float4 v = n0 + r < nv ? *reinterpret_cast<const float4*>(W + (int64_t)(n0 + r) * K + k0 + c4)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
    const float x[4] = {v.x, v.y, v.z, v.w};
    uint16_t q0[4], q1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float e = x[j] * rs, f = x[j] * cs[j];
      const _Float16 h0 = (_Float16)e, h1 = (_Float16)(e - (float)h0);
      const _Float16 g0 = (_Float16)f, g1 = (_Float16)(f - (float)g0);
      q0[j] = __builtin_bit_cast(uint16_t, h0);
      q1[j] = __builtin_bit_cast(uint16_t, h1);
      tile[0][r][c4 + j] = __builtin_bit_cast(uint16_t, g0);
      tile[1][r][c4 + j] = __builtin_bit_cast(uint16_t, g1);
    }
    *reinterpret_cast<uint2*>(d.wf[i] + p2_off(n0 + r, 0, k0 + c4, K)) =
        make_uint2(q0[0] | ((uint32_t)q0[1] << 16), q0[2] | ((uint32_t)q0[3] << 16));
    *reinterpret_cast<uint2*>(d.wf[i] + p2_off(n0 + r, 1, k0 + c4, K)) =
        make_uint2(q1[0] | ((uint32_t)q1[1] << 16), q1[2] | ((uint32_t)q1[3] << 16));
  }
  __syncthreads();
#pragma unroll
  for (int r4 = 0; r4 < 4; ++r4) {
    const int kk = (t >> 4) + 16 * r4;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      uint16_t q[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) q[j] = tile[p][c4 + j][kk];
      *reinterpret_cast<uint2*>(d.wt[i] + p2_off(k0 + kk, p, n0 + c4, N)) =
          make_uint2(q[0] | ((uint32_t)q[1] << 16), q[2] | ((uint32_t)q[3] << 16));
    }
  }
}

// fp32 rows -> their P2 pieces at each row's own scale (the max of its partials): the A operand of
// an AT 2 product when no fused producer wrote it (tests, and producers without a row-max pass)
__global__ __launch_bounds__(256) void split_rows_f16_k(const float* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ amax, int np, int64_t rows, int K,
                                                        uint16_t* __restrict__ out) {
  const int k4 = K / 4;
  const int64_t n = rows * k4;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / k4;
    const int c = (int)(i - r * k4) * 4;
    float m = 0.f;
    for (int j = 0; j < np; ++j) m = fmaxf(m, amax[r * np + j]);
    const float4 v = *reinterpret_cast<const float4*>(x + r * ldx + c);
    store_p2x4(out + r * 2 * K, c, v, ldexpf(1.f, f16_scale_exp(m)));
  }
}

// --precision bf16: W [N][K] fp32 -> W^T [K][N] bf16 (RNE, as the bf16 shadow), every weight of a
// batch in one launch, 64 x 64 tiles transposed through LDS
__global__ __launch_bounds__(256) void weight_bf16_t_k(HxWeightBatch d) {
  __shared__ uint16_t tile[64][66];
  const int blk = blockIdx.x;
  int i = 0;
  while (i + 1 < d.n && blk >= d.start[i + 1]) ++i;   // uniform per workgroup
  const int N = d.N[i], K = d.K[i];
  const int tk = K / 64, loc = blk - d.start[i];
  const int k0 = (loc % tk) * 64, n0 = (loc / tk) * 64;
  const float* W = d.W[i];
  const int t = threadIdx.x, c4 = (t & 15) * 4;
#pragma unroll
  for (int r4 = 0; r4 < 4; ++r4) {
    const int r = (t >> 4) + 16 * r4;
    const float4 v = *reinterpret_cast<const float4*>(W + (int64_t)(n0 + r) * K + k0 + c4);
    tile[r][c4] = hx::f2bf(v.x);
    tile[r][c4 + 1] = hx::f2bf(v.y);
    tile[r][c4 + 2] = hx::f2bf(v.z);
    tile[r][c4 + 3] = hx::f2bf(v.w);
  }
  __syncthreads();
#pragma unroll
  for (int r4 = 0; r4 < 4; ++r4) {
    const int kk = (t >> 4) + 16 * r4;
    uint16_t q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j] = tile[c4 + j][kk];
    *reinterpret_cast<uint2*>(d.wt[i] + (int64_t)(k0 + kk) * N + n0 + c4) =
        make_uint2(q[0] | ((uint32_t)q[1] << 16), q[2] | ((uint32_t)q[3] << 16));
  }
}

}  // namespace

void hx_weight_bf16_t(const HxWeightBatch& d, hipStream_t s) {
  if (d.n < 1) return;
  weight_bf16_t_k<<<d.start[d.n], 256, 0, s>>>(d);
}

// ---------------------------------------------------------------- host API (hx_launch.h)
void hx_split_rows_f16(const float* x, int64_t ldx, const float* amax, int np, int64_t rows, int K, uint16_t* out,
                       hipStream_t s) {
  const int64_t n = rows * (K / 4);
  if (n < 1) return;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 8192);
  split_rows_f16_k<<<blocks, 256, 0, s>>>(x, ldx, amax, np, rows, K, out);
}
void hx_fold_cols(const float* partial, int rows, int N, float* out, int accumulate, hipStream_t s) {
  hx::fold_rows(partial, rows, N, N, N, out, nullptr, nullptr, accumulate, s);
}

int hx_gemm_f16_plan(int M, int N, int K) {
  if (const char* e = getenv("HX_GEMM_F16_CFG")) {
    const int c = atoi(e);
    if (c >= 0 && c < kCfgs && N % cfg_bn(c) == 0) return c;
  }
  // deep reductions (the MLM decoder's data gradient, K = 30720) on the large tile whatever M: split-K
  // slabs fill the CUs, and the big tile halves the operand re-reads of the 128 x 96 one
  if ((M >= 8192 || (K >= 8192 && M >= 2048)) && N % 192 == 0) return 1;
  // batch 32 (M = 4096, r5r): the large tile also wins when its tiles fill >= 70 % of the CUs (QKV
  // 55 vs 61 us, FFN up 80 vs 97, FFN-down dgrad 75 vs 88) or the reduction is deep (K >= 2048:
  // data gradients 64-76 vs 65-83); the 128 x 96 tile keeps the shallow narrow ones (attention
  // output 24 vs 42 us).  Down to M = 512 when the N tiles alone fill the CUs: the MLM decoder
  // forward at batch 32 (640 masked rows x 30528) 122 vs 181-213 us on the 64 x 64 tile (r5bq)
  // (deep reductions from M = 4096: at M = 2048 -- NER fine-tuning batches -- the QKV data
  // gradient runs 38 us on 128 x 96 against 46-50 us on the large tile with split-K, r6j)
  if (M >= 512 && N % 192 == 0 &&
      (10 * ((M + 255) / 256) * (N / 192) >= 7 * hx_cu_slots() || (K >= 2048 && M >= 4096)))
    return 1;
  // 128 x 96 from 1024 rows, or from 512 with a split-K-deep reduction (the decoder's data
  // gradient at batch 32: 117 vs 137-152 us on the large tile, r5bq)
  if ((M >= 1024 || (M >= 512 && K >= 8192)) && N % 96 == 0) return 2;
  if (N % 64 == 0) return 3;
  return -1;
}

// --precision bf16: the same plan, except that the large tile's bf16 products run on 64 x 96
// waves (cfg 1): with one pass per 32-deep stage the A fragments shared by two waves read less LDS
// per MFMA (r4af: FFN up 109 vs 116-121 us, with the GELU epilogue 158 vs 183 us; step 18.88 vs
// 19.02 ms).  The 256 x 256 tile (cfg 5) measured no better on either mode in the step (r4y:
// 36.61 vs 36.65 ms/step forced to 256 x 192; bf16 19.48 with it on every N % 256 product vs 18.8
// without), so it stays an explicit choice (HX_GEMM_F16_CFG=5)
int hx_gemm_bf16_plan(int M, int N, int K) {
  return hx_gemm_f16_plan(M, N, K);
}

int hx_gemm_f16_tiles(int M, int N, int cfg) {
  if (cfg < 0 || cfg >= kCfgs) return 0;
  return (M + cfg_bm(cfg) - 1) / cfg_bm(cfg) * (N / cfg_bn(cfg));
}
int hx_gemm_f16_tm(int M, int cfg) { return cfg < 0 || cfg >= kCfgs ? 0 : (M + cfg_bm(cfg) - 1) / cfg_bm(cfg); }
int hx_gemm_f16_tn(int N, int cfg) { return cfg < 0 || cfg >= kCfgs ? 0 : N / cfg_bn(cfg); }

int hx_gemm_f16_colpart_rows(int M, int cfg) {
  if (cfg < 0 || cfg >= kCfgs) return 0;
  return (M + cfg_bm(cfg) - 1) / cfg_bm(cfg) * cfg_nwm(cfg);
}

int hx_gemm_f16_ks(int M, int N, int K, int cfg) {
  // split-K slabs when the output tiles fill less than half the CUs and the reduction is deep:
  // the MLM decoder's data gradient (K = 30720) and the fine-tuning-sized data gradients
  // (~1-2k token rows, K = 2304 / 3072); each slab keeps >= 512 of the reduction
  if (cfg < 0) return 1;
  const int tiles = hx_gemm_f16_tiles(M, N, cfg), slots = hx_cu_slots();
  if (tiles * 2 > slots || K < 1024) return 1;
  int best = 1;
  for (int ks = 2; ks <= 16; ++ks)
    if (tiles * ks <= slots && K % (16 * ks) == 0 && K / ks >= 512) best = ks;
  return best;
}

// C (+)= sum of the ks slabs (+ bias): the split-K combine with the epilogue the slabs could not apply
__global__ __launch_bounds__(256) void slab_combine_k(const float4* __restrict__ ws, float* __restrict__ C, int64_t ldc,
                                                      int64_t M, int n4, int ks, int beta,
                                                      const float4* __restrict__ bias) {
  const int64_t total = M * n4, slab = M * n4;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / n4;
    const int c = (int)(i - r * n4);
    float4 s = ws[i];
    for (int k = 1; k < ks; ++k) {
      const float4 v = ws[(int64_t)k * slab + i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    if (bias) {
      const float4 b = bias[c];
      s.x += b.x; s.y += b.y; s.z += b.z; s.w += b.w;
    }
    float4* o = reinterpret_cast<float4*>(C + r * ldc) + c;
    if (beta) {
      const float4 v = *o;
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    *o = s;
  }
}

void hx_gemm_f16_slab_combine(const float* ws, float* C, int64_t ldc, int M, int N, int ks, int beta,
                              const float* bias, hipStream_t s) {
  const int64_t n = (int64_t)M * (N / 4);
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  slab_combine_k<<<blocks, 256, 0, s>>>(reinterpret_cast<const float4*>(ws), C, ldc, M, N / 4, ks, beta,
                                        reinterpret_cast<const float4*>(bias));
}

int hx_gemm_f16(const HxGemmF16& p, int cfg, hipStream_t s) {
  const int kd = p.abf16 ? 32 : 16;
  if (cfg < 0 || cfg >= kCfgs || p.M < 1 || p.N % cfg_bn(cfg) || p.K % kd || p.lda % (p.abf16 ? 8 : 4) ||
      p.ldb != (p.abf16 ? 1 : 2) * (int64_t)p.K)
    return -1;
  const int ks = p.ks < 1 ? 1 : p.ks;
  if (p.K % (kd * ks) || (ks > 1 && (p.beta || p.kind || p.bias || p.obf16 || p.c_zs < (int64_t)(p.M - 1) * p.ldc + p.N)))
    return -1;
  if ((p.abf16 && p.kind && !p.obf16) || (p.obf16 && (!p.abf16 || p.ldc % 4)) || (p.apieces && p.abf16)) return -1;
  if (p.kind < 0 || p.kind > 2 || (p.kind && (!p.P || p.beta || p.ldp % 4)) || (p.kind == 2 && !p.aux)) return -1;
  F16Args a;
  a.A = p.A;
  a.lda = p.lda;
  a.a_amax = p.a_amax;
  a.na = p.na;
  a.a_rs = p.a_rs;
  a.B = p.B;
  a.ldb = p.ldb;
  a.b_amax = p.b_amax;
  a.nb = p.nb;
  a.b_rs = p.b_rs;
  a.C = p.C;
  a.ldc = p.ldc;
  a.M = p.M;
  a.N = p.N;
  a.K = p.K;
  a.beta = p.beta;
  a.bias = p.bias;
  a.aux = p.aux;
  a.ldaux = p.ldaux;
  a.P = p.P;
  a.ldp = p.ldp;
  a.colpart = p.colpart;
  a.rowmax = p.rowmax;
  a.colmax = p.colmax;
  a.dmode = p.dmode;
  a.ks = ks;
  a.c_zs = p.c_zs;
  if (p.abf16) {
    if (p.kind == 1) launch_cfg<1, 1, 1>(cfg, a, s);        // bf16 FFN up: gelu'(u), gelu(u) in bf16
    else if (p.kind == 2) launch_cfg<2, 1, 1>(cfg, a, s);   // bf16 FFN-down dgrad * gelu'(u)
    else if (p.obf16 && p.beta) launch_cfg<3, 1, 1>(cfg, a, s);
    else if (p.obf16) launch_cfg<0, 1, 1>(cfg, a, s);
    else if (p.beta) launch_cfg<3, 1, 0>(cfg, a, s);
    else launch_cfg<0, 1, 0>(cfg, a, s);
    return 0;
  }
  if (p.apieces) {   // A already split into P2 pieces by its producer
    if (p.kind == 0 && !p.beta) launch_cfg<0, 2>(cfg, a, s);
    else if (p.kind == 0) launch_cfg<3, 2>(cfg, a, s);
    else if (p.kind == 1) launch_cfg<1, 2>(cfg, a, s);
    else launch_cfg<2, 2>(cfg, a, s);
    return 0;
  }
  if (p.kind == 0 && !p.beta) launch_cfg<0>(cfg, a, s);
  else if (p.kind == 0) launch_cfg<3>(cfg, a, s);
  else if (p.kind == 1) launch_cfg<1>(cfg, a, s);
  else launch_cfg<2>(cfg, a, s);
  return 0;
}

void hx_wgrad_f16_plan(int M, int N, int T, int* cfg, int* nsplit) {
  const int t256 = (M % 256 == 0 && N % 256 == 0) ? (M / 256) * (N / 256) : 0;
  // the large tile also for few-tile shapes whose token splits (one workgroup per CU) keep >= 512
  // tokens each: the attention-output gradient (768 x 768, 9 tiles x 28 splits over 16384 tokens)
  // 78 vs 85-89 us on the 128 tile (r5bm, repeated); at 4096 tokens the splits would be too short
  static const bool few = [] {
    const char* e = getenv("HX_WGRAD_FEW256");
    return !(e && atoi(e) == 0);
  }();
  const int sp_few = t256 ? hx_cu_slots() / t256 : 0;
  const int c = ((t256 >= 24 && t256 <= 512) || (few && t256 >= 8 && t256 < 24 && T / sp_few >= 512)) ? 1 : 0;
  const int tiles = c ? t256 : (M / 128) * (N / 128);
  const int slots = (c ? 1 : 2) * hx_cu_slots();
  // splits fill the CUs: more is faster up to one workgroup per CU (r5y, repeated A/B on one box:
  // QKV 27 tiles x 6 / 7 / 8 / 9 splits 222 / 194 / 178 / 179 us, FFN 36 x 6 / 7 255 / 233 us, x 8
  // (two rounds) 338 us; a single-pass sweep is biased by the warm-up of its first entries)
  int sp = std::max(1, slots / std::max(1, tiles));
  sp = std::min(sp, std::max(1, T / 256));
  if (const char* e = getenv("HX_WGRAD_F16")) {
    int ec = -1, es = -1;
    // "cfg:splits" (splits 0: the plan's for that tile)
    if (sscanf(e, "%d:%d", &ec, &es) == 2 && (ec == 0 || ec == 1) && es >= 0) {
      if (ec == 0 || t256) {
        const int ft = ec ? t256 : (M / 128) * (N / 128), fs = (ec ? 1 : 2) * hx_cu_slots();
        if (es == 0) es = std::min(std::max(1, fs / std::max(1, ft)), std::max(1, T / 256));
        *cfg = ec;
        *nsplit = std::min(es, std::max(1, T / 16));
        return;
      }
    }
  }
  *cfg = c;
  *nsplit = sp;
}

int hx_wgrad_f16(const float* dy, int ldy, const HxColScale& ca, const float* x, int ldx, const HxColScale& cb,
                 float* out, float* ws, int M, int N, int T, int cfg, int nsplit, int mvalid, hipStream_t s) {
  if (ldy % 4 || ldx % 4 || M % 128 || N % 128 || T < 1) return -1;
  if (cfg == 1) {
    if (M % 256 || N % 256) return -1;
    // the add-tid staged kernel (bitwise the same result) unless HX_WGRAD_TID=0: 2-3 % faster
    // standalone (profiles/r6l_wgrad_addtid_ab.log), 0.5 ms/step in the step (36.66 / 36.72 ->
    // 36.18 / 36.15 ms, profiles/r6m_wgrad_addtid_step_ab.txt); read per call (same-process A/B)
    const char* e = getenv("HX_WGRAD_TID");   // 0: ds_write_b128 kernel; 1 (default): 16-token stages; 2: 32
    const int tv = e ? atoi(e) : 1;
    if (tv == 1) {
      wgrad_tid_launch<16>(dy, ldy, ca, x, ldx, cb, out, ws, M, N, T, nsplit, mvalid, s);
      return 0;
    }
    if (tv == 2) {
      wgrad_tid_launch<32>(dy, ldy, ca, x, ldx, cb, out, ws, M, N, T, nsplit, mvalid, s);
      return 0;
    }
    wgrad_launch<256, 256, 128, 64>(dy, ldy, ca, x, ldx, cb, out, ws, M, N, T, nsplit, mvalid, s);
  } else {
    wgrad_launch<128, 128, 64, 64>(dy, ldy, ca, x, ldx, cb, out, ws, M, N, T, nsplit, mvalid, s);
  }
  return 0;
}

// column maxima of a [rows][cols] fp32 matrix: each block a 64-row x 256-column slab (float4 per
// thread), atomic max (non-negative floats order as their bits) into out[cols], zeroed beforehand
__global__ __launch_bounds__(256) void amax_cols_k(const float* __restrict__ x, int64_t rows, int cols, int64_t ld,
                                                   int rows_per_block, float* __restrict__ out) {
  __shared__ float4 red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + lane) * 4;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < cols) {
    for (int64_t r = r0 + w; r < r1; r += 4) {
      const float4 v = *reinterpret_cast<const float4*>(x + r * ld + c);
      m.x = fmaxf(m.x, fabsf(v.x)); m.y = fmaxf(m.y, fabsf(v.y));
      m.z = fmaxf(m.z, fabsf(v.z)); m.w = fmaxf(m.w, fabsf(v.w));
    }
  }
  red[w][lane] = m;
  __syncthreads();
  if (w == 0 && c < cols) {
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      const float4 v = red[j][lane];
      m.x = fmaxf(m.x, v.x); m.y = fmaxf(m.y, v.y); m.z = fmaxf(m.z, v.z); m.w = fmaxf(m.w, v.w);
    }
    atomicMax(reinterpret_cast<unsigned*>(out + c), __float_as_uint(m.x));
    atomicMax(reinterpret_cast<unsigned*>(out + c + 1), __float_as_uint(m.y));
    atomicMax(reinterpret_cast<unsigned*>(out + c + 2), __float_as_uint(m.z));
    atomicMax(reinterpret_cast<unsigned*>(out + c + 3), __float_as_uint(m.w));
  }
}

void hx_amax_cols(const float* x, int64_t rows, int cols, int64_t ld, float* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, (size_t)cols * 4, s);
  if (rows < 1) return;
  const int cb = (cols / 4 + 63) / 64;
  // ~4 workgroups per CU over the row slabs
  int64_t slabs = std::max<int64_t>(1, std::min<int64_t>((rows + 63) / 64, (1024 + cb - 1) / cb));
  const int rpb = (int)((rows + slabs - 1) / slabs);
  slabs = (rows + rpb - 1) / rpb;
  amax_cols_k<<<dim3(cb, (unsigned)slabs), 256, 0, s>>>(x, rows, cols, ld, rpb, out);
}

// max |x| of every row AND every column of a [rows][cols] fp32 matrix in one read: a block = 4
// waves over 64 rows, lane l owns column quads l, l + 64, .. (cols <= 4096: 16 quads); row maxima
// by wave shuffles, column maxima over the block's rows through LDS, then one atomic max per
// column (non-negative floats order as their bits) into colmax, zeroed beforehand.  The operand
// scales of a tensor both a data-gradient GEMM (rows) and a weight gradient (columns) consume
// (the attention backward's dQKV at S > 128, whose key blocks cannot know the final dQ).
constexpr int kRcRows = 64, kRcMaxQ = 16;
__global__ __launch_bounds__(256) void amax_rows_cols_k(const float* __restrict__ x, int64_t rows, int cols,
                                                        int64_t ld, float* __restrict__ rowmax,
                                                        float* __restrict__ colmax) {
  extern __shared__ float4 cred[];   // [4 waves][cols / 4]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nq = cols >> 2;
  const int64_t r0 = (int64_t)blockIdx.x * kRcRows;
  float4 cm[kRcMaxQ];
#pragma unroll
  for (int i = 0; i < kRcMaxQ; ++i) cm[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int rr = w; rr < kRcRows; rr += 4) {
    const int64_t r = r0 + rr;
    if (r >= rows) break;
    const float4* xr = reinterpret_cast<const float4*>(x + r * ld);
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < kRcMaxQ; ++i) {
      const int j = lane + 64 * i;
      if (j < nq) {
        const float4 v = xr[j];
        const float ax = fabsf(v.x), ay = fabsf(v.y), az = fabsf(v.z), aw = fabsf(v.w);
        cm[i].x = fmaxf(cm[i].x, ax); cm[i].y = fmaxf(cm[i].y, ay);
        cm[i].z = fmaxf(cm[i].z, az); cm[i].w = fmaxf(cm[i].w, aw);
        m = fmaxf(m, fmaxf(fmaxf(ax, ay), fmaxf(az, aw)));
      }
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) rowmax[r] = m;
  }
#pragma unroll
  for (int i = 0; i < kRcMaxQ; ++i) {
    const int j = lane + 64 * i;
    if (j < nq) cred[w * nq + j] = cm[i];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < nq; j += 256) {
    float4 v = cred[j];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float4 u = cred[k * nq + j];
      v.x = fmaxf(v.x, u.x); v.y = fmaxf(v.y, u.y); v.z = fmaxf(v.z, u.z); v.w = fmaxf(v.w, u.w);
    }
    unsigned* o = reinterpret_cast<unsigned*>(colmax + 4 * j);
    atomicMax(o, __float_as_uint(v.x));
    atomicMax(o + 1, __float_as_uint(v.y));
    atomicMax(o + 2, __float_as_uint(v.z));
    atomicMax(o + 3, __float_as_uint(v.w));
  }
}

int hx_amax_rows_cols(const float* x, int64_t rows, int cols, int64_t ld, float* rowmax, float* colmax,
                      hipStream_t s) {
  if (cols % 4 || cols > 4 * 64 * kRcMaxQ) return -1;
  (void)hipMemsetAsync(colmax, 0, (size_t)cols * 4, s);
  if (rows < 1) return 0;
  amax_rows_cols_k<<<(unsigned)((rows + kRcRows - 1) / kRcRows), 256, (size_t)cols * 16, s>>>(x, rows, cols, ld,
                                                                                              rowmax, colmax);
  return 0;
}

void hx_amax_rows(const float* x, int64_t rows, int cols, int64_t ld, float* out, hipStream_t s) {
  if (rows < 1) return;
  amax_rows_k<<<(unsigned)((rows + 3) / 4), 256, 0, s>>>(x, rows, cols, ld, out);
}

void hx_split_weight_f16(const HxWeightBatch& d, float* rc, int64_t rc_floats, hipStream_t s) {
  if (d.n < 1) return;
  (void)hipMemsetAsync(rc, 0, (size_t)rc_floats * 4, s);
  amax_weights_k<<<d.start[d.n], 256, 0, s>>>(d, rc);
  split_weight_f16_k<<<d.start[d.n], 256, 0, s>>>(d, rc);
}
