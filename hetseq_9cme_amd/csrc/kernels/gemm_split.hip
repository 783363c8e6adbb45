// fp32 GEMM on the bf16 matrix cores from bf16 PIECES, "NT" form (--fp32-gemm bf16x3/x6):
//
//   C[M][N] (+)= sum over piece pairs (a, b) of A_a[M][K] . B_b[N][K]^T
//
// A = sum_a A_a and B = sum_b B_b are fp32 matrices written as 2 or 3 bf16 pieces
// (ops/split_gemm.py, split.hip); pairs (0,0) (0,1) (1,0) [+ (0,2) (1,1) (2,0)] give
// bf16x3 / bf16x6.  Piece p of row r sits at A + r * lda + p * a_ps (same for B): the
// producers write [rows][pieces][K] tensors, each DISTINCT piece once (half the bytes of a
// pass-stacked operand for bf16x6, the bytes of the fp32 original for bf16x3).
//
// Every forward and data-gradient GEMM of a linear layer runs here (reference sites
// hetseq/bert_modeling.py:334-336 Q/K/V, :383 attention output, :409 + :166-168 FFN up with
// bias_gelu, :419 FFN down): A = activation pieces and B = weight pieces [N_out][K_in]
// (forward), or A = output-gradient pieces and B = TRANSPOSED weight pieces [K_in][N_out]
// (data gradient); beta = 1 accumulates into C (the fused residual gradient).
//
// Structure (the wgrad_split.hip pipeline in NT form):
//  * one workgroup per BM x BN output tile, 8 waves; tiles dealt XCD-aware (the tile list
//    is cut into 8 contiguous ranges, one per XCD, so tiles that share A rows / B rows meet
//    in one XCD's L2);
//  * LDS-DMA staging (buffer_load ... lds): each DISTINCT piece tile of a BK-deep k step is
//    copied global -> LDS once, with no staging registers and no ds_write pass, into NBUF
//    stages (3 at BK = 16: two steps in flight across each barrier, retired by a counted
//    vmcnt; 2 at BK = 32); the XOR swizzle is applied to the per-lane SOURCE address so the
//    lane-linear DMA image reads back conflict-free;
//  * MFMA 32x32x16 bf16: a fragment is ONE ds_read_b128 (row = lane & 31, 8 consecutive k);
//    per 16-deep k-step a wave reads NPC x (MB + NB) fragments and issues passes x MB x NB
//    MFMAs -- every piece fragment is reused by all passes that use it from registers;
//  * epilogues straight from the accumulators after a 4 x 4 lane transpose (DPP quad
//    permutes: each lane then holds 4 consecutive columns of one row -> 16-B fp32 /
//    8-B bf16x4 stores):
//      EPI 0  C (+)= acc
//      EPI 1  u = acc + bias -> C (the FFN pre-activation, kept for the backward) and the
//             pieces of gelu(u) -> P (the FFN-down GEMM's A operand): bias_gelu of
//             bert_modeling.py:104-111 / :166-168 fused into the FFN-up GEMM;
//      EPI 2  t = acc * gelu'(aux (+ bias)) -> pieces P (the FFN-up data-gradient A operand)
//             and per-wave column partial sums of t -> colpart (the FFN-up bias gradient,
//             folded by one small pass): the GELU backward fused into the FFN-down dgrad.
#include <algorithm>

#include <stdio.h>
#include <stdlib.h>

#include "hx_launch.h"
#include "hx_attn.h"
#include "hx_common.h"
#include "hx_reduce.h"

namespace {

using hx::attn::crow;
using hx::attn::f32x16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

// LDS image of a [rows][BK] bf16 tile: 16-B chunk ch of row r at off(r, ch).
//   BK = 32: 64-B rows, ch ^ ((r >> 2) & 3);   BK = 16: 32-B rows, ch ^ ((r >> 3) & 1).
// Either way the 16-lane groups of a ds_read_b128 fragment read (32 consecutive rows, one
// chunk) hit 16 distinct 4-bank slots.  lane_src: the (row within a 1-KiB DMA piece, chunk)
// whose bytes lane L must fetch so that the lane-linear DMA write (image bytes 16 L ..)
// produces that image (the XOR is an involution; pieces start at multiples of RPK rows,
// which keeps the row-dependent XOR bits a function of the lane alone).
template <int BK>
struct Img;
template <>
struct Img<32> {
  static constexpr int RPK = 16;   // rows per KiB
  __device__ __forceinline__ static int off(int r, int ch) { return r * 64 + 16 * (ch ^ ((r >> 2) & 3)); }
  __device__ __forceinline__ static void lane_src(int L, int& rl, int& ch) {
    rl = L >> 2;
    ch = (L & 3) ^ (L >> 4);
  }
};
template <>
struct Img<16> {
  static constexpr int RPK = 32;
  __device__ __forceinline__ static int off(int r, int ch) { return r * 32 + 16 * (ch ^ ((r >> 3) & 1)); }
  __device__ __forceinline__ static void lane_src(int L, int& rl, int& ch) {
    rl = L >> 1;
    ch = (L & 1) ^ ((L >> 4) & 1);
  }
};

// "B16" piece layout (bf16x6): element (r, p, k) at r * 3K + (k / 16) * 48 + p * 16 + k % 16, so
// one 16-deep k step of a row is 96 contiguous bytes holding all three pieces.  The LDS image of
// a stage is the source rows back to back (chunk c = 6 r + 2 p + h of 16 B), with the 16-B chunks
// of every 256-B block XOR-permuted by a function of the block index (period 6): an involution
// inside each block, so one DMA instruction (1 KiB of image) still reads 1 KiB of contiguous
// source, and the 16-lane groups of a ds_read_b128 fragment read (32 consecutive rows, one
// chunk) hit 16 distinct 4-bank slots (exhaustive check: tools/probe/b16_swizzle_check.py).
__device__ __forceinline__ int b16_sw(int blk) {
  const int m = blk % 6;
  return (m == 0 || m == 4 || m == 5) ? 14 : 13;
}
__device__ __forceinline__ int b16_off(int r, int q) {   // byte offset of chunk q of image row r
  const int c = 6 * r + q;
  return 16 * (c ^ b16_sw(c >> 4));
}

// one LDS-DMA wave-instruction: 16 B per lane from buffer byte voff (zeros past the buffer's
// end) to LDS bytes [dst + 16 lane, + 16); dst is wave-uniform.  From asm, so the compiler
// does not drain it (vmcnt(0)) before the next LDS read of the stage being computed; the
// caller retires it with a counted wait before the barrier that publishes the stage.
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
__device__ __forceinline__ void dma_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ u32x4 rsrc_of(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)(size_t)p;
  return u32x4{(uint32_t)a, (uint32_t)(a >> 32) & 0xffffu, bytes, 0x00020000u};
}

template <int NP>
struct PairsNT;
template <>
struct PairsNT<3> {
  static constexpr int a[3] = {0, 0, 1};
  static constexpr int b[3] = {0, 1, 0};
};
template <>
struct PairsNT<6> {
  static constexpr int a[6] = {0, 0, 1, 0, 1, 2};
  static constexpr int b[6] = {0, 1, 0, 2, 1, 0};
};

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

struct Args {
  const uint16_t* A;
  int64_t lda, a_ps;
  const uint16_t* B;
  int64_t ldb, b_ps;
  float* C;
  int64_t ldc;
  int M, N, K, beta;
  const float* bias;
  const float* aux;
  int64_t ldaux;
  uint16_t* P;
  int64_t ldp, p_ps;
  float* colpart;
  uint32_t ksa, ksb;   // bytes between consecutive BK-deep k steps of a row (2 BK natural, 2 BK npc blocked)
  int dmode;           // HxGemmEpi::dmode
  int ks;              // split-K slabs: slab z reduces k steps [z K / ks, (z + 1) K / ks) into C + z c_zs
  int64_t c_zs;
  unsigned long long* stamps;   // diagnostic build (PIPE 9): per wave [dma issue, mfma, dma wait, barrier, total]
};

__device__ __forceinline__ uint2 pack4(const float (&x)[4]) {
  return make_uint2(hx::f2bf(x[0]) | ((uint32_t)hx::f2bf(x[1]) << 16),
                    hx::f2bf(x[2]) | ((uint32_t)hx::f2bf(x[3]) << 16));
}
template <int BM, int BN, int WM, int WN, int NPC, int NP, int BK, int NBUF, int EPI, int PIPE, int LAY = 0,
          int OCC = 1>
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64, OCC) void gemm_piece_k(Args g) {
  constexpr int NWM = BM / WM, NW = NWM * (BN / WN);
  constexpr int MB = WM / 32, NB = WN / 32;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = NPC * (A_BYTES + B_BYTES);
  constexpr int KA = A_BYTES / 1024, KB = B_BYTES / 1024;   // 1-KiB DMA pieces per piece tile
  constexpr int PA = NPC * KA, PTOT = NPC * (KA + KB);
  constexpr int JHI = (PTOT + NW - 1) / NW, JLO = PTOT / NW;   // DMAs per wave and stage
  constexpr int RPK = Img<BK>::RPK;
  static_assert(A_BYTES % 1024 == 0 && B_BYTES % 1024 == 0, "tile / DMA piece mismatch");
  static_assert(NBUF == 2 || NBUF == 3, "stages");
  static_assert(OCC == 1 || NBUF * STAGE <= 80 * 1024, "two workgroups per CU need <= 80 KiB of LDS each");
  static_assert(JLO >= 1, "fewer DMA pieces than waves");
  static_assert(LAY == 0 || (NPC == 3 && BK == 16), "B16 layout: bf16x6, 16-deep stages");
  constexpr bool LA = LAY & 1, LB = LAY & 2;   // A / B operand in the B16 layout
  constexpr int A_REG = NPC * A_BYTES;   // A image bytes of a stage (B image follows)
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int TM = (g.M + BM - 1) / BM, TN = g.N / BN, total = TM * TN;
  const int per = (total * g.ks + 7) / 8;
  const int work0 = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (work0 >= total * g.ks) return;   // uniform per workgroup
  const int z = work0 / total, work = work0 - z * total;   // split-K slab, output tile
  const int nt = work % TN, mt = work / TN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nit = g.K / BK / g.ks, it0 = z * nit;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w % NWM, wn = w / NWM, h = lane >> 5, l32 = lane & 31;
  const int wv = __builtin_amdgcn_readfirstlane(w);

  // buffer resources over this tile's A rows / B rows (rows past M read as zeros: piece p of
  // row r lies inside [r * lda, (r + 1) * lda) because NPC * a_ps <= lda)
  const int mrows = min(BM, g.M - m0);
  const u32x4 ra = rsrc_of(g.A + (int64_t)m0 * g.lda, (uint32_t)((int64_t)mrows * g.lda * 2));
  const u32x4 rb = rsrc_of(g.B + (int64_t)n0 * g.ldb, (uint32_t)((int64_t)BN * g.ldb * 2));

  // this wave's DMA pieces q = wv + NW j of a stage: [A piece tiles | B piece tiles]
  uint32_t voff[JHI];
  int dsto[JHI];
  bool isa[JHI];
  int rl, ch;
  Img<BK>::lane_src(lane, rl, ch);
#pragma unroll
  for (int j = 0; j < JHI; ++j) {
    const int q = wv + NW * j;
    isa[j] = q < PA;
    if ((q < PA && LA) || (q >= PA && LB)) {
      // image chunk x of this lane -> logical chunk c = 6 row + q6 -> source row / 16-B unit
      const int x = 64 * (q < PA ? q : q - PA) + lane;
      const int c = x ^ b16_sw(x >> 4);
      const int r = c / 6, q6 = c - 6 * r;
      voff[j] = (uint32_t)(r * (q < PA ? g.lda : g.ldb) + 8 * q6) * 2;
    } else if (q < PA) {
      const int p = q / KA, r = (q % KA) * RPK + rl;
      voff[j] = (uint32_t)(r * g.lda + p * g.a_ps + 8 * ch) * 2;
    } else {
      const int qb = q - PA, p = qb / KB, r = (qb % KB) * RPK + rl;
      voff[j] = (uint32_t)(r * g.ldb + p * g.b_ps + 8 * ch) * 2;
    }
    dsto[j] = 1024 * q;
  }
  // per-lane LDS byte offsets of the fragments (fixed for the whole k loop)
  int offa[NPC][MB][BK / 16], offb[NPC][NB][BK / 16];
#pragma unroll
  for (int p = 0; p < NPC; ++p)
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
#pragma unroll
      for (int a = 0; a < MB; ++a)
        offa[p][a][ks] = LA ? b16_off(wm * WM + 32 * a + l32, 2 * p + h)
                                  : p * A_BYTES + Img<BK>::off(wm * WM + 32 * a + l32, 2 * ks + h);
#pragma unroll
      for (int b = 0; b < NB; ++b)
        offb[p][b][ks] = A_REG + (LB ? b16_off(wn * WN + 32 * b + l32, 2 * p + h)
                                           : p * B_BYTES + Img<BK>::off(wn * WN + 32 * b + l32, 2 * ks + h));
    }
  const int cnt = (PTOT - wv + NW - 1) / NW;   // JHI or JLO
  const uint32_t lds0 = (uint32_t)(size_t)(lds_void*)lds;   // LDS byte address of the stages
  auto dma = [&](int it, int buf) {
    const uint32_t st = lds0 + buf * STAGE;
    const uint32_t koa = (uint32_t)(it0 + it) * g.ksa, kob = (uint32_t)(it0 + it) * g.ksb;
#pragma unroll
    for (int j = 0; j < JHI; ++j) {
      if (j < JLO || j < cnt) dma16(isa[j] ? ra : rb, st + dsto[j], voff[j] + (isa[j] ? koa : kob));
    }
  };
  auto dma_one = [&](int it, int buf, int j) {   // this wave's j-th DMA piece of stage it
    const uint32_t st = lds0 + buf * STAGE;
    const uint32_t ko = (uint32_t)(it0 + it) * (isa[j] ? g.ksa : g.ksb);
    dma16(isa[j] ? ra : rb, st + dsto[j], voff[j] + ko);
  };
  auto wait_stage = [&]() {   // all but this wave's youngest stage of DMAs landed
    if constexpr (JHI == JLO) {
      dma_wait<JLO>();
    } else {
      if (cnt == JHI) dma_wait<JHI>();
      else dma_wait<JLO>();
    }
  };

  f32x16 acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = f32x16{0};

  auto mma = [&](int buf) {
    const char* st = lds + buf * STAGE;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[NPC][MB], fb[NPC][NB];
#pragma unroll
      for (int p = 0; p < NPC; ++p) {
#pragma unroll
        for (int a = 0; a < MB; ++a)
          fa[p][a] = *reinterpret_cast<const bf16x8*>(st + offa[p][a][ks]);
#pragma unroll
        for (int b = 0; b < NB; ++b)
          fb[p][b] = *reinterpret_cast<const bf16x8*>(st + offb[p][b][ks]);
      }
#pragma unroll
      for (int q = 0; q < NP; ++q)
#pragma unroll
        for (int a = 0; a < MB; ++a)
#pragma unroll
          for (int b = 0; b < NB; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[PairsNT<NP>::a[q]][a], fb[PairsNT<NP>::b[q]][b],
                                                                acc[a][b], 0, 0, 0);
    }
  };

  // MFMA passes of one stage with the next stages' DMA pieces issued between them (one per pass,
  // pinned by sched barriers): the DMA issue -- ~100-150 cycles per piece when issued back to
  // back (profiles/r3_gemm_split.md, stamp build) -- then hides in the shadow of the wave's own
  // MFMAs instead of stalling both waves of the SIMD at the top of every k step
  auto mma_dma = [&](int buf, int dit, int dbuf) {
    const char* st = lds + buf * STAGE;
    bf16x8 fa[NPC][MB], fb[NPC][NB];
#pragma unroll
    for (int p = 0; p < NPC; ++p) {
#pragma unroll
      for (int a = 0; a < MB; ++a) fa[p][a] = *reinterpret_cast<const bf16x8*>(st + offa[p][a][0]);
#pragma unroll
      for (int b = 0; b < NB; ++b) fb[p][b] = *reinterpret_cast<const bf16x8*>(st + offb[p][b][0]);
    }
#pragma unroll
    for (int q = 0; q < NP; ++q) {
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[PairsNT<NP>::a[q]][a], fb[PairsNT<NP>::b[q]][b],
                                                              acc[a][b], 0, 0, 0);
        }
      if (dit >= 0) {
        // pieces j = q (and the leftovers after the last pass)
#pragma unroll
        for (int j = q; j < JHI; j += NP) {
          if (j < JLO || j < cnt) {
            __builtin_amdgcn_sched_barrier(0);
            dma_one(dit, dbuf, j);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    }
  };

  if constexpr (PIPE == 3) {
    static_assert(BK == 16 && NBUF == 3, "interleaved-DMA variant: 16-deep stages, 3 buffers");
    dma(0, 0);
    if (nit > 1) {
      dma(1, 1);
      wait_stage();
    } else {
      dma_wait<0>();
    }
    __syncthreads();
    int cur = 0;
    for (int it = 0; it < nit; ++it) {
      const int nxt2 = cur == 0 ? 2 : cur - 1;
      mma_dma(cur, it + 2 < nit ? it + 2 : -1, nxt2);
      if (it + 2 < nit) wait_stage();
      else dma_wait<0>();
      __syncthreads();
      cur = cur == 2 ? 0 : cur + 1;
    }
  } else if constexpr (PIPE == 4) {
    // Two stages, two workgroups per CU (OCC 2, <= 80 KiB of LDS each): stage it + 1's DMA pieces
    // are issued between stage it's MFMA passes and retired before the barrier that ends the
    // step.  Latency the single in-flight stage cannot hide -- and one workgroup's epilogue
    // stores -- are covered by the OTHER workgroup's MFMAs on the same SIMDs.
    static_assert(BK == 16 && NBUF == 2, "two-stage interleaved variant: 16-deep stages, 2 buffers");
    dma(0, 0);
    dma_wait<0>();
    __syncthreads();
    for (int it = 0; it < nit; ++it) {
      mma_dma(it & 1, it + 1 < nit ? it + 1 : -1, (it + 1) & 1);
      dma_wait<0>();
      __syncthreads();
    }
  } else if constexpr (PIPE == 1) {
    // Fragments of the stage being multiplied live in registers (two named sets, loop
    // unrolled by 2), so three stages can be in flight in three LDS buffers and the LDS
    // reads of stage it + 1 overlap the second MFMA group of stage it:
    //   group 1 (all fragments consumed) | own DMA of it+1 landed | barrier |
    //   reads of it+1 -> other set, DMA of it+3 into stage it's buffer | group 2
    static_assert(BK == 16 && NBUF == 3, "register-pipelined variant: one 16-deep k step per stage");
    typedef bf16x8 Frag[NPC][MB + NB];
    auto rd = [&](int buf, Frag& F) {
      const char* st = lds + buf * STAGE;
#pragma unroll
      for (int p = 0; p < NPC; ++p) {
#pragma unroll
        for (int a = 0; a < MB; ++a)
          F[p][a] = *reinterpret_cast<const bf16x8*>(st + offa[p][a][0]);
#pragma unroll
        for (int b = 0; b < NB; ++b)
          F[p][MB + b] = *reinterpret_cast<const bf16x8*>(st + offb[p][b][0]);
      }
    };
    // pass q of the product (PairsNT order); group 1 = the first half of the passes
    auto pass = [&](const Frag& F, int q) {
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[PairsNT<NP>::a[q]][a], F[PairsNT<NP>::b[q]][MB + b],
                                                              acc[a][b], 0, 0, 0);
    };
    constexpr int G1 = (NP + 1) / 2;
    auto step = [&](int it, int cur, Frag& Fc, Frag& Fn) {
#pragma unroll
      for (int q = 0; q < G1; ++q) pass(Fc, q);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // every read of stage it done
      if (it + 2 < nit) wait_stage();
      else dma_wait<0>();
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      __builtin_amdgcn_sched_barrier(0);
      const int nxt = cur == 2 ? 0 : cur + 1;
      if (it + 1 < nit) rd(nxt, Fn);
      if (it + 3 < nit) dma(it + 3, cur);
#pragma unroll
      for (int q = G1; q < NP; ++q) pass(Fc, q);
      return nxt;
    };
    Frag F0, F1;
    dma(0, 0);
    if (nit > 1) dma(1, 1);
    if (nit > 2) dma(2, 2);
    // stage 0 landed: stages 1, 2 may stay in flight
    if (nit > 2) {
      if constexpr (JHI == JLO) dma_wait<2 * JLO>();
      else if (cnt == JHI) dma_wait<2 * JHI>();
      else dma_wait<2 * JLO>();
    } else if (nit > 1) {
      wait_stage();
    } else {
      dma_wait<0>();
    }
    __syncthreads();
    rd(0, F0);
    int cur = 0;
    for (int it = 0; it < nit; it += 2) {
      cur = step(it, cur, F0, F1);
      if (it + 1 >= nit) break;
      cur = step(it + 1, cur, F1, F0);
    }
  } else if constexpr (PIPE == 2) {
    // One fragment register set, refilled in place: bf16x6 passes ordered so that the three
    // fragment groups the post-barrier passes do not use are reloaded (next stage) right
    // after the barrier, the rest as soon as their last MFMA has issued.
    //   before the barrier: (0,2) (0,1) (1,1) (2,0)    after: (0,0) (1,0)
    //   reloads: b2 b1 a2 | after (0,0): a0 | after (1,0): a1 b0
    // The next stage opens with (0,2) (0,1), whose fragments were reloaded first.
    static_assert(BK == 16 && NBUF == 3 && NP == 6, "in-place register pipeline: bf16x6, 16-deep stages");
    bf16x8 fa[3][MB], fb[3][NB];
    auto rda = [&](int buf, int p) {
      const char* st = lds + buf * STAGE;
#pragma unroll
      for (int a = 0; a < MB; ++a)
        fa[p][a] = *reinterpret_cast<const bf16x8*>(st + offa[p][a][0]);
    };
    auto rdb = [&](int buf, int p) {
      const char* st = lds + buf * STAGE;
#pragma unroll
      for (int b = 0; b < NB; ++b)
        fb[p][b] = *reinterpret_cast<const bf16x8*>(st + offb[p][b][0]);
    };
    auto pass = [&](int pa, int pb) {
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[pa][a], fb[pb][b], acc[a][b], 0, 0, 0);
    };
    dma(0, 0);
    if (nit > 1) dma(1, 1);
    if (nit > 2) dma(2, 2);
    if (nit > 2) {
      if constexpr (JHI == JLO) dma_wait<2 * JLO>();
      else if (cnt == JHI) dma_wait<2 * JHI>();
      else dma_wait<2 * JLO>();
    } else if (nit > 1) {
      wait_stage();
    } else {
      dma_wait<0>();
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      rda(0, p);
      rdb(0, p);
    }
    int cur = 0;
    for (int it = 0; it < nit; ++it) {
      pass(0, 2);
      pass(0, 1);
      pass(1, 1);
      pass(2, 0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (it + 2 < nit) wait_stage();
      else dma_wait<0>();
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      __builtin_amdgcn_sched_barrier(0);
      const int nxt = cur == 2 ? 0 : cur + 1;
      const bool more = it + 1 < nit;
      if (more) {
        rdb(nxt, 2);
        rdb(nxt, 1);
        rda(nxt, 2);
      }
      if (it + 3 < nit) dma(it + 3, cur);
      pass(0, 0);
      if (more) rda(nxt, 0);
      pass(1, 0);
      if (more) {
        rda(nxt, 1);
        rdb(nxt, 0);
      }
      cur = nxt;
    }
  } else if constexpr (NBUF == 2) {
    dma(0, 0);
    dma_wait<0>();
    __syncthreads();
    for (int it = 0; it < nit; ++it) {
      if (it + 1 < nit) dma(it + 1, (it + 1) & 1);
      mma(it & 1);
      dma_wait<0>();
      __syncthreads();
    }
  } else {
    // stage it + 2 goes into the buffer step it - 1 read (all waves passed the barrier after
    // those reads); before each barrier only stage it + 1 must have landed
    dma(0, 0);
    if (nit > 1) {
      dma(1, 1);
      wait_stage();
    } else {
      dma_wait<0>();
    }
    __syncthreads();
    int cur = 0;
    unsigned long long sd = 0, sm = 0, sw = 0, sb = 0, t00 = 0;
    if constexpr (PIPE == 9) t00 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < nit; ++it) {
      const int nxt2 = cur == 0 ? 2 : cur - 1;
      unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0;
      if constexpr (PIPE == 9) {
        __builtin_amdgcn_sched_barrier(0);
        t0 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
      }
      if (it + 2 < nit) dma(it + 2, nxt2);
      if constexpr (PIPE == 9) {
        __builtin_amdgcn_sched_barrier(0);
        t1 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
      }
      mma(cur);
      if constexpr (PIPE == 9) {
        __builtin_amdgcn_sched_barrier(0);
        t2 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
      }
      if (it + 2 < nit) wait_stage();
      else dma_wait<0>();
      if constexpr (PIPE == 9) {
        __builtin_amdgcn_sched_barrier(0);
        t3 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
      }
      __syncthreads();
      if constexpr (PIPE == 9) {
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t4 = __builtin_amdgcn_s_memtime();
        sd += t1 - t0;
        sm += t2 - t1;
        sw += t3 - t2;
        sb += t4 - t3;
      }
      cur = cur == 2 ? 0 : cur + 1;
    }
    if constexpr (PIPE == 9) {
      if (lane == 0 && g.stamps) {
        unsigned long long* o = g.stamps + ((int64_t)blockIdx.x * NW + w) * 5;
        o[0] = sd;
        o[1] = sm;
        o[2] = sw;
        o[3] = sb;
        o[4] = __builtin_amdgcn_s_memtime() - t00;
      }
    }
  }

  // ---- epilogue: 4 x 4 quad transpose, then lane (l32 & 3) owns row 8 gq + 4 h + (l32 & 3)
  // of each 32 x 32 block and its columns (l32 & ~3) .. + 3.  Buffer resources over the
  // tile's valid rows: stores past M are dropped, loads past M return 0 (no branches).
  const int mrow = wm * WM + 4 * h + (l32 & 3), ncol = wn * WN + (l32 & ~3);
  const hx::Buf cbuf(g.C + z * g.c_zs + (int64_t)m0 * g.ldc + n0, (uint32_t)((int64_t)mrows * g.ldc * 4));
  auto coff = [&](int a, int b, int gq) { return (uint32_t)((mrow + 32 * a + 8 * gq) * g.ldc + ncol + 32 * b) * 4; };
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  // transpose one 4-row group in place: acc[a][b][4 gq + i] = column i of this lane's row
  auto tr = [&](int a, int b, int gq) {
    float v[4] = {acc[a][b][4 * gq], acc[a][b][4 * gq + 1], acc[a][b][4 * gq + 2], acc[a][b][4 * gq + 3]};
    transpose4(v, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[a][b][4 * gq + i] = v[i];
  };
  if constexpr (EPI == 0 || EPI == 3) {
    // EPI 3 = EPI 0 with beta: one row block of accumulators at a time (a sched barrier keeps
    // the compiler from hoisting every block's C loads: 256-VGPR cap); row block a + 1's C
    // loads are issued before row block a is summed, so one load latency per tile is exposed
    // instead of one per row block
    f32x4 c[2][NB][4];
    auto ldc = [&](int a, f32x4 (&d)[NB][4]) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          d[b][gq] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(cbuf.r, coff(a, b, gq), 0, 0));
    };
    if constexpr (EPI == 3) ldc(0, c[0]);
#pragma unroll
    for (int a = 0; a < MB; ++a) {
      if constexpr (EPI == 3) {
        if (a + 1 < MB) ldc(a + 1, c[(a + 1) & 1]);
      }
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          tr(a, b, gq);
          f32x4 o = {acc[a][b][4 * gq], acc[a][b][4 * gq + 1], acc[a][b][4 * gq + 2], acc[a][b][4 * gq + 3]};
          if constexpr (EPI == 3) o += c[a & 1][b][gq];
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), cbuf.r, coff(a, b, gq), 0, 0);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    const hx::Buf pbuf(g.P + (int64_t)m0 * g.ldp + n0, (uint32_t)((int64_t)mrows * g.ldp * 2));
    auto poff = [&](int a, int b, int gq, int p) {
      return (uint32_t)((int64_t)(mrow + 32 * a + 8 * gq) * g.ldp + p * g.p_ps + ncol + 32 * b) * 2;
    };
    float csum[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) csum[b][i] = 0.f;
    const hx::Buf xbuf(EPI == 2 ? g.aux + (int64_t)m0 * g.ldaux + n0 : g.C, (uint32_t)((int64_t)mrows * g.ldaux * 4));
    // the bias columns of this lane (all row blocks share them), loaded once
    float bias[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
      if (g.bias) t = *reinterpret_cast<const float4*>(g.bias + n0 + ncol + 32 * b);
      bias[b][0] = t.x; bias[b][1] = t.y; bias[b][2] = t.z; bias[b][3] = t.w;
    }
    // EPI 2: the aux block of (a, b) is loaded while the previous block is processed (two
    // register sets), so the tile exposes one load latency instead of MB * NB
    f32x4 ub[2][4];
    auto ldu = [&](int a, int b, f32x4 (&d)[4]) {
#pragma unroll
      for (int gq = 0; gq < 4; ++gq)
        d[gq] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              xbuf.r, (uint32_t)((mrow + 32 * a + 8 * gq) * g.ldaux + ncol + 32 * b) * 4, 0,
                                              0));
    };
    if constexpr (EPI == 2) ldu(0, 0, ub[0]);
#pragma unroll
    for (int a = 0; a < MB; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const float* bb = bias[b];
        const int blk = a * NB + b;
        if constexpr (EPI == 2) {
          if (blk + 1 < MB * NB) ldu((blk + 1) / NB, (blk + 1) % NB, ub[(blk + 1) & 1]);
        }
        const f32x4* u = ub[blk & 1];
        // row groups in pairs (gq, gq + 1): after the quad transpose a lane holds 4 columns of
        // one row; lanes l and l ^ 4 hold the two halves of 8 consecutive columns of the same
        // row, so one swizzle per piece word gives the even lane row gq's 8 columns and the odd
        // lane row gq + 1's -- the piece stores go out as 16-B (8 bf16) stores, half the store
        // instructions of 8-B ones (the epilogue is store-issue bound: MI355X_MICROARCH.md, the
        // attention store-tail row of the price list)
        const bool odd = (l32 & 4) != 0;
#pragma unroll
        for (int gp = 0; gp < 2; ++gp) {
          uint2 pk[2][NPC];
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
          const int gq = 2 * gp + s2;
          tr(a, b, gq);
          float v[4] = {acc[a][b][4 * gq], acc[a][b][4 * gq + 1], acc[a][b][4 * gq + 2], acc[a][b][4 * gq + 3]};
          if constexpr (EPI == 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] += bb[i];
            if (g.dmode) {
              // gelu(u) and gelu'(u) from ONE erf (hx::gelu_f / hx::gelu_grad_f bit for bit)
              f32x4 o;
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const float e = erff(v[i] * (1.0f / 1.41421f));
                o[i] = 0.5f * (1.0f + e) + hx::gelu_pdf_f(v[i]);
                v[i] = v[i] * 0.5f * (1.0f + e);
              }
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), cbuf.r, coff(a, b, gq), 0, 0);
            } else {
              const f32x4 o = {v[0], v[1], v[2], v[3]};
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), cbuf.r, coff(a, b, gq), 0, 0);
#pragma unroll
              for (int i = 0; i < 4; ++i) v[i] = hx::gelu_f(v[i]);
            }
          } else {
            const bool in = mrow + 32 * a + 8 * gq < mrows;   // rows past M: no bias-gradient share
            if (g.dmode) {   // aux holds gelu'(u) already
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                v[i] *= u[gq][i];
                csum[b][i] += in ? v[i] : 0.f;
              }
            } else {
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                v[i] *= hx::gelu_grad_f(u[gq][i] + bb[i]);
                csum[b][i] += in ? v[i] : 0.f;
              }
            }
          }
#pragma unroll
          for (int p = 0; p < NPC; ++p) {
            float hp[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              hp[i] = hx::bf2f(hx::f2bf(v[i]));
              if (p + 1 < NPC) v[i] -= hp[i];
            }
            pk[s2][p] = pack4(hp);
          }
          }
          // 0x101f: swizzle bitmask mode, and 0x1f, xor 4 (lane l <-> l ^ 4)
#pragma unroll
          for (int p = 0; p < NPC; ++p) {
            const uint2 snd = odd ? pk[0][p] : pk[1][p];
            const uint32_t r0 = (uint32_t)__builtin_amdgcn_ds_swizzle((int)snd.x, 0x101f);
            const uint32_t r1 = (uint32_t)__builtin_amdgcn_ds_swizzle((int)snd.y, 0x101f);
            const u32x4 o = odd ? u32x4{r0, r1, pk[1][p].x, pk[1][p].y} : u32x4{pk[0][p].x, pk[0][p].y, r0, r1};
            __builtin_amdgcn_raw_buffer_store_b128(o, pbuf.r, poff(a, b, 2 * gp + (odd ? 1 : 0), p) - (odd ? 8u : 0u),
                                                   0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    if constexpr (EPI == 2) {
      if (g.colpart) {
        // sum over the 4 rows of a quad and the two 32-lane halves; lanes (l32 & 3) == 0,
        // h == 0 then hold this wave's 4-column sums -> partial row (mt * NWM + wm)
        float* row = g.colpart + (int64_t)(mt * NWM + wm) * g.N + n0 + wn * WN;
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float t = csum[b][i];
            t += qx1(t);
            t += qx2(t);
            t += __shfl_xor(t, 32, 64);
            csum[b][i] = t;
          }
        if ((l32 & 3) == 0 && h == 0) {
#pragma unroll
          for (int b = 0; b < NB; ++b)
            *reinterpret_cast<float4*>(row + 32 * b + l32) =
                make_float4(csum[b][0], csum[b][1], csum[b][2], csum[b][3]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------- configurations
// cfg 0: 256 x 192 tile, waves 4 (M) x 2 (N) of 64 x 96, BK 16, 3 stages (bf16x6 126 KiB LDS):
//        exactly one, three and four rounds of 256 workgroups at N = 768 / 2304 / 3072, M = 16384
// cfg 1: 256 x 256 tile, waves 2 x 4 of 128 x 64, BK 16, 3 stages (144 KiB): the wgrad_split
//        geometry (0.75 fragment reads per MFMA)
// cfg 2: 256 x 128 tile, waves 4 x 2 of 64 x 64, BK 32, 2 stages (144 KiB)
// bf16x3 (2 pieces) runs the same tiles at BK 32 with 2 stages (cfg 0: 112 KiB, cfg 1: 128, cfg 2: 96).
// cfg 3 (bf16x6): cfg 0's tile with the in-place register pipeline (PIPE 2)
// cfg 4 (bf16x6): 256 x 128 tile, waves 4 x 2 of 64 x 64, BK 16, 3 stages, two fragment sets (PIPE 1)
// cfg 5 (bf16x6): cfg 1's tile, PIPE 2;   cfg 6 (bf16x6): cfg 4's tile, PIPE 2
// cfg 7 (bf16x6): 256 x 128 tile, 4 waves (2 x 2) of 128 x 64, BK 16, 2 stages (72 KiB), two
//        workgroups per CU (PIPE 4): one workgroup's epilogue overlaps the other's MFMAs
// (round 3, removed: 4 waves of 128 x 96 at one wave per SIMD with both fragment sets in registers
//  needs > 256 VGPRs + AGPR accumulators, and hipcc spilled 100-200 dwords inside the k loop)
constexpr int kCfgs = 8;
int cfg_bm(int) { return 256; }
int cfg_bn(int c) { return (c == 0 || c == 3) ? 192 : (c == 1 || c == 5) ? 256 : 128; }
int cfg_nwm(int c) { return (c == 1 || c == 5 || c == 7) ? 2 : 4; }

template <int BM, int BN, int WM, int WN, int NPC, int NP, int BK, int NBUF, int EPI, int PIPE = 0, int LAY = 0,
          int OCC = 1>
void launch_one(const Args& a, hipStream_t s) {
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  const int total = ((a.M + BM - 1) / BM) * (a.N / BN) * a.ks;
  const int per = (total + 7) / 8;
  const size_t smem = (size_t)NBUF * NPC * (BM + BN) * BK * 2;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(
        reinterpret_cast<const void*>(&gemm_piece_k<BM, BN, WM, WN, NPC, NP, BK, NBUF, EPI, PIPE, LAY, OCC>),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr = true;
  }
  gemm_piece_k<BM, BN, WM, WN, NPC, NP, BK, NBUF, EPI, PIPE, LAY, OCC><<<8 * per, NT, smem, s>>>(a);
}

// HX_GEMM_PIPE (read per launch, so one process can A/B variants): 3 = interleaved DMA (default).
// Measured and removed in round 3 (tools/probe/gemm_stagger_probe.py): the two waves of each SIMD
// staggered by one pass (MI355X_MICROARCH.md 'Two waves per SIMD' item 9) 2-3 % slower on every
// BERT shape (profiles/r3_gemm_stagger_probe.log); the same pipeline on 16x16x32 MFMAs (two
// 16-deep pieces side by side along k, three MFMAs per 16x16 block and stage) 1-6 % slower --
// the clock gain of the 16x16 shape (r3_mfma16_clock_probe.log: a timing-only swap of the same
// fragments, since removed) does not survive its 26 instead
// of 15 fragment reads per k step (profiles/r3_gemm_mfma16_probe.log).  Ping-pong (the two waves
// of each SIMD half a k step apart: one multiplies while the other reads its fragments, two
// barrier-delimited phases per k step, MI355X_MICROARCH.md 'Two waves per SIMD') was correct
// at every k-step count but 0.5-2.4 % slower on the plain shapes and 11 % on the GELU epilogue
// (profiles/r3_gemm_pingpong_probe.log): with the clock held at 1.8-1.9 GHz by power
// (profiles/r3_gemm_pmc.md) the fragment-read gaps it closes are not what limits the loop.
static int pipe_mode() {
  const char* e = getenv("HX_GEMM_PIPE");
  return e ? atoi(e) : 3;
}

template <int NPC, int NP, int EPI, int PIPE, int LAY>
void launch_lay(int cfg, const Args& a, hipStream_t s) {
  if (cfg == 7)
    launch_one<256, 128, 128, 64, NPC, NP, 16, 2, EPI, 4, LAY, 2>(a, s);
  else if (cfg == 0)
    launch_one<256, 192, 64, 96, NPC, NP, 16, 3, EPI, PIPE, LAY>(a, s);
  else
    launch_one<256, 256, 128, 64, NPC, NP, 16, 3, EPI, PIPE, LAY>(a, s);
}

template <int NPC, int NP, int EPI>
void launch_cfg(int cfg, int lay, const Args& a, hipStream_t s) {
  constexpr int BK = NPC == 3 ? 16 : 32, NBUF = NPC == 3 ? 3 : 2;
  if constexpr (NPC == 3) {
    const int pm = pipe_mode();
    if (cfg == 7 || (pm == 3 && (cfg == 0 || cfg == 1))) {   // DMA pieces interleaved with the passes
      if (lay == 0) launch_lay<NPC, NP, EPI, 3, 0>(cfg, a, s);
      else if (lay == 1) launch_lay<NPC, NP, EPI, 3, 1>(cfg, a, s);
      else if (lay == 2) launch_lay<NPC, NP, EPI, 3, 2>(cfg, a, s);
      else launch_lay<NPC, NP, EPI, 3, 3>(cfg, a, s);
      return;
    }
    if (lay) {   // B16 piece layout(s), plain pipeline
      if (cfg == 3 || cfg == 5) {   // lay == 3 (host check)
        if (cfg == 3) launch_one<256, 192, 64, 96, NPC, NP, 16, 3, EPI, 2, 3>(a, s);
        else launch_one<256, 256, 128, 64, NPC, NP, 16, 3, EPI, 2, 3>(a, s);
        return;
      }
      if (lay == 1) launch_lay<NPC, NP, EPI, 0, 1>(cfg, a, s);
      else if (lay == 2) launch_lay<NPC, NP, EPI, 0, 2>(cfg, a, s);
      else launch_lay<NPC, NP, EPI, 0, 3>(cfg, a, s);
      return;
    }
  }
  if (cfg == 0)
    launch_one<256, 192, 64, 96, NPC, NP, BK, NBUF, EPI>(a, s);
  else if (cfg == 1)
    launch_one<256, 256, 128, 64, NPC, NP, BK, NBUF, EPI>(a, s);
  else if (cfg == 2)
    launch_one<256, 128, 64, 64, NPC, NP, 32, 2, EPI>(a, s);
  else if constexpr (NPC == 3) {
    if (cfg == 3)
      launch_one<256, 192, 64, 96, NPC, NP, 16, 3, EPI, 2>(a, s);
    else if (cfg == 4)
      launch_one<256, 128, 64, 64, NPC, NP, 16, 3, EPI, 1>(a, s);
    else if (cfg == 5)
      launch_one<256, 256, 128, 64, NPC, NP, 16, 3, EPI, 2>(a, s);
    else if (cfg == 9)
      launch_one<256, 192, 64, 96, NPC, NP, 16, 3, EPI, 9>(a, s);
    else
      launch_one<256, 128, 64, 64, NPC, NP, 16, 3, EPI, 2>(a, s);
  }
}

}  // namespace

int hx_gemm_split_plan(int M, int N, int K, int passes, int lay) {
  (void)K;
  if (const char* e = getenv("HX_GEMM_CFG")) {
    const int c = atoi(e);
    if (c >= 0 && c < kCfgs && N % cfg_bn(c) == 0 && (c < 3 || passes == 6) &&
        (!lay || c == 0 || c == 1 || c == 7 || ((c == 3 || c == 5) && lay == 3)))
      return c;
  }
  // measured at M = 16384, bf16x6 (tools/probe/gemm_layout_probe.py, qkv_plan_probe.py):
  // N = 768 on the 256 x 192 tile (one round of 256 workgroups), N = 2304 on 256 x 192 (B16
  // weights; 256 x 128 if the weights are natural), wide outputs (3072) on 256 x 256
  if (N % 192 == 0 && N <= 1536) {
    // 256 x 192 fills exactly one round of 256 CUs at M = 16384, N = 768.  With CUs reserved for
    // a concurrent comm kernel (cu_reserve.hip) that round no longer fits: take the tile whose
    // rounds are fuller (256 x 256: 192 tiles, one round on >= 192 free CUs)
    const int slots = hx_cu_slots();
    if (slots < hx_num_cus() && N % 256 == 0) {
      // rounds of slot-filling waves, in units of one 256 x 192 tile's time (256 x 256: 4/3)
      const int t0 = (M + 255) / 256 * (N / 192), t1 = (M + 255) / 256 * (N / 256);
      const double r0 = (double)((t0 + slots - 1) / slots), r1 = (double)((t1 + slots - 1) / slots) * (256.0 / 192.0);
      if (r1 < r0) return 1;
    }
    return 0;
  }
  if (N % 2304 == 0) return lay ? 0 : 2;
  if (N % 256 == 0) return 1;
  if (N % 192 == 0) return 0;
  if (N % 128 == 0 && !lay) return 2;
  return -1;
}

// should the B operand (weight pieces) of an N-column product be written in the B16 layout?
// bf16x6 on the 256 x 192 / 256 x 256 tiles: 3-9 % faster (tools/probe/gemm_layout_probe.py),
// the QKV forward (N = 2304) included: 256 x 192 over B16 weights 282 us against 306 us for the
// 256 x 128 tile over natural ones (tools/probe/qkv_plan_probe.py, profiles/r3_qkv_plan_probe.log).
int hx_gemm_split_weight_b16(int N, int passes) {
  if (passes != 6) return 0;
  const int c = hx_gemm_split_plan(1 << 14, N, 768, passes, 2);
  return (c == 0 || c == 1 || c == 7) ? 1 : 0;
}

int hx_gemm_split_ks(int M, int N, int K, int passes) {
  const int cfg = hx_gemm_split_plan(M, N, K, passes, 0);
  if (cfg < 0) return 1;
  const int bk = (passes == 6 && cfg != 2) ? 16 : 32;
  const int tiles = (M + cfg_bm(cfg) - 1) / cfg_bm(cfg) * (N / cfg_bn(cfg)), slots = hx_cu_slots();
  if (tiles * 2 > slots || K < 8192) return 1;
  // the most slabs that keep one round (tiles * ks <= slots), each slab >= 2048 deep
  int best = 1;
  for (int ks = 2; ks <= 16; ++ks)
    if (tiles * ks <= slots && K % (bk * ks) == 0 && K / ks >= 2048) best = ks;
  return best;
}

int hx_gemm_split_colpart_rows(int M, int cfg) {
  if (cfg < 0 || cfg >= kCfgs) return 0;
  return (M + cfg_bm(cfg) - 1) / cfg_bm(cfg) * cfg_nwm(cfg);
}

int hx_gemm_split_nt(const void* A, int64_t lda, int64_t a_ps, const void* B, int64_t ldb, int64_t b_ps, float* C,
                     int64_t ldc, int M, int N, int K, int passes, int beta, const HxGemmEpi* epi, int cfg,
                     hipStream_t s, int lay, int ks, int64_t c_zs) {
  const int npc = passes == 6 ? 3 : passes == 3 ? 2 : 0;
  if (!npc || M < 1 || cfg < 0 || cfg >= kCfgs || N % cfg_bn(cfg)) return -1;
  if (cfg >= 3 && npc != 3) return -1;
  const int bk = (npc == 3 && cfg != 2) ? 16 : 32;
  if (K % bk || npc * a_ps > lda || npc * b_ps > ldb) return -1;
  // split-K: plain stores of ks partial products (C + z c_zs), whole k steps per slab
  if (ks < 1 || K % (bk * ks) || (ks > 1 && (beta || (epi && epi->kind) || c_zs < (int64_t)(M - 1) * ldc + N)))
    return -1;
  // lay bit 0 / bit 1: A / B operand in the B16 layout [rows][K / 16][3][16] (bf16x6, cfgs 0 1 3 5)
  // instead of [rows][npc][K]: one 16-deep k step of a row is 96 contiguous bytes
  if (lay && (lay > 3 || npc != 3 || !(cfg == 0 || cfg == 1 || cfg == 7 || ((cfg == 3 || cfg == 5) && lay == 3))))
    return -1;
  Args a;
  a.A = (const uint16_t*)A;
  a.lda = lda;
  a.a_ps = a_ps;
  a.B = (const uint16_t*)B;
  a.ldb = ldb;
  a.b_ps = b_ps;
  a.C = C;
  a.ldc = ldc;
  a.M = M;
  a.N = N;
  a.K = K;
  a.beta = beta;
  const int kind = epi ? epi->kind : 0;
  a.bias = epi ? epi->bias : nullptr;
  a.aux = epi ? epi->aux : nullptr;
  a.ldaux = epi ? epi->ldaux : 0;
  a.P = epi ? epi->P : nullptr;
  a.ldp = epi ? epi->ldp : 0;
  a.p_ps = epi ? epi->p_ps : 0;
  a.colpart = epi ? epi->colpart : nullptr;
  a.dmode = epi ? epi->dmode : 0;
  a.ks = ks;
  a.c_zs = c_zs;
  a.ksa = (uint32_t)(bk * 2 * ((lay & 1) ? npc : 1));
  a.ksb = (uint32_t)(bk * 2 * ((lay & 2) ? npc : 1));
  a.stamps = nullptr;
  if (kind == 1 && (!a.P || beta)) return -1;
  if (kind == 2 && (!a.P || !a.aux)) return -1;
  if (kind < 0 || kind > 2) return -1;
#define HX_GS(NPC_, NP_)                                          \
  do {                                                            \
    if (kind == 0 && !beta) launch_cfg<NPC_, NP_, 0>(cfg, lay, a, s);  \
    else if (kind == 0) launch_cfg<NPC_, NP_, 3>(cfg, lay, a, s);      \
    else if (kind == 1) launch_cfg<NPC_, NP_, 1>(cfg, lay, a, s);      \
    else launch_cfg<NPC_, NP_, 2>(cfg, lay, a, s);                     \
  } while (0)
  if (passes == 6) HX_GS(3, 6);
  else HX_GS(2, 3);
#undef HX_GS
  return 0;
}

void hx_fold_cols(const float* partial, int rows, int N, float* out, int accumulate, hipStream_t s) {
  hx::fold_rows(partial, rows, N, N, N, out, nullptr, nullptr, accumulate, s);
}

// diagnostic: cfg 0's kernel (EPI 0) with per-phase s_memtime stamps, one record of 5 counters per
// wave (grid 8 * ceil(tiles / 8) workgroups x 8 waves); returns the grid size
int hx_gemm_split_stamps(const void* A, const void* B, float* C, int M, int N, int K, unsigned long long* stamps,
                         hipStream_t s, int lay) {
  if (N % 192 || K % 16) return -1;
  Args a{};
  a.A = (const uint16_t*)A;
  a.lda = 3 * (int64_t)K;
  a.a_ps = K;
  a.B = (const uint16_t*)B;
  a.ldb = 3 * (int64_t)K;
  a.b_ps = K;
  a.C = C;
  a.ldc = N;
  a.M = M;
  a.N = N;
  a.K = K;
  a.ksa = a.ksb = lay ? 96 : 32;
  a.ks = 1;
  a.stamps = stamps;
  if (lay)
    launch_one<256, 192, 64, 96, 3, 6, 16, 3, 0, 9, 1>(a, s);
  else
    launch_one<256, 192, 64, 96, 3, 6, 16, 3, 0, 9>(a, s);
  const int total = ((M + 255) / 256) * (N / 192);
  return 8 * ((total + 7) / 8);
}

// ---------------------------------------------------------------- diagnostic: LDS-DMA shape probe
// Every workgroup (8 waves) streams `iters` stages of 42 one-KiB LDS-DMA pieces (the 256 x 192
// bf16x6 stage) into a 3-stage LDS ring, with the GEMM's counted waits and barriers but no MFMA.
// Each piece reads seg-byte contiguous segments from 1024 / seg consecutive rows of a shared
// 1344-row x `ld`-byte region (8.3 MB at ld 6144: Infinity-Cache resident); every shape sweeps the
// same region band by band, so only the per-instruction segment shape differs.
namespace {
__global__ __launch_bounds__(512) void dma_probe_k(const uint16_t* src, uint32_t bytes, int seg, int ld, int iters) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int PTOT = 42, NW = 8, STAGE = PTOT * 1024;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(w);
  const u32x4 rs = rsrc_of(src, bytes);
  const uint32_t lds0 = (uint32_t)(size_t)(lds_void*)lds;
  const int R = 1024 / seg, csteps = ld / seg;
  const uint32_t lofs = (uint32_t)((lane * 16 / seg) * ld + (lane * 16) % seg);
  const int cnt = (PTOT - wv + NW - 1) / NW;
  auto dma = [&](int it, int buf) {
    const int itw = it + (int)blockIdx.x;   // workgroups at different points of the sweep
    const int band = (itw / csteps) % (1344 / (PTOT * R));
    const uint32_t col = (uint32_t)(itw % csteps) * seg;
    for (int j = 0; j < 6; ++j) {
      const int q = wv + NW * j;
      if (q < PTOT) {
        const uint32_t so = (uint32_t)((band * PTOT + q) * R) * ld + col;
        dma16(rs, lds0 + buf * STAGE + 1024 * q, so + lofs);
      }
    }
  };
  dma(0, 0);
  dma(1, 1);
  __syncthreads();
  int cur = 0;
  for (int it = 0; it < iters; ++it) {
    const int nxt2 = cur == 0 ? 2 : cur - 1;
    if (it + 2 < iters) dma(it + 2, nxt2);
    if (it + 2 < iters) {
      if (cnt == 6) dma_wait<6>();
      else dma_wait<5>();
    } else {
      dma_wait<0>();
    }
    __syncthreads();
    cur = cur == 2 ? 0 : cur + 1;
  }
}
}  // namespace
void hx_dma_probe(const void* src, uint32_t bytes, int seg, int ld, int iters, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&dma_probe_k), hipFuncAttributeMaxDynamicSharedMemorySize,
                              3 * 42 * 1024);
    attr = true;
  }
  if ((uint64_t)1344 * ld > bytes) return;
  dma_probe_k<<<grid, 512, 3 * 42 * 1024, s>>>((const uint16_t*)src, bytes, seg, ld, iters);
}
