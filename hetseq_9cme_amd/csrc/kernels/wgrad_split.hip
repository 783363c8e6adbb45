// Weight gradient of an fp32 linear layer on the bf16 matrix cores (--fp32-gemm bf16x3/x6):
//
//   dW[M][N] (fp32) = sum over tokens t and piece pairs (a, b) of dY_a[t][M]^T . X_b[t][N]
//
// where dY = dY_0 + dY_1 (+ dY_2) and X = X_0 + X_1 (+ X_2) are the bf16 pieces written by
// split.hip (ops/split_gemm.py) and the pairs are (0,0) (0,1) (1,0) [+ (0,2) (1,1) (2,0)].
//
// The first form of this product ran the generic tokens-as-reduction kernel
// (wgrad_bf16.hip) over the stacked [passes * T] plane rows, i.e. it streamed every pass
// operand from memory and LDS separately: dY_0 twice for bf16x3, X_0 three times for
// bf16x6.  Here each DISTINCT piece of a token block is staged once (global -> registers
// -> swizzled LDS tile) and every pass reuses it from registers:
//
//   per 16-token MFMA step and wave (64 x 64 outputs): NA + NB piece fragments per 32-row
//   block, then 3 (6) x 4 MFMAs -- 0.67 (0.5) KB of LDS fragment reads per MFMA instead
//   of 1 KB, and 2/3 (1/2) of the global / L2 bytes per FLOP.
//
// Everything else follows wgrad_bf16.hip: 64-token pipeline steps staged two steps ahead in
// registers, XOR-swizzled 8 x 32 subtiles read as k-major fragments with the gfx950
// transposing LDS read (ds_read_b64_tr_b16), split-K over token ranges to fill the CUs,
// fp32 partial tiles summed by one vectorised pass (no float atomics), XCD-aware work
// ranges.
#include <algorithm>

#include <stdio.h>
#include <stdlib.h>

#include "hx_launch.h"
#include "hx_attn.h"
#include "hx_common.h"

namespace {

using hx::attn::crow;
using hx::attn::f32x16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;   // tokens per pipeline step (two 16-deep MFMA k-steps per barrier)

// LDS image of a [BK rows][W columns] bf16 tile (wgrad_bf16.hip's layout): 8-row x 32-column
// subtiles of 512 B, XOR-swizzled 16-B chunks, odd subtiles with the rows of each pair
// swapped (conflict-free 16-B stores and transposed reads).
template <int W>
__device__ __forceinline__ int toff(int row, int ch) {
  return (row >> 3) * (16 * W) + 512 * (ch >> 2) + 64 * ((row & 7) ^ ((ch >> 2) & 1)) +
         16 * ((ch & 3) ^ ((row >> 2) & 3));
}
template <int W>
__device__ __forceinline__ void tr_base(int lane, int (&lo)[2], int (&hi)[2]) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = 8 * (g >> 1) + q, ch = 2 * (g & 1) + (p >> 1);
  lo[0] = toff<W>(row, ch) + 8 * (p & 1);
  hi[0] = toff<W>(row + 4, ch) + 8 * (p & 1);
  lo[1] = toff<W>(row, ch + 4) - 512 + 8 * (p & 1);
  hi[1] = toff<W>(row + 4, ch + 4) - 512 + 8 * (p & 1);
}
template <int W>
__device__ __forceinline__ bf16x8 frag(const char* tile, const int (&lo)[2], const int (&hi)[2], int k0, int c0,
                                       int odd) {
  const int d = (k0 >> 4) * (32 * W) + (c0 >> 5) * 512;
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(tile + lo[odd] + d));
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(tile + hi[odd] + d));
  const v4i16 v[2] = {a, b};
  return *reinterpret_cast<const bf16x8*>(v);
}

// one LDS-DMA wave-instruction: 16 B per lane from buffer byte voff (zeros past the buffer's
// end) to LDS bytes [dst + 16 lane, + 16); dst is wave-uniform.  Issued from asm: the
// compiler would otherwise wait for every outstanding DMA (vmcnt(0)) before the next LDS
// read of ANY address, i.e. before the fragment reads of the step being computed, which
// serialises staging and MFMA work.  The caller retires the DMAs itself (dma_wait) before
// the barrier that publishes the buffer.  M0 is written and restored inside the statement.
__device__ __forceinline__ void dma16(u32x4 rsrc, char* dst, uint32_t voff) {
  const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_void*)dst);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(m), "s"(rsrc)
               : "memory");
}
template <int N>
__device__ __forceinline__ void dma_wait() {   // at most N of this wave's DMAs still in flight
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// raw buffer descriptor over [p, p + bytes): stride 0, reads past the end return zeros
__device__ __forceinline__ u32x4 rsrc_of(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)(size_t)p;
  return u32x4{(uint32_t)a, (uint32_t)(a >> 32) & 0xffffu, bytes, 0x00020000u};
}

// piece pairs (a, b) of the product, in pass order (ops/split_gemm.py)
template <int NP>
struct Pairs;
template <>
struct Pairs<3> {
  static constexpr int a[3] = {0, 0, 1};
  static constexpr int b[3] = {0, 1, 0};
};
template <>
struct Pairs<6> {
  static constexpr int a[6] = {0, 0, 1, 0, 1, 2};
  static constexpr int b[6] = {0, 1, 0, 2, 1, 0};
};

struct PieceBases {
  const uint16_t* a[3];   // dY pieces (same row stride lda)
  const uint16_t* b[3];   // X pieces (same row stride ldb)
};

// Second product of a GROUPED launch (hx_wgrad_split_group): same tokens T, tile shape and split
// count; its work items follow the first product's, so the two fill one round of workgroups
// together (e.g. the 9-tile attention-output dW beside the 27-tile QKV dW: alone it runs 14-way
// token splits at 0.93 PF/s).  M == 0: no second product.
struct Prob2 {
  PieceBases P;
  int lda, ldb;
  float* out;
  int M, N, mvalid, mord;
};

// AHEAD: token steps staged ahead in registers (2: two register sets; 1: one set, fewer
// VGPRs -- the bf16x6 256 x 128 tile spills with two).  MORD: work order inside a token
// split, 0 = output-column tiles fastest, 1 = output-row tiles fastest (the tiles one XCD
// runs together then share both operands' token slabs in its L2 when M has few row tiles).
// BKT: tokens per pipeline stage; NBUF: LDS stages (3 only with LDS-DMA staging, AHEAD 0:
// two stages in flight across each barrier, retired by a counted wait).
template <int BM, int BN, int WM, int WN, int NPC, int NP, int AHEAD, int MORD, int BKT = BK, int NBUF = 2>
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64) void wgrad_split_k(PieceBases P, int lda, int ldb,
                                                                           float* __restrict__ out, int M, int N,
                                                                           int T, int kchunk, int nsplit,
                                                                           int mvalid, Prob2 g2) {
  constexpr int NWM = BM / WM, NW = NWM * (BN / WN), NT = NW * 64;
  constexpr int MB = WM / 32, NB = WN / 32;
  constexpr int CA = BKT * BM / 8 / NT, CB = BKT * BN / 8 / NT;   // 16-B chunks per thread per piece
  static_assert(WM % 64 == 0 && WN % 64 == 0, "subtile parity of fragment a is a & 1");
  static_assert(AHEAD == 0 || (CA >= 1 && CB >= 1 && BKT * BM / 8 % NT == 0 && BKT * BN / 8 % NT == 0),
                "tile / thread mismatch");
  static_assert(NBUF == 2 || (NBUF == 3 && AHEAD == 0), "three stages need LDS-DMA staging");
  constexpr int A_BYTES = BKT * BM * 2, B_BYTES = BKT * BN * 2;
  constexpr int STAGE = NPC * (A_BYTES + B_BYTES);
  extern __shared__ __attribute__((aligned(16))) char lds[];   // [2 stages][NPC A tiles, NPC B tiles]

  const int total1 = (M / BM) * (N / BN) * nsplit;
  const int total2 = g2.M ? (g2.M / BM) * (g2.N / BN) * nsplit : 0;
  const int per = (total1 + total2 + 7) / 8;
  int work = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (work >= total1 + total2) return;   // uniform per workgroup
  bool mord = MORD;
  if (work >= total1) {   // the grouped launch's second product (uniform per workgroup)
    work -= total1;
    P = g2.P;
    lda = g2.lda;
    ldb = g2.ldb;
    out = g2.out;
    M = g2.M;
    N = g2.N;
    mvalid = g2.mvalid;
    mord = g2.mord;
  }
  const int TM = M / BM, TN = N / BN;
  const int nt = mord ? (work / TM) % TN : work % TN;
  const int mt = mord ? work % TM : (work / TN) % TM;
  const int sp = work / (TN * TM);
  const int m0 = mt * BM, n0 = nt * BN;
  const int t0 = sp * kchunk, t1 = min(T, t0 + kchunk);
  const int nit = (t1 - t0 + BKT - 1) / BKT;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w % NWM, wn = w / NWM, h = lane >> 5, l32 = lane & 31;

  // one buffer resource per piece over rows [t0, t1): loads past t1 return zeros
  const uint32_t abytes = (uint32_t)((int64_t)(t1 - t0) * lda * 2), bbytes = (uint32_t)((int64_t)(t1 - t0) * ldb * 2);
  const hx::Buf abuf[3] = {hx::Buf(P.a[0] + (int64_t)t0 * lda, abytes), hx::Buf(P.a[1] + (int64_t)t0 * lda, abytes),
                           hx::Buf(P.a[2] + (int64_t)t0 * lda, abytes)};
  const hx::Buf bbuf[3] = {hx::Buf(P.b[0] + (int64_t)t0 * ldb, bbytes), hx::Buf(P.b[1] + (int64_t)t0 * ldb, bbytes),
                           hx::Buf(P.b[2] + (int64_t)t0 * ldb, bbytes)};
  uint32_t va[CA], vb[CB];
  int sa[CA], sb[CB];
#pragma unroll
  for (int i = 0; i < CA; ++i) {
    const int e = tid + i * NT, row = e / (BM / 8), ch = e % (BM / 8);
    va[i] = (uint32_t)(row * lda + m0 + 8 * ch) * 2;
    sa[i] = toff<BM>(row, ch);
  }
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    const int e = tid + i * NT, row = e / (BN / 8), ch = e % (BN / 8);
    vb[i] = (uint32_t)(row * ldb + n0 + 8 * ch) * 2;
    sb[i] = toff<BN>(row, ch);
  }
  int alo[2], ahi[2], blo[2], bhi[2];
  tr_base<BM>(lane, alo, ahi);
  tr_base<BN>(lane, blo, bhi);

  u32x4 ra0[NPC][CA ? CA : 1], rb0[NPC][CB ? CB : 1], ra1[NPC][CA ? CA : 1], rb1[NPC][CB ? CB : 1];
  auto load = [&](int it, u32x4 (&ra)[NPC][CA], u32x4 (&rb)[NPC][CB]) {
    const uint32_t soa = (uint32_t)it * BKT * lda * 2, sob = (uint32_t)it * BKT * ldb * 2;
#pragma unroll
    for (int p = 0; p < NPC; ++p) {
#pragma unroll
      for (int i = 0; i < CA; ++i) ra[p][i] = __builtin_amdgcn_raw_buffer_load_b128(abuf[p].r, va[i], soa, 0);
#pragma unroll
      for (int i = 0; i < CB; ++i) rb[p][i] = __builtin_amdgcn_raw_buffer_load_b128(bbuf[p].r, vb[i], sob, 0);
    }
  };
  auto store = [&](int buf, const u32x4 (&ra)[NPC][CA], const u32x4 (&rb)[NPC][CB]) {
    char* st = lds + buf * STAGE;
#pragma unroll
    for (int p = 0; p < NPC; ++p) {
      char* at = st + p * A_BYTES;
      char* bt = st + NPC * A_BYTES + p * B_BYTES;
#pragma unroll
      for (int i = 0; i < CA; ++i) *reinterpret_cast<u32x4*>(at + sa[i]) = ra[p][i];
#pragma unroll
      for (int i = 0; i < CB; ++i) *reinterpret_cast<u32x4*>(bt + sb[i]) = rb[p][i];
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
    for (int ks = 0; ks < BKT / 16; ++ks) {
      bf16x8 fa[NPC][MB], fb[NPC][NB];
#pragma unroll
      for (int p = 0; p < NPC; ++p) {
#pragma unroll
        for (int a = 0; a < MB; ++a)
          fa[p][a] = frag<BM>(st + p * A_BYTES, alo, ahi, 16 * ks, wm * WM + 32 * a, a & 1);
#pragma unroll
        for (int b = 0; b < NB; ++b)
          fb[p][b] = frag<BN>(st + NPC * A_BYTES + p * B_BYTES, blo, bhi, 16 * ks, wn * WN + 32 * b, b & 1);
      }
#pragma unroll
      for (int q = 0; q < NP; ++q)
#pragma unroll
        for (int a = 0; a < MB; ++a)
#pragma unroll
          for (int b = 0; b < NB; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[Pairs<NP>::a[q]][a], fb[Pairs<NP>::b[q]][b],
                                                                acc[a][b], 0, 0, 0);
    }
  };

  if constexpr (AHEAD == 0) {
    // LDS-DMA staging (buffer_load ... lds): no staging registers and no ds_write pass.  A
    // DMA wave-instruction writes 1 KiB of LDS lane-linearly, so each lane loads the 16-B
    // chunk whose swizzled image position (toff) is its lane slot: the inverse of toff on the
    // SOURCE address, the same image as store() writes.  NBUF 2: step it + 1 is in flight
    // while step it runs on the matrix cores and is retired (dma_wait<0>) before the barrier
    // that publishes it; NBUF 3: two steps in flight, a counted wait retires the older one.
    constexpr int JA = A_BYTES / 1024 / NW, JB = B_BYTES / 1024 / NW;   // 1-KiB pieces per wave and piece
    static_assert(JA >= 1 && JB >= 1 && A_BYTES % (1024 * NW) == 0 && B_BYTES % (1024 * NW) == 0,
                  "tile / wave mismatch");
    const int wv = __builtin_amdgcn_readfirstlane(w);
    auto src = [&](int o, int W, int ld, int c0) {   // image byte o of a [BKT][W] tile -> source byte offset
      const int rb = o / (16 * W), rem = o % (16 * W), sub = rem >> 9;
      const int row = 8 * rb + (((rem & 511) >> 6) ^ (sub & 1));
      const int ch = 4 * sub + (((rem & 63) >> 4) ^ ((row >> 2) & 3));
      return (uint32_t)(row * ld + c0 + 8 * ch) * 2;
    };
    u32x4 ra[3], rb[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      ra[p] = rsrc_of(P.a[p] + (int64_t)t0 * lda, abytes);
      rb[p] = rsrc_of(P.b[p] + (int64_t)t0 * ldb, bbytes);
    }
    uint32_t da[JA], db[JB];
#pragma unroll
    for (int j = 0; j < JA; ++j) da[j] = src(1024 * (wv * JA + j) + 16 * lane, BM, lda, m0);
#pragma unroll
    for (int j = 0; j < JB; ++j) db[j] = src(1024 * (wv * JB + j) + 16 * lane, BN, ldb, n0);
    auto dma = [&](int it, int buf) {
      const uint32_t soa = (uint32_t)it * BKT * lda * 2, sob = (uint32_t)it * BKT * ldb * 2;
      char* st = lds + buf * STAGE;
#pragma unroll
      for (int p = 0; p < NPC; ++p) {
#pragma unroll
        for (int j = 0; j < JA; ++j)
          dma16(ra[p], st + p * A_BYTES + 1024 * (wv * JA + j), da[j] + soa);
#pragma unroll
        for (int j = 0; j < JB; ++j)
          dma16(rb[p], st + NPC * A_BYTES + p * B_BYTES + 1024 * (wv * JB + j), db[j] + sob);
      }
    };
    if constexpr (NBUF == 2) {
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
      // stage it + 2 is issued into the buffer step it - 1 read (retired by the last barrier);
      // before the barrier only stage it + 1 must have landed, stage it + 2 stays in flight
      constexpr int PER = NPC * (JA + JB);   // DMA wave-instructions per stage
      dma(0, 0);
      if (nit > 1) dma(1, 1);
      if (nit > 1) dma_wait<PER>(); else dma_wait<0>();
      __syncthreads();
      int cur = 0;
      for (int it = 0; it < nit; ++it) {
        const int nxt2 = cur == 0 ? 2 : cur - 1;
        if (it + 2 < nit) dma(it + 2, nxt2);
        mma(cur);
        if (it + 2 < nit) dma_wait<PER>(); else dma_wait<0>();
        __syncthreads();
        cur = cur == 2 ? 0 : cur + 1;
      }
    }
  } else if constexpr (AHEAD == 2) {
    load(0, ra0, rb0);
    load(1, ra1, rb1);
    store(0, ra0, rb0);
    __syncthreads();
    for (int it = 0; it < nit; it += 2) {
      load(it + 2, ra0, rb0);
      mma(0);
      store(1, ra1, rb1);
      __syncthreads();
      if (it + 1 >= nit) break;
      load(it + 3, ra1, rb1);
      mma(1);
      store(0, ra0, rb0);
      __syncthreads();
    }
  } else {
    // one register set: step it + 1 is loaded while step it runs on the matrix cores, then
    // written to the other LDS buffer (last read before the previous barrier)
    load(0, ra0, rb0);
    store(0, ra0, rb0);
    __syncthreads();
    for (int it = 0; it < nit; ++it) {
      const int cur = it & 1;
      if (it + 1 < nit) load(it + 1, ra0, rb0);
      mma(cur);
      if (it + 1 < nit) store(cur ^ 1, ra0, rb0);
      __syncthreads();
    }
  }

  float* o = out + (nsplit > 1 ? (int64_t)sp * M * N : 0);
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int n = n0 + wn * WN + 32 * b + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WM + 32 * a + crow(r, h);
        if (m < mvalid) o[(int64_t)m * N + n] = acc[a][b][r];   // rows past mvalid: padding
      }
    }
}

__global__ __launch_bounds__(256) void split_sum2_k(const float4* __restrict__ ws, float4* __restrict__ out,
                                                   int64_t n4, int64_t slab4, int nsplit) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 s = ws[i];
    for (int k = 1; k < nsplit; ++k) {
      const float4 v = ws[(int64_t)k * slab4 + i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    out[i] = s;
  }
}

template <int BM, int BN, int WM, int WN, int NPC, int NP, int AHEAD, int MORD, int BKT = BK, int NBUF = 2>
void launch(const PieceBases& P, int lda, int ldb, float* out, float* ws, int M, int N, int T, int nsplit,
            int mvalid, hipStream_t s, const Prob2* second = nullptr, float* ws2 = nullptr) {
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  const int kchunk = ((T + nsplit - 1) / nsplit + BK - 1) / BK * BK;
  nsplit = (T + kchunk - 1) / kchunk;
  Prob2 g2{};
  if (second) {
    g2 = *second;
    if (nsplit > 1) {   // partial slabs into ws2 (all rows), folded by the second sum pass
      g2.out = ws2;
      g2.mvalid = g2.M;
    }
  }
  const int total = (M / BM) * (N / BN) * nsplit + (g2.M ? (g2.M / BM) * (g2.N / BN) * nsplit : 0);
  const int per = (total + 7) / 8;
  const size_t smem = NBUF * (size_t)NPC * BKT * (BM + BN) * sizeof(uint16_t);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_split_k<BM, BN, WM, WN, NPC, NP, AHEAD, MORD, BKT, NBUF>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr = true;
  }
  wgrad_split_k<BM, BN, WM, WN, NPC, NP, AHEAD, MORD, BKT, NBUF><<<8 * per, NT, smem, s>>>(
      P, lda, ldb, nsplit > 1 ? ws : out, M, N, T, kchunk, nsplit, nsplit > 1 ? M : mvalid, g2);
  if (nsplit > 1) {
    auto fold = [&](const float* w, float* o, int m, int n, int mv) {
      const int64_t n4 = (int64_t)mv * n / 4, slab4 = (int64_t)m * n / 4;
      const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
      split_sum2_k<<<blocks, 256, 0, s>>>(reinterpret_cast<const float4*>(w), reinterpret_cast<float4*>(o), n4, slab4,
                                          nsplit);
    };
    fold(ws, out, M, N, mvalid);
    if (second) fold(ws2, second->out, second->M, second->N, second->mvalid);
  }
}

}  // namespace

// cfg 0: 128x128 workgroup tile, 4 waves of 64x64; cfg 1: 256x128, 8 waves of 64x64;
// cfg 2 (bf16x6 only): 256x256, 8 waves of 128x64, LDS-DMA staging into three 16-token
// stages (0.75 fragment reads per MFMA instead of 1, 2/3 of the staged bytes per FLOP).
// The split count fills one round of workgroup slots (256 for cfgs 1 / 2, 512 for cfg 0);
// HX_WGRAD_SPLIT_CFG="cfg:nsplit" overrides (tools/bench_wgrad.py --split).
static int tile_m(int c) { return c == 0 ? 128 : 256; }
static int tile_n(int c) { return c == 2 ? 256 : 128; }
static bool cfg_ok(int c, int M, int N, int passes) {
  return c >= 0 && c <= 2 && (c != 2 || passes == 6) && M % tile_m(c) == 0 && N % tile_n(c) == 0;
}
void hx_wgrad_split_plan(int M, int N, int T, int passes, int* cfg, int* nsplit) {
  // cfg 2 where its tiles fill the 256 slots evenly (BERT: QKV, FFN-up / -down dW 3-10 %
  // faster than cfg 1); with fewer tiles (768 x 768: 9) the deep token split's partial sums
  // cost more than the larger tile saves, with more than one round (the MLM decoder) the
  // last round runs part-empty (profiles/r2_wgrad_split_dma.log)
  const int tiles2 = (M / 256) * (N / 256);
  int c = cfg_ok(2, M, N, passes) && tiles2 >= 24 && tiles2 <= 256 ? 2 : cfg_ok(1, M, N, passes) ? 1 : 0;
  // one round of workgroup slots on the CUs a concurrent comm kernel leaves free (cu_reserve.hip)
  int slots = (c == 0 ? 2 : 1) * hx_cu_slots();
  // (planning for a fraction of the slots beside the side stream's partner kernels measured slower:
  // 50 / 75 % gave 52.44-52.50 ms/step against 52.04 / 52.25 at 100 %, round 3)
  const int tiles0 = (M / tile_m(c)) * (N / tile_n(c));
  int s = std::max(1, slots / std::max(1, tiles0));
  s = std::min(s, std::max(1, T / 256));
  if (const char* e = getenv("HX_WGRAD_SPLIT_CFG")) {
    int ec = -1, es = -1;
    if (sscanf(e, "%d:%d", &ec, &es) == 2 && es >= 1 && cfg_ok(ec, M, N, passes)) {
      c = ec;
      s = std::min(es, std::max(1, T / BK));
    }
  }
  *cfg = c;
  *nsplit = s;
}

int hx_wgrad_split(const void* const* dy_pieces, int ldy, const void* const* x_pieces, int ldx, int passes,
                   float* out, float* ws, int M, int N, int T, int cfg, int nsplit, int mvalid, hipStream_t s) {
  PieceBases P;
  const int npc = passes == 6 ? 3 : 2;
  for (int i = 0; i < 3; ++i) {
    P.a[i] = (const uint16_t*)dy_pieces[i < npc ? i : 0];
    P.b[i] = (const uint16_t*)x_pieces[i < npc ? i : 0];
  }
  // HX_WGRAD_SPLIT_VAR="ahead,mord" selects a pipeline variant (tools/bench_wgrad.py --split)
  // default: two register stages; output-row tiles fastest when there are fewer of them
  // than column tiles (768 x 3072 FFN-down dW: 421 -> 406 us; tools/bench_wgrad.py --split 6
  // --variants, profiles/r2_wgrad_split_variants.log -- the other variants are within 3 %)
  // bf16x6: LDS-DMA staging (AHEAD 0) -- 6-8 % faster than the register pipelines at every
  // BERT shape; bf16x3 keeps two register stages (its DMA variant is up to 12 % slower)
  int ahead = passes == 6 ? 0 : 2, mord = M < N ? 1 : 0;
  if (const char* e = getenv("HX_WGRAD_SPLIT_VAR")) {
    int a = 0, o = 0;
    if (sscanf(e, "%d,%d", &a, &o) == 2 && (a >= 0 && a <= 2) && (o == 0 || o == 1)) {
      ahead = a;
      mord = o;
    }
  }
#define HX_WS_LAUNCH(BM_, NPC_, NP_)                                                           \
  do {                                                                                         \
    if (ahead == 0 && mord == 0)                                                               \
      launch<BM_, 128, 64, 64, NPC_, NP_, 0, 0>(P, ldy, ldx, out, ws, M, N, T, nsplit, mvalid, s);     \
    else if (ahead == 0)                                                                       \
      launch<BM_, 128, 64, 64, NPC_, NP_, 0, 1>(P, ldy, ldx, out, ws, M, N, T, nsplit, mvalid, s);     \
    else if (ahead == 2 && mord == 0)                                                          \
      launch<BM_, 128, 64, 64, NPC_, NP_, 2, 0>(P, ldy, ldx, out, ws, M, N, T, nsplit, mvalid, s);     \
    else if (ahead == 2)                                                                       \
      launch<BM_, 128, 64, 64, NPC_, NP_, 2, 1>(P, ldy, ldx, out, ws, M, N, T, nsplit, mvalid, s);     \
    else if (mord == 0)                                                                        \
      launch<BM_, 128, 64, 64, NPC_, NP_, 1, 0>(P, ldy, ldx, out, ws, M, N, T, nsplit, mvalid, s);     \
    else                                                                                       \
      launch<BM_, 128, 64, 64, NPC_, NP_, 1, 1>(P, ldy, ldx, out, ws, M, N, T, nsplit, mvalid, s);     \
  } while (0)
  if (passes == 3) {
    if (cfg == 1)
      HX_WS_LAUNCH(256, 2, 3);
    else
      HX_WS_LAUNCH(128, 2, 3);
  } else if (passes == 6) {
    if (cfg == 2) {
      if (mord == 0)
        launch<256, 256, 128, 64, 3, 6, 0, 0, 16, 3>(P, ldy, ldx, out, ws, M, N, T, nsplit, mvalid, s);
      else
        launch<256, 256, 128, 64, 3, 6, 0, 1, 16, 3>(P, ldy, ldx, out, ws, M, N, T, nsplit, mvalid, s);
    } else if (cfg == 1)
      HX_WS_LAUNCH(256, 3, 6);
    else
      HX_WS_LAUNCH(128, 3, 6);
  } else {
    return -1;
  }
#undef HX_WS_LAUNCH
  return 0;
}

// Two weight gradients over the same tokens in ONE launch (bf16x6, both on the 256 x 256 tile):
// the token split count fills one round of workgroup slots with the two products' tiles
// together.  Returns the split count (the caller sizes ws1 / ws2 as nsplit * M * N floats when
// it is > 1), or -1 when the pair does not qualify.
int hx_wgrad_split_group_plan(int M1, int N1, int M2, int N2, int T, int passes) {
  if (passes != 6 || !cfg_ok(2, M1, N1, passes) || !cfg_ok(2, M2, N2, passes)) return -1;
  const int tiles = (M1 / 256) * (N1 / 256) + (M2 / 256) * (N2 / 256);
  if (tiles > hx_cu_slots()) return -1;
  int s = std::max(1, hx_cu_slots() / tiles);
  return std::min(s, std::max(1, T / 256));
}

int hx_wgrad_split_group(const void* const* dy1, int ldy1, const void* const* x1, int ldx1, float* out1, float* ws1,
                         int M1, int N1, int mvalid1, const void* const* dy2, int ldy2, const void* const* x2, int ldx2,
                         float* out2, float* ws2, int M2, int N2, int mvalid2, int T, int nsplit, hipStream_t s) {
  if (!cfg_ok(2, M1, N1, 6) || !cfg_ok(2, M2, N2, 6) || nsplit < 1) return -1;
  PieceBases P1;
  Prob2 g2{};
  for (int i = 0; i < 3; ++i) {
    P1.a[i] = (const uint16_t*)dy1[i];
    P1.b[i] = (const uint16_t*)x1[i];
    g2.P.a[i] = (const uint16_t*)dy2[i];
    g2.P.b[i] = (const uint16_t*)x2[i];
  }
  g2.lda = ldy2;
  g2.ldb = ldx2;
  g2.out = out2;
  g2.M = M2;
  g2.N = N2;
  g2.mvalid = mvalid2;
  g2.mord = M2 < N2 ? 1 : 0;
  if (M1 < N1)
    launch<256, 256, 128, 64, 3, 6, 0, 1, 16, 3>(P1, ldy1, ldx1, out1, ws1, M1, N1, T, nsplit, mvalid1, s, &g2, ws2);
  else
    launch<256, 256, 128, 64, 3, 6, 0, 0, 16, 3>(P1, ldy1, ldx1, out1, ws1, M1, N1, T, nsplit, mvalid1, s, &g2, ws2);
  return 0;
}
