// Weight gradient of y = x W^T for bf16 activations: dW[M][N] (fp32) = dY[T][M]^T . X[T][N].
//
// Both operands are stored with the reduction index (tokens, T = B*S = 16384 for BERT
// phase 1) as the ROW index, and the output is small (768 x 3072 = 2.4 M elements), so
// the library GEMMs for this "TN" case run at ~450 TF/s on MI355X (measured by
// tools/bench_wgrad.py: 165-175 us for the 77 GFLOP FFN weight gradients, i.e. 18% of
// the 2.5 PF/s bf16 MFMA peak).  This kernel:
//
//  * splits the token reduction over ``nsplit`` workgroups per output tile so the grid
//    fills the 256 CUs even though there are only 9-36 output tiles; partial tiles go
//    to an fp32 workspace and one vectorised pass sums them (no float atomics: at
//    ~1.3 TB/s the atomic rate would cost more than the GEMM);
//  * stages [32 tokens][BM | BN] tiles in LDS exactly as they sit in memory (16-B
//    coalesced loads, XOR-swizzled 16-B chunks) and builds the k-major MFMA fragments
//    with the gfx950 transposing LDS read ``ds_read_b64_tr_b16`` (two per fragment) --
//    no transposed copies of the 100 MB activations;
//  * double-buffers the LDS tiles with the next tile's global loads in flight in
//    registers: one barrier per 32-token step;
//  * maps workgroups XCD-aware: the hardware deals consecutive workgroup ids round-robin
//    to the 8 XCDs, so the work list is cut into 8 contiguous ranges, one per XCD, and
//    the workgroups of one XCD walk neighbouring output tiles of the same token range
//    (shared dY / X rows stay in that XCD's L2).
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

// BK = tokens per pipeline step (BK / 16 MFMA k-steps per barrier): a template parameter,
// 32 or 64 per tile configuration (see the cfg table at the bottom)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// LDS image of a [BK rows][W columns] bf16 tile: 8-row x 32-column subtiles of 512 B with
// XOR-swizzled 16-B chunks (cdna_hip_programming.md T10 layout (a)); in odd subtiles the
// rows of each pair swap places (row slot (row & 7) ^ 1).  Byte offset of 16-B chunk ch of
// row `row`.  The 16-B stores are serviced in groups of 8 lanes on 32 banks (128 B): the 8
// chunks of a group span two subtiles 512 B apart, which without the row swap land on the
// same 64 B of banks (2-way conflict on every store, ~30 % of the LDS-array cycles in the
// PMC trace); with it they cover all 32 banks.  The transposed reads (2 x 32 lanes on 64
// banks) stay conflict-free.  Linear in 32-column PAIRS of blocks (+1024 B) and 16-row
// k-steps (+32W B), so a wave needs two address registers per operand and subtile parity
// (rows q and q+4, even/odd subtile): every other fragment read is an immediate offset.
template <int W>
__device__ __forceinline__ int toff(int row, int ch) {
  return (row >> 3) * (16 * W) + 512 * (ch >> 2) + 64 * ((row & 7) ^ ((ch >> 2) & 1)) +
         16 * ((ch & 3) ^ ((row >> 2) & 3));
}
// per-lane byte offsets of the two transposed reads of the (k0 = 0, c0 = 0) fragment (even
// subtile) and of the c0 = 32 fragment minus its 512-B subtile base (odd subtile)
template <int W>
__device__ __forceinline__ void tr_base(int lane, int (&lo)[2], int (&hi)[2]) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = 8 * (g >> 1) + q, ch = 2 * (g & 1) + (p >> 1);
  lo[0] = toff<W>(row, ch) + 8 * (p & 1);
  hi[0] = toff<W>(row + 4, ch) + 8 * (p & 1);
  lo[1] = toff<W>(row, ch + 4) - 512 + 8 * (p & 1);
  hi[1] = toff<W>(row + 4, ch + 4) - 512 + 8 * (p & 1);
}
// k-major 32x32x16 operand fragment of columns c0 .. c0+31 (c0 % 32 == 0), rows k0 .. k0+15
// (k0 % 16 == 0): lane l holds column c0 + (l & 31), rows k0 + 8(l >> 5) + j -- the gfx950
// transposing LDS read delivers 4 rows of one column per read (two reads per fragment)
// (odd = subtile parity (c0 >> 5) & 1, a compile-time constant at every call site)
template <int W>
__device__ __forceinline__ bf16x8 frag(const char* tile, const int (&lo)[2], const int (&hi)[2], int k0, int c0,
                                       int odd) {
  const int d = (k0 >> 4) * (32 * W) + (c0 >> 5) * 512;
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(tile + lo[odd] + d));
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(tile + hi[odd] + d));
  const v4i16 v[2] = {a, b};
  return *reinterpret_cast<const bf16x8*>(v);
}

template <int BM, int BN, int WM, int WN, int BK>
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64) void wgrad_bf16_k(
    const uint16_t* __restrict__ A, int lda, const uint16_t* __restrict__ B, int ldb, float* __restrict__ out,
    int M, int N, int T, int kchunk, int nsplit, int mvalid) {
  constexpr int NWM = BM / WM, NW = NWM * (BN / WN), NT = NW * 64;
  constexpr int MB = WM / 32, NB = WN / 32;
  constexpr int CA = BK * BM / 8 / NT, CB = BK * BN / 8 / NT;   // 16-B chunks per thread
  static_assert(WM % 64 == 0 && WN % 64 == 0, "subtile parity of fragment a is a & 1");
  static_assert(CA >= 1 && CB >= 1 && BK * BM / 8 % NT == 0 && BK * BN / 8 % NT == 0, "tile / thread mismatch");
  constexpr int A_BYTES = BK * BM * 2, B_BYTES = BK * BN * 2;
  extern __shared__ __attribute__((aligned(16))) char lds[];   // [2] A tiles, then [2] B tiles

  // ---- XCD-aware work index (see header); every lane of the workgroup takes the same exit
  const int TM = M / BM, TN = N / BN, total = TM * TN * nsplit;
  const int per = (total + 7) / 8;   // grid = 8 * per workgroups
  const int work = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (work >= total) return;         // tail of the last XCD's range: no work
  const int nt = work % TN, mt = (work / TN) % TM, sp = work / (TN * TM);
  const int m0 = mt * BM, n0 = nt * BN;
  const int t0 = sp * kchunk, t1 = min(T, t0 + kchunk);
  const int nit = (t1 - t0 + BK - 1) / BK;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w % NWM, wn = w / NWM, h = lane >> 5, l32 = lane & 31;

  // Operand rows [t0, t1) of this split through buffer resources: a load past t1 returns
  // zeros (the tail of the last step and the steps past the end), so loads need no
  // clamping, branches or selects; per-lane 32-bit offsets are loop-invariant and the
  // step only advances the scalar offset.
  const hx::Buf abuf(A + (int64_t)t0 * lda, (uint32_t)((int64_t)(t1 - t0) * lda * 2));
  const hx::Buf bbuf(B + (int64_t)t0 * ldb, (uint32_t)((int64_t)(t1 - t0) * ldb * 2));
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

  // Global tile loads run TWO steps ahead (two register stages): a load issued at the top
  // of step it is written to LDS at the end of step it+1, so its latency hides behind
  // two steps of MFMAs instead of one.
  u32x4 ra0[CA], rb0[CB], ra1[CA], rb1[CB];
  auto load = [&](int it, u32x4 (&ra)[CA], u32x4 (&rb)[CB]) {
    const uint32_t soa = (uint32_t)it * BK * lda * 2, sob = (uint32_t)it * BK * ldb * 2;
#pragma unroll
    for (int i = 0; i < CA; ++i) ra[i] = __builtin_amdgcn_raw_buffer_load_b128(abuf.r, va[i], soa, 0);
#pragma unroll
    for (int i = 0; i < CB; ++i) rb[i] = __builtin_amdgcn_raw_buffer_load_b128(bbuf.r, vb[i], sob, 0);
  };
  auto store = [&](int buf, const u32x4 (&ra)[CA], const u32x4 (&rb)[CB]) {
    char* at = lds + buf * A_BYTES;
    char* bt = lds + 2 * A_BYTES + buf * B_BYTES;
#pragma unroll
    for (int i = 0; i < CA; ++i) *reinterpret_cast<u32x4*>(at + sa[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < CB; ++i) *reinterpret_cast<u32x4*>(bt + sb[i]) = rb[i];
  };

  f32x16 acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = f32x16{0};

  auto mma = [&](int buf) {
    const char* at = lds + buf * A_BYTES;
    const char* bt = lds + 2 * A_BYTES + buf * B_BYTES;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[MB], fb[NB];
#pragma unroll
      for (int a = 0; a < MB; ++a) fa[a] = frag<BM>(at, alo, ahi, 16 * ks, wm * WM + 32 * a, a & 1);
#pragma unroll
      for (int b = 0; b < NB; ++b) fb[b] = frag<BN>(bt, blo, bhi, 16 * ks, wn * WN + 32 * b, b & 1);
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
    }
  };

  load(0, ra0, rb0);
  load(1, ra1, rb1);
  store(0, ra0, rb0);
  __syncthreads();
  // step it computes LDS buffer it&1; register stage it&1 is free (stored a step ago)
  for (int it = 0; it < nit; it += 2) {
    load(it + 2, ra0, rb0);
    mma(0);
    store(1, ra1, rb1);       // step it+1's tile (zeros past the end: harmless)
    __syncthreads();
    if (it + 1 >= nit) break;
    load(it + 3, ra1, rb1);
    mma(1);
    store(0, ra0, rb0);
    __syncthreads();
  }

  // ---- epilogue: rows m (accumulator rows), columns n (lanes): 128-B coalesced fp32 stores;
  // rows from mvalid on (the tile padding of M) are not stored
  float* o = out + (nsplit > 1 ? (int64_t)sp * M * N : 0);
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int n = n0 + wn * WN + 32 * b + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WM + 32 * a + crow(r, h);
        if (m < mvalid) o[(int64_t)m * N + n] = acc[a][b][r];
      }
    }
}

// out[i] = sum_s ws[s][i]  (float4) over the first n4 of each slab of slab4
__global__ __launch_bounds__(256) void split_sum_k(const float4* __restrict__ ws, float4* __restrict__ out, int64_t n4,
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

template <int BM, int BN, int WM, int WN, int BK>
void launch(const uint16_t* A, int lda, const uint16_t* B, int ldb, float* out, float* ws, int M, int N, int T,
            int nsplit, int mvalid, hipStream_t s) {
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  const int kchunk = ((T + nsplit - 1) / nsplit + BK - 1) / BK * BK;
  nsplit = (T + kchunk - 1) / kchunk;   // no empty splits
  const int total = (M / BM) * (N / BN) * nsplit;
  const int per = (total + 7) / 8;
  const size_t smem = 2 * BK * (BM + BN) * sizeof(uint16_t);
  static bool attr = false;
  if (!attr) {   // > 64 KiB of dynamic LDS needs the opt-in (160 KiB per CU on gfx950)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_bf16_k<BM, BN, WM, WN, BK>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr = true;
  }
  wgrad_bf16_k<BM, BN, WM, WN, BK><<<8 * per, NT, smem, s>>>(A, lda, B, ldb, nsplit > 1 ? ws : out, M, N, T, kchunk,
                                                      nsplit, nsplit > 1 ? M : mvalid);
  if (nsplit > 1) {
    const int64_t n4 = (int64_t)mvalid * N / 4, slab4 = (int64_t)M * N / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
    split_sum_k<<<blocks, 256, 0, s>>>(reinterpret_cast<const float4*>(ws), reinterpret_cast<float4*>(out), n4,
                                       slab4, nsplit);
  }
}

}  // namespace

// Tile configurations (cfg index -> BM x BN workgroup tile, waves of 64 x 64, BK tokens per step):
//   0: 128x128, 4 waves, BK 32      1: 256x128, 8 waves, BK 32
//   2: 256x128, 8 waves, BK 64      3: 128x128, 4 waves, BK 64
// (128-wide wave tiles spill at this staging depth: 20-100 TF/s, dropped.)
// HX_WGRAD_CFG="cfg:nsplit" overrides the plan (tuning sweeps: tools/bench_wgrad.py --sweep).
static const int kTileM[4] = {128, 256, 256, 128};
static const int kTileN[4] = {128, 128, 128, 128};
static const int kBK[4] = {32, 32, 64, 64};

void hx_wgrad_bf16_plan(int M, int N, int T, int* cfg, int* nsplit) {
  // One wave of workgroups: the 8-wave 256x128 kernel runs one workgroup per CU (256 slots),
  // the 4-wave 128x128 one two (512 slots).  The split count fills the slots without
  // spilling into a second, mostly empty round (measured on MI355X, T = 16384: FFN dW
  // 3 splits -> 216 workgroups 99 us vs 7 splits -> 504 workgroups 119 us;
  // tools/bench_wgrad.py --sweep).  The 256 x 128 tile takes the 64-token step (half the
  // barriers: FFN dW 98 -> 96 us, QKV 82 -> 79 us at T = 16384, +5-8 % on the pass-stacked
  // rows of the split fp32 path); the 128 x 128 one only on long token ranges.
  const bool big = M % 256 == 0 && N % 128 == 0;
  int c = big ? 2 : (T >= 32768 ? 3 : 0);
  const int slots = (c == 1 || c == 2) ? 256 : 512;
  const int tiles0 = (M / kTileM[c]) * (N / kTileN[c]);
  int s = std::max(1, slots / std::max(1, tiles0));
  s = std::min(s, std::max(1, T / 256));   // at least 256 tokens per split
  if (const char* e = getenv("HX_WGRAD_CFG")) {
    int ec = -1, es = -1;
    if (sscanf(e, "%d:%d", &ec, &es) == 2 && ec >= 0 && ec < 4 && es >= 1 && M % kTileM[ec] == 0 &&
        N % kTileN[ec] == 0) {
      c = ec;
      s = std::min(es, std::max(1, T / kBK[ec]));
    }
  }
  *cfg = c;
  *nsplit = s;
}

void hx_wgrad_bf16(const void* dy, int ldy, const void* x, int ldx, float* out, float* ws, int M, int N, int T,
                   int cfg, int nsplit, int mvalid, hipStream_t s) {
  const uint16_t *a = (const uint16_t*)dy, *b = (const uint16_t*)x;
  switch (cfg) {
    case 1: launch<256, 128, 64, 64, 32>(a, ldy, b, ldx, out, ws, M, N, T, nsplit, mvalid, s); break;
    case 2: launch<256, 128, 64, 64, 64>(a, ldy, b, ldx, out, ws, M, N, T, nsplit, mvalid, s); break;
    case 3: launch<128, 128, 64, 64, 64>(a, ldy, b, ldx, out, ws, M, N, T, nsplit, mvalid, s); break;
    default: launch<128, 128, 64, 64, 32>(a, ldy, b, ldx, out, ws, M, N, T, nsplit, mvalid, s); break;
  }
}
