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
// Used for the forward (A = activation pieces, B = weight pieces [N_out][K_in]) and the data
// gradient (A = output-gradient pieces, B = TRANSPOSED weight pieces [K_in][N_out]) of every
// linear layer; beta = 1 accumulates into C (the fused residual gradient).
//
// Structure (one workgroup per 256 x 128 output tile, 8 waves of 64 x 64):
//  * 32-deep k steps; each distinct piece tile (A: 256 x 32, B: 128 x 32 bf16) is loaded
//    once per step with 16-B buffer loads (rows past M read as zeros), staged two steps
//    ahead in registers and written to LDS as [row][32] with XOR-swizzled 16-B chunks
//    (chunk ^ (row >> 2) & 3: conflict-free 16-B stores and fragment reads);
//  * MFMA 32x32x16 bf16: a fragment is ONE ds_read_b128 (row = lane & 31, 8 consecutive k);
//    per 16-deep k-step a wave reads NPC x (2 A + 2 B) fragments and issues passes x 4
//    MFMAs -- every piece fragment is reused by all passes that use it;
//  * XCD-aware tile order: consecutive workgroup ids go round-robin to the 8 XCDs, so the
//    tile list is cut into 8 contiguous ranges and neighbouring tiles (sharing A rows / B
//    rows) land in one XCD's L2;
//  * epilogue straight from the accumulators (128-B row segments), optional + C.
#include <algorithm>

#include "hx_launch.h"
#include "hx_attn.h"
#include "hx_common.h"

namespace {

using hx::attn::crow;
using hx::attn::f32x16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;

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

// byte offset of 16-B chunk ch (0..3) of row r in a [rows][32] bf16 tile
__device__ __forceinline__ int soff(int r, int ch) { return r * 64 + 16 * (ch ^ ((r >> 2) & 3)); }

template <int BM, int BN, int WM, int WN, int NPC, int NP>
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64) void gemm_split_nt_k(
    const uint16_t* __restrict__ A, int64_t lda, int64_t a_ps, const uint16_t* __restrict__ B, int64_t ldb,
    int64_t b_ps, float* __restrict__ C, int64_t ldc, int M, int N, int K, int beta) {
  constexpr int NWM = BM / WM, NW = NWM * (BN / WN), NT = NW * 64;
  constexpr int MB = WM / 32, NB = WN / 32;
  constexpr int CA = BM * 4 / NT, CB = BN * 4 / NT;   // 16-B chunks per thread per piece per k step
  static_assert(CA >= 1 && CB >= 1 && BM * 4 % NT == 0 && BN * 4 % NT == 0, "tile / thread mismatch");
  constexpr int A_BYTES = BM * 64, B_BYTES = BN * 64;
  constexpr int STAGE = NPC * (A_BYTES + B_BYTES);
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int TM = (M + BM - 1) / BM, TN = N / BN, total = TM * TN;
  const int per = (total + 7) / 8;
  const int work = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (work >= total) return;   // uniform per workgroup
  const int nt = work % TN, mt = work / TN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nit = K / BK;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w % NWM, wn = w / NWM, h = lane >> 5, l32 = lane & 31;

  // buffer resources over this tile's rows: A rows past M read as zeros
  const int mrows = min(BM, M - m0);
  const hx::Buf abuf(A + (int64_t)m0 * lda, (uint32_t)((int64_t)(mrows - 1) * lda * 2 + (NPC - 1) * a_ps * 2 + K * 2));
  const hx::Buf bbuf(B + (int64_t)n0 * ldb, (uint32_t)((int64_t)(BN - 1) * ldb * 2 + (NPC - 1) * b_ps * 2 + K * 2));
  uint32_t va[CA], vb[CB];
  int sa[CA], sb[CB];
#pragma unroll
  for (int i = 0; i < CA; ++i) {
    const int e = tid + i * NT, row = e >> 2, ch = e & 3;
    va[i] = row < mrows ? (uint32_t)(row * lda + 8 * ch) * 2 : 0x80000000u;   // out of range -> zeros
    sa[i] = soff(row, ch);
  }
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    const int e = tid + i * NT, row = e >> 2, ch = e & 3;
    vb[i] = (uint32_t)(row * ldb + 8 * ch) * 2;
    sb[i] = soff(row, ch);
  }

  u32x4 ra0[NPC][CA], rb0[NPC][CB], ra1[NPC][CA], rb1[NPC][CB];
  auto load = [&](int it, u32x4 (&ra)[NPC][CA], u32x4 (&rb)[NPC][CB]) {
    if (it >= nit) return;
    const uint32_t ko = (uint32_t)it * BK * 2;
#pragma unroll
    for (int p = 0; p < NPC; ++p) {
#pragma unroll
      for (int i = 0; i < CA; ++i)
        ra[p][i] = __builtin_amdgcn_raw_buffer_load_b128(abuf.r, va[i], ko + (uint32_t)(p * a_ps * 2), 0);
#pragma unroll
      for (int i = 0; i < CB; ++i)
        rb[p][i] = __builtin_amdgcn_raw_buffer_load_b128(bbuf.r, vb[i], ko + (uint32_t)(p * b_ps * 2), 0);
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

  // fragment of rows r0 + (lane & 31), k = 16 ks + 8 h .. + 7: one 16-B LDS read
  auto frag = [&](const char* tile, int r0, int ks) -> bf16x8 {
    const int r = r0 + l32;
    return *reinterpret_cast<const bf16x8*>(tile + soff(r, 2 * ks + h));
  };
  auto mma = [&](int buf) {
    const char* st = lds + buf * STAGE;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[NPC][MB], fb[NPC][NB];
#pragma unroll
      for (int p = 0; p < NPC; ++p) {
#pragma unroll
        for (int a = 0; a < MB; ++a) fa[p][a] = frag(st + p * A_BYTES, wm * WM + 32 * a, ks);
#pragma unroll
        for (int b = 0; b < NB; ++b) fb[p][b] = frag(st + NPC * A_BYTES + p * B_BYTES, wn * WN + 32 * b, ks);
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

  load(0, ra0, rb0);
  load(1, ra1, rb1);
  store(0, ra0, rb0);
  __syncthreads();
  for (int it = 0; it < nit; it += 2) {
    load(it + 2, ra0, rb0);
    mma(0);
    if (it + 1 >= nit) break;
    store(1, ra1, rb1);
    __syncthreads();
    load(it + 3, ra1, rb1);
    mma(1);
    if (it + 2 >= nit) break;
    store(0, ra0, rb0);
    __syncthreads();
  }

  // epilogue: accumulator register r of lane (h, l32) = row crow(r, h), column l32
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int n = n0 + wn * WN + 32 * b + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WM + 32 * a + crow(r, h);
        if (m < M) {
          float* dst = C + (int64_t)m * ldc + n;
          *dst = beta ? *dst + acc[a][b][r] : acc[a][b][r];
        }
      }
    }
}

template <int BM, int BN, int WM, int WN, int NPC, int NP>
void launch(const uint16_t* A, int64_t lda, int64_t a_ps, const uint16_t* B, int64_t ldb, int64_t b_ps, float* C,
            int64_t ldc, int M, int N, int K, int beta, hipStream_t s) {
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  const int total = ((M + BM - 1) / BM) * (N / BN);
  const int per = (total + 7) / 8;
  const size_t smem = 2 * (size_t)NPC * (BM + BN) * BK * sizeof(uint16_t);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_split_nt_k<BM, BN, WM, WN, NPC, NP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr = true;
  }
  gemm_split_nt_k<BM, BN, WM, WN, NPC, NP><<<8 * per, NT, smem, s>>>(A, lda, a_ps, B, ldb, b_ps, C, ldc, M, N, K,
                                                                    beta);
}

}  // namespace

int hx_gemm_split_nt(const void* A, int64_t lda, int64_t a_ps, const void* B, int64_t ldb, int64_t b_ps, float* C,
                     int64_t ldc, int M, int N, int K, int passes, int beta, hipStream_t s) {
  if (N % 128 || K % BK || M < 1) return -1;
  const uint16_t *a = (const uint16_t*)A, *b = (const uint16_t*)B;
  if (passes == 3)
    launch<256, 128, 64, 64, 2, 3>(a, lda, a_ps, b, ldb, b_ps, C, ldc, M, N, K, beta, s);
  else if (passes == 6)
    launch<256, 128, 64, 64, 3, 6>(a, lda, a_ps, b, ldb, b_ps, C, ldc, M, N, K, beta, s);
  else
    return -1;
  return 0;
}
