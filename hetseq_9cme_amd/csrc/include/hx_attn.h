// Pieces shared by the fp32-MFMA (attention.hip) and bf16-MFMA (attention_bf16.hip)
// fused attention kernels: the 32x32 accumulator row map and the forward dropout
// step that applies the Philox decisions and builds the transposed bitmask word.
#pragma once
#include "hx_common.h"

namespace hx {
namespace attn {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// accumulator register r of a 32x32 MFMA tile (32x32x2 f32 and 32x32x16 bf16 alike),
// lane half h -> row index
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// v_writelane_b32 with a compile-time lane: put a wave-uniform value into one lane of a
// VGPR.  Through the LLVM intrinsic (this clang has no builtin for it), not an asm block:
// the compiler must see the instruction to put the wait states gfx950 needs between the
// VALU write of the ballot SGPR and this read of it -- an asm block hid it, and some
// lanes' words were lost depending on the schedule.
extern "C" __device__ int hx_llvm_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane");
template <int L>
__device__ __forceinline__ uint32_t write_lane(uint32_t v, uint32_t val) {
  return (uint32_t)hx_llvm_writelane((int)val, L, (int)v);
}

// Forward dropout for accumulator register R of both 32-key sub-blocks (keys on the
// accumulator rows, queries on the lanes): apply the lane's decisions, and build the
// transposed bitmask word: a ballot over the wave gives, for register R, the
// 32-query words of keys crow(R,0) (lanes 0-31) and crow(R,1) (lanes 32-63); lane L
// collects the word of key kt + L.  Decision bits: kb[R>>3] (keys 0-31) and
// kb[2 + (R>>3)] (keys 32-63), bit R&7 -- 8 decisions per Philox call.
template <int R>
__device__ __forceinline__ void drop_step(f32x16& s0, f32x16& s1, const uint32_t (&kb)[4], float inv_keep,
                                          uint32_t& myword) {
  if constexpr (R < 16) {
    const bool k0 = (kb[R >> 3] >> (R & 7)) & 1, k1 = (kb[2 + (R >> 3)] >> (R & 7)) & 1;
    s0[R] = k0 ? s0[R] * inv_keep : 0.f;
    s1[R] = k1 ? s1[R] * inv_keep : 0.f;
    const uint64_t b0 = __ballot(k0), b1 = __ballot(k1);
    constexpr int L0 = (R & 3) + 8 * (R >> 2);
    myword = write_lane<L0>(myword, (uint32_t)b0);
    myword = write_lane<L0 + 4>(myword, (uint32_t)(b0 >> 32));
    myword = write_lane<32 + L0>(myword, (uint32_t)b1);
    myword = write_lane<36 + L0>(myword, (uint32_t)(b1 >> 32));
    if constexpr ((R & 3) == 3) __builtin_amdgcn_sched_barrier(0);   // keep ballots from piling up in SGPRs
    drop_step<R + 1>(s0, s1, kb, inv_keep, myword);
  }
}

// Philox counter of (query q, 64-key tile kt, lane half h): 4 calls x 8 decisions
// cover the 64 keys of the tile for one query.  Shared by both kernels so the
// dropout pattern does not depend on the activation precision.
__device__ __forceinline__ uint64_t drop_counter(int64_t bh, int S, int q, int Sp, int kt, int h) {
  return (((uint64_t)(bh * S + q) * (uint64_t)(Sp >> 6) + (kt >> 6)) * 2 + h) * 4;
}

}  // namespace attn
}  // namespace hx
