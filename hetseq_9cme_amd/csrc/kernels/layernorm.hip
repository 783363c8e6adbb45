// Fused (bias + dropout + residual + LayerNorm) forward / backward and the fused
// BERT embedding (3 gathers + sum + LayerNorm + dropout).
//
// Reference sites (all TF-style LN, eps inside the sqrt, bert_modeling.py:276-289):
//   BertSelfOutput / BertOutput  : LN(dropout(dense(h) + b) + residual)  (:387-391, :423-427)
//   BertPredictionHeadTransform  : LN(gelu(dense(h) + b))                 (:526-527)
//   BertEmbeddings               : dropout(LN(word[id] + pos[s] + type[tt])) (:306-320)
// The reference issues ~8 elementwise/reduction kernels per LN forward and ~15 in
// autograd backward; here each is ONE row-per-wave kernel:
//   * a wave64 owns a row; H = CH*256 columns are held in registers as CH float4 per
//     lane (H=768 -> 3 x 16 B per lane), so the row is read once and written once;
//   * dropout masks come from Philox(seed, stream, element) and are regenerated in
//     backward (nothing stored);
//   * backward produces dz (= d residual), dy (= d dense-output), and per-block
//     column partials of dgamma / dbeta / dbias that a second kernel folds; rows are
//     grid-strided over a bounded number of workgroups so the partial slab stays small.
// Activations may be fp32 or bf16 (T); statistics and affine params are fp32.
#include "hx_gemm.h"
#include "hx_launch.h"
#include "hx_vec.h"
#include "hx_reduce.h"

namespace {

constexpr int NT = 256;             // 4 waves
constexpr int WPB = NT / 64;

template <int CH>
struct Row {
  float4 v[CH];
};

// max |x| of the wave's row -> amax_row[r] (the fp16x3 GEMMs' per-row operand scale, ops/gemm16.py)
__device__ __forceinline__ float row_amax_out(float m, float* __restrict__ amax_row, int64_t r) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (amax_row && (threadIdx.x & 63) == 0) amax_row[r] = m;
  return m;
}
// the row's fp16 P2 pieces at its own scale (row max m): the A operand of the consumer GEMM,
// already split (gemm_f16.hip AT 2), [rows][2H]
template <int CH>
__device__ __forceinline__ void row_pieces_out(const Row<CH>& v, float m, uint16_t* __restrict__ pieces, int64_t r,
                                               int H) {
  const float sc = ldexpf(1.f, hx::g::f16_scale_exp(m));
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int j = (c * 64 + lane) * 4;
    if (j < H) hx::g::store_p2x4(pieces + r * 2 * H, j, v.v[c], sc);
  }
}
__device__ __forceinline__ float amax4(float m, float4 v) {
  return fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
}

// ----------------------------------------------------------------------------- fwd
template <typename T, int CH, bool kDropAfter>
__global__ __launch_bounds__(NT) void ln_fwd_k(const T* __restrict__ y, const float* __restrict__ bias,
                                             const T* __restrict__ res, const float* __restrict__ gamma,
                                             const float* __restrict__ beta, T* __restrict__ out,
                                             T* __restrict__ zsave, float* __restrict__ mean_out,
                                             float* __restrict__ rstd_out, int64_t rows, int H, float eps,
                                             float keep_prob, const uint64_t* __restrict__ seedp, uint64_t stream,
                                             float* __restrict__ amax_part, uint16_t* __restrict__ pieces) {
  const uint64_t seed = *seedp;   // per-update Philox key, device-resident (graph-safe)
  const int lane = threadIdx.x & 63;
  const int64_t wave = blockIdx.x * (int64_t)WPB + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * WPB;
  const float inv_keep = keep_prob > 0.f ? 1.f / keep_prob : 0.f;
  const bool drop = keep_prob < 1.f;
  // one row of look-ahead (grid-strided launches): the next row's y / res loads are in flight
  // while this row reduces and stores
  Row<CH> yn, qn;
  auto load_row = [&](int64_t r) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      if (j < H) {
        yn.v[c] = hx::load4(y + r * H + j);
        if (res) qn.v[c] = hx::load4(res + r * H + j);
      }
    }
  };
  if (wave < rows) load_row(wave);
  for (int64_t r = wave; r < rows; r += nw) {
    float am = 0.f;
    Row<CH> x;
    const Row<CH> yc = yn, qc = qn;
    if (r + nw < rows) load_row(r + nw);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      float4 v = hx::f4(0.f);
      if (j < H) {
        v = yc.v[c];
        if (bias) {
          const float4 b = *reinterpret_cast<const float4*>(bias + j);
          v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
        }
        if (drop && !kDropAfter) {
          const uint32_t k = hx::keep4(seed, stream, (uint64_t)(r * H + j) >> 2, keep_prob);
          v.x = (k & 1) ? v.x * inv_keep : 0.f;
          v.y = (k & 2) ? v.y * inv_keep : 0.f;
          v.z = (k & 4) ? v.z * inv_keep : 0.f;
          v.w = (k & 8) ? v.w * inv_keep : 0.f;
        }
        if (res) {
          const float4 q = qc.v[c];
          v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
        }
        if (zsave) hx::store4(zsave + r * H + j, v);
      }
      x.v[c] = v;
      s += v.x + v.y + v.z + v.w;
    }
    const float mean = hx::wave_sum(s) / H;
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      if (j < H) {
        const float4 v = x.v[c];
        const float a = v.x - mean, b = v.y - mean, cc = v.z - mean, d = v.w - mean;
        ss += a * a + b * b + cc * cc + d * d;
      }
    }
    const float var = hx::wave_sum(ss) / H;
    const float rstd = 1.0f / sqrtf(var + eps);
    if (lane == 0) {
      mean_out[r] = mean;
      rstd_out[r] = rstd;
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      if (j < H) {
        const float4 g = *reinterpret_cast<const float4*>(gamma + j);
        const float4 b = *reinterpret_cast<const float4*>(beta + j);
        const float4 v = x.v[c];
        float4 o = make_float4(g.x * ((v.x - mean) * rstd) + b.x, g.y * ((v.y - mean) * rstd) + b.y,
                               g.z * ((v.z - mean) * rstd) + b.z, g.w * ((v.w - mean) * rstd) + b.w);
        if (drop && kDropAfter) {
          const uint32_t k = hx::keep4(seed, stream, (uint64_t)(r * H + j) >> 2, keep_prob);
          o.x = (k & 1) ? o.x * inv_keep : 0.f;
          o.y = (k & 2) ? o.y * inv_keep : 0.f;
          o.z = (k & 4) ? o.z * inv_keep : 0.f;
          o.w = (k & 8) ? o.w * inv_keep : 0.f;
        }
        hx::store4(out + r * H + j, o);
        am = amax4(am, o);
        x.v[c] = o;
      }
    }
    if (pieces) row_pieces_out(x, row_amax_out(am, amax_part, r), pieces, r, H);
    else if (amax_part) row_amax_out(am, amax_part, r);
  }
}

// ----------------------------------------------------------------------------- bwd
// dout -> (optional dropout-after inverse) -> LN backward -> dz ; dy = dz*mask/keep
// partial[blk][0:H)=dgamma, [H:2H)=dbeta, [2H:3H)=dbias(dy)
template <typename T, int CH, bool kDropAfter>
__global__ __launch_bounds__(NT) void ln_bwd_k(const T* __restrict__ dout, const T* __restrict__ z,
                                             const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                             const float* __restrict__ gamma, T* __restrict__ dz_out,
                                             T* __restrict__ dy_out, float* __restrict__ partial, int64_t rows,
                                             int H, float keep_prob, const uint64_t* __restrict__ seedp, uint64_t stream,
                                             int want_dbias, float* __restrict__ amax_part, int want_cmax,
                                             uint16_t* __restrict__ pieces) {
  const uint64_t seed = *seedp;   // per-update Philox key, device-resident (graph-safe)
  __shared__ float red[WPB][CH * 256];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t wave = blockIdx.x * (int64_t)WPB + w;
  const int64_t nw = (int64_t)gridDim.x * WPB;
  const float inv_keep = keep_prob > 0.f ? 1.f / keep_prob : 0.f;
  const bool drop = keep_prob < 1.f;
  Row<CH> dg, db, dbias, cmx;   // cmx: column max |dy| (|dz| without dy), the weight gradient's scale
#pragma unroll
  for (int c = 0; c < CH; ++c) dg.v[c] = db.v[c] = dbias.v[c] = cmx.v[c] = hx::f4(0.f);
  float4 gam[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int j = (c * 64 + lane) * 4;
    gam[c] = j < H ? *reinterpret_cast<const float4*>(gamma + j) : hx::f4(0.f);
  }

  // one row of look-ahead: the next row's loads are in flight while this row computes
  Row<CH> zn, dn;
  float mn = 0.f, rn = 0.f;
  auto load_row = [&](int64_t r) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      if (j < H) {
        zn.v[c] = hx::load4(z + r * H + j);
        dn.v[c] = hx::load4(dout + r * H + j);
      }
    }
    mn = mean_in[r];
    rn = rstd_in[r];
  };
  if (wave < rows) load_row(wave);

  for (int64_t r = wave; r < rows; r += nw) {
    const Row<CH> zc = zn, dc = dn;
    const float mean = mn, rstd = rn;
    float am = 0.f;   // max |dy| (max |dz| without a separate dy): the upstream GEMMs' row scale
    if (r + nw < rows) load_row(r + nw);
    Row<CH> xh, dxh;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      float4 xv = hx::f4(0.f), dv = hx::f4(0.f);
      if (j < H) {
        const float4 zz = zc.v[c];
        float4 d = dc.v[c];
        if (drop && kDropAfter) {
          const uint32_t k = hx::keep4(seed, stream, (uint64_t)(r * H + j) >> 2, keep_prob);
          d.x = (k & 1) ? d.x * inv_keep : 0.f;
          d.y = (k & 2) ? d.y * inv_keep : 0.f;
          d.z = (k & 4) ? d.z * inv_keep : 0.f;
          d.w = (k & 8) ? d.w * inv_keep : 0.f;
        }
        const float4 g = gam[c];
        xv = make_float4((zz.x - mean) * rstd, (zz.y - mean) * rstd, (zz.z - mean) * rstd, (zz.w - mean) * rstd);
        dv = make_float4(d.x * g.x, d.y * g.y, d.z * g.z, d.w * g.w);
        dg.v[c].x += d.x * xv.x; dg.v[c].y += d.y * xv.y; dg.v[c].z += d.z * xv.z; dg.v[c].w += d.w * xv.w;
        db.v[c].x += d.x; db.v[c].y += d.y; db.v[c].z += d.z; db.v[c].w += d.w;
        s1 += dv.x + dv.y + dv.z + dv.w;
        s2 += dv.x * xv.x + dv.y * xv.y + dv.z * xv.z + dv.w * xv.w;
      }
      xh.v[c] = xv;
      dxh.v[c] = dv;
    }
    const float m1 = hx::wave_sum(s1) / H;
    const float m2 = hx::wave_sum(s2) / H;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      if (j < H) {
        const float4 xv = xh.v[c], dv = dxh.v[c];
        float4 dz = make_float4(rstd * (dv.x - m1 - xv.x * m2), rstd * (dv.y - m1 - xv.y * m2),
                                rstd * (dv.z - m1 - xv.z * m2), rstd * (dv.w - m1 - xv.w * m2));
        hx::store4(dz_out + r * H + j, dz);
        xh.v[c] = dz;   // the consumer GEMM's operand (dy below when separate): its pieces
        if (!dy_out) {
          am = amax4(am, dz);
          if (want_cmax) cmx.v[c] = hx::max4(cmx.v[c], hx::abs4(dz));
        }
        if (dy_out) {
          float4 dy = dz;
          if (drop && !kDropAfter) {
            const uint32_t k = hx::keep4(seed, stream, (uint64_t)(r * H + j) >> 2, keep_prob);
            dy.x = (k & 1) ? dy.x * inv_keep : 0.f;
            dy.y = (k & 2) ? dy.y * inv_keep : 0.f;
            dy.z = (k & 4) ? dy.z * inv_keep : 0.f;
            dy.w = (k & 8) ? dy.w * inv_keep : 0.f;
          }
          hx::store4(dy_out + r * H + j, dy);
          xh.v[c] = dy;
          am = amax4(am, dy);
          if (want_cmax) cmx.v[c] = hx::max4(cmx.v[c], hx::abs4(dy));
          if (want_dbias) {
            dbias.v[c].x += dy.x; dbias.v[c].y += dy.y; dbias.v[c].z += dy.z; dbias.v[c].w += dy.w;
          }
        }
      }
    }
    if (pieces) row_pieces_out(xh, row_amax_out(am, amax_part, r), pieces, r, H);
    else if (amax_part) row_amax_out(am, amax_part, r);
  }
  // fold the 4 waves' column partials through LDS (each accumulator selected at
  // compile time: a runtime-selected reference would demote them to scratch)
  auto fold = [&](const Row<CH>& src, int q) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      *reinterpret_cast<float4*>(&red[w][j]) = src.v[c];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < H; j += NT) {
      float a = 0.f;
#pragma unroll
      for (int ww = 0; ww < WPB; ++ww) a = q == 3 ? fmaxf(a, red[ww][j]) : a + red[ww][j];
      partial[((int64_t)blockIdx.x * 4 + q) * H + j] = a;
    }
    __syncthreads();
  };
  fold(dg, 0);
  fold(db, 1);
  if (want_dbias) fold(dbias, 2);
  if (want_cmax) fold(cmx, 3);
}

// ------------------------------------------------------------------------ embedding
template <typename T, int CH>
__global__ __launch_bounds__(NT) void embed_ln_fwd_k(const int64_t* __restrict__ ids, const int64_t* __restrict__ tt,
                                                   const float* __restrict__ wte, const float* __restrict__ wpe,
                                                   const float* __restrict__ wtt, const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, T* __restrict__ out,
                                                   T* __restrict__ zsave, float* __restrict__ mean_out,
                                                   float* __restrict__ rstd_out, int64_t rows, int S, int H,
                                                   float eps, float keep_prob, const uint64_t* __restrict__ seedp, uint64_t stream,
                                                   float* __restrict__ amax_part, uint16_t* __restrict__ pieces) {
  const uint64_t seed = *seedp;   // per-update Philox key, device-resident (graph-safe)
  const int lane = threadIdx.x & 63;
  const int64_t wave = blockIdx.x * (int64_t)WPB + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * WPB;
  const float inv_keep = keep_prob > 0.f ? 1.f / keep_prob : 0.f;
  for (int64_t r = wave; r < rows; r += nw) {
    float am = 0.f;
    const int64_t id = ids[r];
    const int64_t ty = tt ? tt[r] : 0;
    const int64_t pos = r % S;
    Row<CH> x;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      float4 v = hx::f4(0.f);
      if (j < H) {
        const float4 a = *reinterpret_cast<const float4*>(wte + id * H + j);
        const float4 b = *reinterpret_cast<const float4*>(wpe + pos * H + j);
        const float4 d = *reinterpret_cast<const float4*>(wtt + ty * H + j);
        v = make_float4(a.x + b.x + d.x, a.y + b.y + d.y, a.z + b.z + d.z, a.w + b.w + d.w);
        hx::store4(zsave + r * H + j, v);
      }
      x.v[c] = v;
      s += v.x + v.y + v.z + v.w;
    }
    const float mean = hx::wave_sum(s) / H;
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      if (j < H) {
        const float4 v = x.v[c];
        const float a = v.x - mean, b = v.y - mean, cc = v.z - mean, d = v.w - mean;
        ss += a * a + b * b + cc * cc + d * d;
      }
    }
    const float rstd = 1.0f / sqrtf(hx::wave_sum(ss) / H + eps);
    if (lane == 0) {
      mean_out[r] = mean;
      rstd_out[r] = rstd;
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      if (j < H) {
        const float4 g = *reinterpret_cast<const float4*>(gamma + j);
        const float4 b = *reinterpret_cast<const float4*>(beta + j);
        const float4 v = x.v[c];
        float4 o = make_float4(g.x * ((v.x - mean) * rstd) + b.x, g.y * ((v.y - mean) * rstd) + b.y,
                               g.z * ((v.z - mean) * rstd) + b.z, g.w * ((v.w - mean) * rstd) + b.w);
        if (keep_prob < 1.f) {
          const uint32_t k = hx::keep4(seed, stream, (uint64_t)(r * H + j) >> 2, keep_prob);
          o.x = (k & 1) ? o.x * inv_keep : 0.f;
          o.y = (k & 2) ? o.y * inv_keep : 0.f;
          o.z = (k & 4) ? o.z * inv_keep : 0.f;
          o.w = (k & 8) ? o.w * inv_keep : 0.f;
        }
        hx::store4(out + r * H + j, o);
        am = amax4(am, o);
        x.v[c] = o;
      }
    }
    // (fp32 runs) the first layer's QKV GEMM operand, pre-split at the row scale (ln_fwd_k's pieces)
    if (pieces) row_pieces_out(x, row_amax_out(am, amax_part, r), pieces, r, H);
    else if (amax_part) row_amax_out(am, amax_part, r);
  }
}

// word-embedding gradient: scatter-add rows of dz into dW[ids] (fp32 atomics,
// whole 16-B contiguous lane groups -> 256 contiguous bytes per wave instruction).

// position + token-type gradients: block (s-tile) reduces over the batch dim.
// dpos[s][j] = sum_b dz[b,s,j] ; dtype[t][j] += sum over rows with tt==t (atomics per block)
// Word-embedding gradient from rows visited in id-sorted order (order = argsort(ids)).
// Wave w owns sorted positions [w*kSegRows, (w+1)*kSegRows) (8 rows: 2048 waves at
// B*S = 16384 keep every CU busy): it sums each run of
// equal ids in registers and writes the run once.  A run that may continue into a
// neighbouring wave's chunk (the chunk's first and last run) is added atomically;
// every interior run's id occurs nowhere else, so a plain read-add-write is exact.
// Frequent ids ([CLS], [SEP], [MASK], "the" in real text) thus cost a handful of
// atomics per element instead of one per occurrence.
constexpr int kSegRows = 8;
template <typename T, int CH>
__global__ __launch_bounds__(NT) void embed_word_grad_sorted_k(const T* __restrict__ dz,
                                                             const int64_t* __restrict__ ids,
                                                             const int64_t* __restrict__ order,
                                                             float* __restrict__ dw, int64_t rows, int H) {
  const int lane = threadIdx.x & 63;
  const int64_t seg = blockIdx.x * (int64_t)WPB + (threadIdx.x >> 6);
  const int64_t p0 = seg * kSegRows;
  if (p0 >= rows) return;
  const int64_t p1 = p0 + kSegRows < rows ? p0 + kSegRows : rows;
  float4 acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = hx::f4(0.f);
  // the chunk's (row, id) pairs: one per lane, loaded in parallel, then broadcast
  const int cnt = (int)(p1 - p0);
  const int64_t myr = lane < cnt ? order[p0 + lane] : 0;
  const int64_t myid = lane < cnt ? ids[myr] : -1;
  int64_t cur = __shfl(myid, 0, 64);
  bool first_run = true;
  auto flush = [&](int64_t id, bool atomic) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      if (j < H) {
        float* d = dw + id * H + j;
        if (atomic) {
          atomicAdd(d, acc[c].x); atomicAdd(d + 1, acc[c].y); atomicAdd(d + 2, acc[c].z); atomicAdd(d + 3, acc[c].w);
        } else {
          float4 o = *reinterpret_cast<float4*>(d);
          o.x += acc[c].x; o.y += acc[c].y; o.z += acc[c].z; o.w += acc[c].w;
          *reinterpret_cast<float4*>(d) = o;
        }
      }
      acc[c] = hx::f4(0.f);
    }
  };
  for (int k = 0; k < cnt; ++k) {
    const int64_t r = __shfl(myr, k, 64);
    const int64_t id = __shfl(myid, k, 64);
    if (id != cur) {
      flush(cur, first_run);
      first_run = false;
      cur = id;
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      if (j < H) {
        const float4 v = hx::load4(dz + r * H + j);
        acc[c].x += v.x; acc[c].y += v.y; acc[c].z += v.z; acc[c].w += v.w;
      }
    }
  }
  flush(cur, true);   // the last run may continue in the next chunk
}

// token-type embedding gradient (few types): part[block][t][H] = sum of the block's rows r with
// tt[r] == t, a wave per row as the LayerNorm kernels (the row read once), the 4 waves' sums folded
// through LDS; fold_rows sums the blocks.  Replaces one_hot(tt)^T . dz (a one-hot tensor and a
// [NT x rows] x [rows x H] library GEMM: 32 us fp32, 73 us bf16 at 16384 x 768).
template <typename T, int CH, int NTY>
__global__ __launch_bounds__(NT) void type_grad_k(const T* __restrict__ dz, const int64_t* __restrict__ tt,
                                                  float* __restrict__ part, int64_t rows, int H) {
  __shared__ float red[WPB][CH * 256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t nw = (int64_t)gridDim.x * WPB;
  Row<CH> acc[NTY];
#pragma unroll
  for (int t = 0; t < NTY; ++t)
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[t].v[c] = hx::f4(0.f);
  for (int64_t r = blockIdx.x * (int64_t)WPB + w; r < rows; r += nw) {
    const int ty = (int)tt[r];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int j = (c * 64 + lane) * 4;
      if (j < H) {
        const float4 v = hx::load4(dz + r * H + j);
#pragma unroll
        for (int t = 0; t < NTY; ++t)
          if (ty == t) {
            acc[t].v[c].x += v.x; acc[t].v[c].y += v.y; acc[t].v[c].z += v.z; acc[t].v[c].w += v.w;
          }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NTY; ++t) {
#pragma unroll
    for (int c = 0; c < CH; ++c) *reinterpret_cast<float4*>(&red[w][(c * 64 + lane) * 4]) = acc[t].v[c];
    __syncthreads();
    for (int j = threadIdx.x; j < H; j += NT)
      part[((int64_t)blockIdx.x * NTY + t) * H + j] = (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]);
    __syncthreads();
  }
}

int pick_ch(int H) {
  const int c = (H + 255) / 256;
  if (c <= 1) return 1;
  if (c <= 2) return 2;
  if (c <= 3) return 3;
  if (c <= 4) return 4;
  return 8;
}

inline int ln_grid(int64_t rows, int cap) {
  int64_t g = (rows + WPB - 1) / WPB;
  return (int)(g < cap ? (g < 1 ? 1 : g) : cap);
}

#define HX_CH_DISPATCH(H, ...)          \
  switch (pick_ch(H)) {                 \
    case 1: { constexpr int CH = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int CH = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int CH = 3; __VA_ARGS__; } break; \
    case 4: { constexpr int CH = 4; __VA_ARGS__; } break; \
    default: { constexpr int CH = 8; __VA_ARGS__; } break; \
  }

template <typename T>
void ln_fwd_t(const void* y, const float* bias, const void* res, const float* gamma, const float* beta, void* out,
              void* zsave, float* mean, float* rstd, int64_t rows, int H, float eps, float keep_prob, const uint64_t* seed,
              uint64_t stream, int drop_after, hipStream_t s, float* amax_part, uint16_t* pieces) {
  const int grid = hx_ln_fwd_blocks(rows);
  HX_CH_DISPATCH(H, {
    if (drop_after)
      ln_fwd_k<T, CH, true><<<grid, NT, 0, s>>>((const T*)y, bias, (const T*)res, gamma, beta, (T*)out, (T*)zsave,
                                                mean, rstd, rows, H, eps, keep_prob, seed, stream, amax_part, pieces);
    else
      ln_fwd_k<T, CH, false><<<grid, NT, 0, s>>>((const T*)y, bias, (const T*)res, gamma, beta, (T*)out, (T*)zsave,
                                                 mean, rstd, rows, H, eps, keep_prob, seed, stream, amax_part, pieces);
  })
}

template <typename T>
void ln_bwd_t(const void* dout, const void* z, const float* mean, const float* rstd, const float* gamma, void* dz,
              void* dy, float* partial, int nblk, int64_t rows, int H, float keep_prob, const uint64_t* seed,
              uint64_t stream, int drop_after, int want_dbias, float* dgamma, float* dbeta, float* dbias,
              int accumulate, hipStream_t s, float* amax_part, float* colmax, uint16_t* pieces) {
  const int wc = colmax != nullptr;
  HX_CH_DISPATCH(H, {
    if (drop_after)
      ln_bwd_k<T, CH, true><<<nblk, NT, 0, s>>>((const T*)dout, (const T*)z, mean, rstd, gamma, (T*)dz, (T*)dy,
                                                partial, rows, H, keep_prob, seed, stream, want_dbias, amax_part, wc,
                                                pieces);
    else
      ln_bwd_k<T, CH, false><<<nblk, NT, 0, s>>>((const T*)dout, (const T*)z, mean, rstd, gamma, (T*)dz, (T*)dy,
                                                 partial, rows, H, keep_prob, seed, stream, want_dbias, amax_part, wc,
                                                 pieces);
  })
  // partial is [nblk][4][H]: fold rows of length 4H into dgamma | dbeta | dbias (sums) and the
  // column maxima (max)
  hx::fold_rows(partial, nblk, 4 * (int64_t)H, wc ? 4 * H : (want_dbias ? 3 : 2) * H, H, dgamma, dbeta,
                want_dbias ? dbias : nullptr, accumulate, s, 3 * H, colmax);
}

}  // namespace

namespace {
int env_cap(const char* name, int dflt) {
  const char* e = getenv(name);
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : dflt;
}
}  // namespace

int hx_ln_bwd_blocks(int64_t rows) { return ln_grid(rows, env_cap("HX_LN_BWD_CAP", 512)); }
int hx_ln_fwd_blocks(int64_t rows) { return ln_grid(rows, env_cap("HX_LN_FWD_CAP", 4096)); }

void hx_ln_fwd(int bf16, const void* y, const float* bias, const void* res, const float* gamma, const float* beta,
               void* out, void* zsave, float* mean, float* rstd, int64_t rows, int H, float eps, float keep_prob,
               const uint64_t* seed, uint64_t stream, int drop_after, hipStream_t s, float* amax_part,
               uint16_t* pieces) {
  if (bf16)
    ln_fwd_t<uint16_t>(y, bias, res, gamma, beta, out, zsave, mean, rstd, rows, H, eps, keep_prob, seed, stream,
                       drop_after, s, nullptr, nullptr);
  else
    ln_fwd_t<float>(y, bias, res, gamma, beta, out, zsave, mean, rstd, rows, H, eps, keep_prob, seed, stream,
                    drop_after, s, amax_part, pieces);
}

void hx_ln_bwd(int bf16, const void* dout, const void* z, const float* mean, const float* rstd, const float* gamma,
               void* dz, void* dy, float* partial, int nblk, int64_t rows, int H, float keep_prob, const uint64_t* seed,
               uint64_t stream, int drop_after, int want_dbias, float* dgamma, float* dbeta, float* dbias,
               int accumulate, hipStream_t s, float* amax_part, float* colmax, uint16_t* pieces) {
  if (bf16)
    ln_bwd_t<uint16_t>(dout, z, mean, rstd, gamma, dz, dy, partial, nblk, rows, H, keep_prob, seed, stream,
                       drop_after, want_dbias, dgamma, dbeta, dbias, accumulate, s, nullptr, nullptr, nullptr);
  else
    ln_bwd_t<float>(dout, z, mean, rstd, gamma, dz, dy, partial, nblk, rows, H, keep_prob, seed, stream, drop_after,
                    want_dbias, dgamma, dbeta, dbias, accumulate, s, amax_part, colmax, pieces);
}

void hx_embed_ln_fwd(int bf16, const int64_t* ids, const int64_t* tt, const float* wte, const float* wpe,
                     const float* wtt, const float* gamma, const float* beta, void* out, void* zsave, float* mean,
                     float* rstd, int64_t rows, int S, int H, float eps, float keep_prob, const uint64_t* seed,
                     uint64_t stream, hipStream_t s, float* amax_part, uint16_t* pieces) {
  const int grid = ln_grid(rows, 4096);
  HX_CH_DISPATCH(H, {
    if (bf16)
      embed_ln_fwd_k<uint16_t, CH><<<grid, NT, 0, s>>>(ids, tt, wte, wpe, wtt, gamma, beta, (uint16_t*)out,
                                                       (uint16_t*)zsave, mean, rstd, rows, S, H, eps, keep_prob,
                                                       seed, stream, nullptr, nullptr);
    else
      embed_ln_fwd_k<float, CH><<<grid, NT, 0, s>>>(ids, tt, wte, wpe, wtt, gamma, beta, (float*)out,
                                                    (float*)zsave, mean, rstd, rows, S, H, eps, keep_prob, seed,
                                                    stream, amax_part, pieces);
  })
}

int hx_type_grad_blocks(int64_t rows) { return ln_grid(rows, 1024); }

void hx_type_grad(int bf16, const void* dz, const int64_t* tt, float* part, float* dwtt, int64_t rows, int H, int ntypes,
                  hipStream_t s) {
  const int grid = hx_type_grad_blocks(rows);
  HX_CH_DISPATCH(H, {
    switch (ntypes) {
      case 1:
        if (bf16) type_grad_k<uint16_t, CH, 1><<<grid, NT, 0, s>>>((const uint16_t*)dz, tt, part, rows, H);
        else type_grad_k<float, CH, 1><<<grid, NT, 0, s>>>((const float*)dz, tt, part, rows, H);
        break;
      case 2:
        if (bf16) type_grad_k<uint16_t, CH, 2><<<grid, NT, 0, s>>>((const uint16_t*)dz, tt, part, rows, H);
        else type_grad_k<float, CH, 2><<<grid, NT, 0, s>>>((const float*)dz, tt, part, rows, H);
        break;
      default:
        if (bf16) type_grad_k<uint16_t, CH, 3><<<grid, NT, 0, s>>>((const uint16_t*)dz, tt, part, rows, H);
        else type_grad_k<float, CH, 3><<<grid, NT, 0, s>>>((const float*)dz, tt, part, rows, H);
        break;
    }
  })
  // [grid][ntypes][H] -> dwtt[t] (rows of ntypes H, one output segment per type)
  hx::fold_rows(part, grid, (int64_t)ntypes * H, ntypes * H, H, dwtt, ntypes > 1 ? dwtt + H : nullptr,
                ntypes > 2 ? dwtt + 2 * H : nullptr, 0, s);
}

void hx_embed_word_grad_sorted(int bf16, const void* dz, const int64_t* ids, const int64_t* order, float* dwte,
                               int64_t rows, int H, hipStream_t s) {
  const int64_t nseg = (rows + kSegRows - 1) / kSegRows;
  const int grid = (int)((nseg + WPB - 1) / WPB);
  HX_CH_DISPATCH(H, {
    if (bf16)
      embed_word_grad_sorted_k<uint16_t, CH><<<grid, NT, 0, s>>>((const uint16_t*)dz, ids, order, dwte, rows, H);
    else
      embed_word_grad_sorted_k<float, CH><<<grid, NT, 0, s>>>((const float*)dz, ids, order, dwte, rows, H);
  })
}

