// Optimizer-side kernels over the FLAT fp32 parameter / gradient / moment buffers.
//
// Replaces the reference's per-parameter Python loops (hetseq/optim.py:59-70
// multiply_grads + clip_grad_norm_, :162-231 Adam, :263-304 Adadelta; ~1,850
// launches per BERT step) with:
//   1. grad_norm_partial : one grid-stride L2 reduction over the whole flat grad
//      buffer (float4 loads, per-block double partial)
//   2. grad_norm_finalize: one workgroup folds the partials, applies the pending
//      grad scale (W / sample_size, a DEVICE scalar), computes the clip coefficient
//      and folds it into the same scalar -- no host synchronisation.
//   3. adam / adadelta   : one streaming pass per contiguous parameter run reading
//      p, g, m, v once (16 B per lane per stream) and writing p, m, v (+ optional
//      bf16 shadow of p for the bf16 compute path).
// HBM-bound: BERT-base (110.1M params) Adam moves 7 x 440 MB = 3.1 GB -> ~0.5 ms.
#include "hx_common.h"
#include "hx_launch.h"

namespace {

constexpr int NT = 256;

__global__ __launch_bounds__(NT) void grad_norm_partial_k(const float* __restrict__ g, int64_t n,
                                                        double* __restrict__ partial) {
  __shared__ float scratch[NT / 64];
  const int64_t n4 = n >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float acc = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * NT) {
    const float4 v = g4[i];
    acc = fmaf(v.x, v.x, acc);
    acc = fmaf(v.y, v.y, acc);
    acc = fmaf(v.z, v.z, acc);
    acc = fmaf(v.w, v.w, acc);
  }
  // tail (n not a multiple of 4)
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    acc = fmaf(g[i], g[i], acc);
  const float s = hx::block_sum<NT>(acc, scratch);
  if (threadIdx.x == 0) partial[blockIdx.x] = (double)s;
}

__global__ __launch_bounds__(NT) void grad_norm_finalize_k(const double* __restrict__ partial, int np,
                                                         float* __restrict__ gscale, float* __restrict__ out_norm,
                                                         float* __restrict__ clipped, float max_norm) {
  __shared__ double sd[NT / 64];
  double acc = 0.0;
  for (int i = threadIdx.x; i < np; i += NT) acc += partial[i];
  acc = hx::wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) sd[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < NT / 64; ++w) t += sd[w];
    const float gs = gscale[0];
    const float norm = (float)sqrt(t) * fabsf(gs);
    out_norm[0] = norm;
    if (max_norm > 0.f) {
      const float coef = fminf(1.0f, max_norm / (norm + 1e-6f));
      clipped[0] = norm > max_norm ? 1.f : 0.f;
      gscale[0] = gs * coef;
    } else {
      clipped[0] = 0.f;
    }
  }
}

// One Adam element update with every rounding spelled out (explicit fma / _rn ops, nothing
// left to contraction), so every kernel that uses it -- the per-run kernel, the device-mask
// kernel, with or without the bf16 shadow -- produces bitwise the same parameters.
__device__ __forceinline__ void adam1(float& x, const float gg, float& m, float& v, float gs, float b1, float b2,
                                      float ob1, float ob2, float eps, float step_size, float wd_lr) {
  const float gr = __fmul_rn(gg, gs);
  m = fmaf(m, b1, __fmul_rn(ob1, gr));
  v = fmaf(v, b2, __fmul_rn(__fmul_rn(ob2, gr), gr));
  const float denom = __fadd_rn(sqrtf(v), eps);
  x = fmaf(-wd_lr, x, x);
  x = fmaf(-step_size, __fdiv_rn(m, denom), x);
}

template <bool kShadow>
__device__ __forceinline__ void adam4(float4& pp, const float4 gg, float4& mm, float4& vv, float gs, float b1,
                                      float b2, float ob1, float ob2, float eps, float step_size, float wd_lr) {
  float* pa = &pp.x;
  const float* ga = &gg.x;
  float* ma = &mm.x;
  float* va = &vv.x;
#pragma unroll
  for (int j = 0; j < 4; ++j) adam1(pa[j], ga[j], ma[j], va[j], gs, b1, b2, ob1, ob2, eps, step_size, wd_lr);
}

typedef float f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ntload(const float4* a) {
  const f32x4_t r = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(a));
  return make_float4(r.x, r.y, r.z, r.w);
}
__device__ __forceinline__ void ntstore(float4 v, float4* a) {
  f32x4_t r = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(r, reinterpret_cast<f32x4_t*>(a));
}

// Streaming update: every byte of p/g/m/v is touched once per step (7 x 4 B per
// parameter, 3 GB for BERT-base), so two independent float4 groups per thread
// per iteration keep more loads in flight and non-temporal hints keep the
// stream from evicting the L2 / MALL working set of the next kernels.
template <bool kShadow>
__global__ __launch_bounds__(NT) void adam_k(float* __restrict__ p, const float* __restrict__ g,
                                           float* __restrict__ m, float* __restrict__ v,
                                           uint16_t* __restrict__ shadow, const float* __restrict__ gscale,
                                           int64_t n, float b1, float b2, float eps, float step_size,
                                           float wd_lr, const float* __restrict__ hp) {
  const float gs = gscale[0];
  if (hp) {   // graph-captured step: per-update step size / decay written before each replay
    step_size = hp[0];
    wd_lr = hp[1];
  }
  const float ob1 = 1.f - b1, ob2 = 1.f - b2;
  const int64_t n4 = n >> 2;
  float4* P = reinterpret_cast<float4*>(p);
  const float4* G = reinterpret_cast<const float4*>(g);
  float4* M = reinterpret_cast<float4*>(m);
  float4* V = reinterpret_cast<float4*>(v);
  const int64_t stride = (int64_t)gridDim.x * NT;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n4; i += 2 * stride) {
    const int64_t i2 = i + stride;
    const bool two = i2 < n4;
    float4 p0 = ntload(P + i), m0 = ntload(M + i), v0 = ntload(V + i);
    const float4 g0 = ntload(G + i);
    float4 p1 = make_float4(0.f, 0.f, 0.f, 0.f), m1 = p1, v1 = p1, g1 = p1;
    if (two) {
      p1 = ntload(P + i2); m1 = ntload(M + i2); v1 = ntload(V + i2); g1 = ntload(G + i2);
    }
    adam4<kShadow>(p0, g0, m0, v0, gs, b1, b2, ob1, ob2, eps, step_size, wd_lr);
    ntstore(p0, P + i); ntstore(m0, M + i); ntstore(v0, V + i);
    if (kShadow)
      reinterpret_cast<ushort4*>(shadow)[i] = make_ushort4(hx::f2bf(p0.x), hx::f2bf(p0.y), hx::f2bf(p0.z),
                                                           hx::f2bf(p0.w));
    if (two) {
      adam4<kShadow>(p1, g1, m1, v1, gs, b1, b2, ob1, ob2, eps, step_size, wd_lr);
      ntstore(p1, P + i2); ntstore(m1, M + i2); ntstore(v1, V + i2);
      if (kShadow)
        reinterpret_cast<ushort4*>(shadow)[i2] = make_ushort4(hx::f2bf(p1.x), hx::f2bf(p1.y), hx::f2bf(p1.z),
                                                              hx::f2bf(p1.w));
    }
  }
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    float x = p[i], mi = m[i], vi = v[i];
    adam1(x, g[i], mi, vi, gs, b1, b2, ob1, ob2, eps, step_size, wd_lr);
    m[i] = mi;
    v[i] = vi;
    p[i] = x;
    if (kShadow) shadow[i] = hx::f2bf(x);
  }
}

__global__ __launch_bounds__(NT) void adadelta_k(float* __restrict__ p, const float* __restrict__ g,
                                               float* __restrict__ sq, float* __restrict__ acc,
                                               const float* __restrict__ gscale, int64_t n, float lr, float rho,
                                               float eps, float wd, const float* __restrict__ hp) {
  const float gs = gscale[0];
  if (hp) lr = hp[0];
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    float gr = g[i] * gs;
    const float x = p[i];
    if (wd != 0.f) gr = gr + wd * x;
    const float s = sq[i] * rho + (1.f - rho) * gr * gr;
    const float std_ = sqrtf(s + eps);
    const float delta = sqrtf(acc[i] + eps) / std_ * gr;
    p[i] = x - lr * delta;
    acc[i] = acc[i] * rho + (1.f - rho) * delta * delta;
    sq[i] = s;
  }
}

// --find-unused-parameters without a host round trip: the per-parameter "used on some
// rank" flags arrive as a slice of the all-reduced stats vector (f64 sums, > 0 = used).
// adam_steps_k advances the per-parameter step counters ON DEVICE and writes each
// parameter's (step size, wd * lr) -- 0-step parameters are skipped entirely, exactly the
// reference's `if p.grad is None: continue` (hetseq/optim.py:186-189) -- and
// adam_masked_k runs one block per <= kMaskChunk-element slice of ONE parameter (a static
// table built once from the flat layout), so an unused parameter's blocks exit at once.
constexpr int kMaskChunk = NT * 4 * 4;   // 4096 floats per block

__global__ __launch_bounds__(NT) void adam_steps_k(int nparam, const double* __restrict__ used,
                                                 int* __restrict__ steps, float* __restrict__ hp, double lr,
                                                 double b1, double b2, double wd, const double* __restrict__ lr_dev) {
  if (lr_dev) lr = lr_dev[0];   // graph-captured updates: this update's lr, written before the replay
  for (int i = threadIdx.x; i < nparam; i += NT) {
    const bool u = used[i] > 0.0;
    const int t = steps[i] + (u ? 1 : 0);
    steps[i] = t;
    // same float64 arithmetic as the host path (optimizers.py _Adam._host_step)
    const double ss = u ? lr * sqrt(1.0 - pow(b2, (double)t)) / (1.0 - pow(b1, (double)t)) : 0.0;
    hp[2 * i] = (float)ss;
    hp[2 * i + 1] = u ? (float)(wd * lr) : 0.f;
  }
}

template <bool kShadow>
__global__ __launch_bounds__(NT) void adam_masked_k(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ m, float* __restrict__ v,
                                                  uint16_t* __restrict__ shadow, const float* __restrict__ gscale,
                                                  const int64_t* __restrict__ table, const double* __restrict__ used,
                                                  const float* __restrict__ hp, float b1, float b2, float eps) {
  const int64_t* row = table + 3 * (int64_t)blockIdx.x;   // (param, start, end): float offsets, 4-aligned
  const int pi = (int)row[0];
  if (!(used[pi] > 0.0)) return;
  const float step_size = hp[2 * pi], wd_lr = hp[2 * pi + 1];
  const float gs = gscale[0];
  const float ob1 = 1.f - b1, ob2 = 1.f - b2;
  const int64_t a = row[1] >> 2, e = row[2] >> 2;
  float4* P = reinterpret_cast<float4*>(p);
  const float4* G = reinterpret_cast<const float4*>(g);
  float4* M = reinterpret_cast<float4*>(m);
  float4* V = reinterpret_cast<float4*>(v);
  for (int64_t i = a + threadIdx.x; i < e; i += NT) {
    float4 pp = ntload(P + i), mm = ntload(M + i), vv = ntload(V + i);
    const float4 gg = ntload(G + i);
    adam4<kShadow>(pp, gg, mm, vv, gs, b1, b2, ob1, ob2, eps, step_size, wd_lr);
    ntstore(pp, P + i); ntstore(mm, M + i); ntstore(vv, V + i);
    if (kShadow)
      reinterpret_cast<ushort4*>(shadow)[i] = make_ushort4(hx::f2bf(pp.x), hx::f2bf(pp.y), hx::f2bf(pp.z),
                                                           hx::f2bf(pp.w));
  }
}

inline int grid_for(int64_t n_vec, int cap = 4096) {
  int64_t b = (n_vec + NT - 1) / NT;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

}  // namespace

int hx_grad_norm_partials() { return 1024; }

void hx_grad_norm_clip(const float* g, int64_t n, double* partial_ws, float* gscale, float* out_norm,
                       float* clipped, float max_norm, hipStream_t s) {
  const int np = hx_grad_norm_partials();
  grad_norm_partial_k<<<np, NT, 0, s>>>(g, n, partial_ws);
  grad_norm_finalize_k<<<1, NT, 0, s>>>(partial_ws, np, gscale, out_norm, clipped, max_norm);
}

void hx_adam(float* p, const float* g, float* m, float* v, uint16_t* shadow, const float* gscale, int64_t n,
             float b1, float b2, float eps, float step_size, float wd_lr, const float* hp, hipStream_t s) {
  const int grid = grid_for((n + 3) / 4, 8192);
  if (shadow)
    adam_k<true><<<grid, NT, 0, s>>>(p, g, m, v, shadow, gscale, n, b1, b2, eps, step_size, wd_lr, hp);
  else
    adam_k<false><<<grid, NT, 0, s>>>(p, g, m, v, shadow, gscale, n, b1, b2, eps, step_size, wd_lr, hp);
}

void hx_adadelta(float* p, const float* g, float* sq, float* acc, const float* gscale, int64_t n, float lr,
                 float rho, float eps, float wd, const float* hp, hipStream_t s) {
  adadelta_k<<<grid_for(n, 8192), NT, 0, s>>>(p, g, sq, acc, gscale, n, lr, rho, eps, wd, hp);
}

int hx_adam_mask_chunk() { return kMaskChunk; }

void hx_adam_masked(float* p, const float* g, float* m, float* v, uint16_t* shadow, const float* gscale,
                    const int64_t* table, int nblocks, const double* used, int* steps, float* hp, int nparam,
                    double lr, double b1, double b2, float eps, double wd, const double* lr_dev, hipStream_t s) {
  adam_steps_k<<<1, NT, 0, s>>>(nparam, used, steps, hp, lr, b1, b2, wd, lr_dev);
  if (nblocks <= 0) return;
  if (shadow)
    adam_masked_k<true><<<nblocks, NT, 0, s>>>(p, g, m, v, shadow, gscale, table, used, hp, (float)b1, (float)b2,
                                                eps);
  else
    adam_masked_k<false><<<nblocks, NT, 0, s>>>(p, g, m, v, shadow, gscale, table, used, hp, (float)b1, (float)b2,
                                                 eps);
}
