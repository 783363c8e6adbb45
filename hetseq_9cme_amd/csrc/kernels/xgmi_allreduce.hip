// Intra-node gradient all-reduce over xGMI peer mappings.
//
// The reference hands every gradient bucket to NCCL through DDP
// (hetseq/controller.py:79-87, 25 MB buckets from options.py:215-216).  On a fully
// connected MI355X node each GPU has a direct xGMI link to each of its 7 peers, so a
// "two-shot" all-reduce drives all links at once instead of walking a ring:
//
//   phase 0  every rank copies its bucket into its own IPC-exported staging buffer;
//   phase 1  (reduce-scatter) rank r pulls chunk r of every peer's staging buffer over
//            xGMI, sums the W copies in rank order and writes the sum to its bucket and
//            to chunk r of its staging buffer;
//   phase 2  (all-gather) rank r pulls every other chunk p from rank p's staging buffer.
//
// Per rank and bucket of n floats that is 2 (W-1)/W n floats of xGMI reads spread
// evenly over the W-1 links.  Each chunk is summed by exactly one rank, so every rank
// ends with bitwise identical gradients (the replicas never drift).
//
// Cross-GPU synchronisation is per workgroup, never grid-wide: workgroup b of every rank
// handles the same float4 positions j of every chunk (grid-stride set J_b), so block b of
// rank r only ever needs block b of its peers.  A hand-off is
//   producer  every wave drains its stores (s_waitcnt vmcnt(0)), workgroup barrier, one
//             lane issues a system-scope release (L2 write-back) and stores the call's
//             epoch into flag[phase][b][r] of every peer (relaxed system-scope atomics
//             into the peer's uncached signal page);
//   consumer  one lane per peer polls its own signal page (system-scope relaxed loads,
//             bounded by a real-time deadline), one system-scope acquire, barrier, then
//             plain loads of the peer's staging buffer.
// Epochs grow monotonically per call (the host counter advances identically on every
// rank because buckets are launched in the same order everywhere), so flags are never
// reset.  A wait that passes its deadline sets an error word and lets the kernel drain
// (no wave can spin forever); the host reads the word and raises.
//
// Simulation mode (tests): gridDim.y = W launches every rank's workgroups in ONE grid on
// one device (rank = blockIdx.y), which checks chunking, tails and the flag protocol
// without a second GPU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "hx_launch.h"

namespace {

constexpr int MAXW = 8;     // one node: at most 8 GPUs on xGMI
constexpr int NT = 256;     // threads per workgroup
constexpr int NPHASE = 3;

struct Peers {
  float* stg[MAXW];       // staging buffers (index = rank), peer ones IPC-mapped
  uint32_t* flg[MAXW];    // signal pages: [NPHASE][G][MAXW] epochs, then the error word
  float* buf[MAXW];       // bucket of each simulated rank (only [rank] used otherwise)
};

__device__ __forceinline__ uint32_t* flag_at(uint32_t* page, int ph, int b, int G, int src) {
  return page + ((size_t)ph * G + b) * MAXW + src;
}

// all stores of this workgroup drained, then flags raised at every peer
__device__ __forceinline__ void signal_peers(const Peers& P, int W, int r, int ph, int b, int G, uint32_t epoch,
                                             int mute) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && r != mute) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope: write back L2 for remote readers
    for (int q = 0; q < W; ++q)
      if (q != r) __hip_atomic_store(flag_at(P.flg[q], ph, b, G, r), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__device__ __forceinline__ void wait_peers(const Peers& P, int W, int r, int ph, int b, int G, uint32_t epoch,
                                           uint64_t timeout_ticks) {
  const int t = threadIdx.x;
  if (t < 64) {
    if (t < W && t != r) {
      uint32_t* f = flag_at(P.flg[r], ph, b, G, t);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz constant clock
      while ((int32_t)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
          uint32_t* err = P.flg[r] + (size_t)NPHASE * G * MAXW;
          __hip_atomic_fetch_or(err, 1u << ph, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");      // system scope: drop stale L1/L2 lines
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// float4 position j of a chunk starting at element `base`, valid elements [base, end)
__device__ __forceinline__ void copy_pos(float* dst, const float* src, int64_t e, int64_t end) {
  if (e + 4 <= end) {
    *reinterpret_cast<float4*>(dst + e) = *reinterpret_cast<const float4*>(src + e);
  } else {
    for (int64_t k = e; k < end; ++k) dst[k] = src[k];
  }
}

template <int W>
__global__ __launch_bounds__(NT) void xar_k(Peers P, int64_t n, int64_t c, int rank0, uint32_t epoch,
                                            uint64_t timeout_ticks, int mute) {
  const int G = gridDim.x, b = blockIdx.x;
  const int r = rank0 + (int)blockIdx.y;
  float* buf = P.buf[r];
  float* mine = P.stg[r];
  const int64_t c4 = (c + 3) >> 2;
  const int64_t stride = (int64_t)G * NT;
  const int64_t j0 = (int64_t)b * NT + threadIdx.x;

  // ---- phase 0: publish my copy of every chunk the peers will reduce
#pragma unroll
  for (int p = 0; p < W; ++p) {
    if (p == r) continue;
    const int64_t base = p * c, end = base + c < n ? base + c : n;
    for (int64_t j = j0; j < c4; j += stride) {
      const int64_t e = base + 4 * j;
      if (e < end) copy_pos(mine, buf, e, end);
    }
  }
  signal_peers(P, W, r, 0, b, G, epoch, mute);
  wait_peers(P, W, r, 0, b, G, epoch, timeout_ticks);

  // ---- phase 1: reduce chunk r (rank order, identical on every rank), keep it staged
  {
    const int64_t base = (int64_t)r * c, end = base + c < n ? base + c : n;
    for (int64_t j = j0; j < c4; j += stride) {
      const int64_t e = base + 4 * j;
      if (e >= end) break;
      if (e + 4 <= end) {
        float4 v[W];
#pragma unroll
        for (int q = 0; q < W; ++q)
          v[q] = *reinterpret_cast<const float4*>((q == r ? buf : P.stg[q]) + e);
        float4 s = v[0];
#pragma unroll
        for (int q = 1; q < W; ++q) {
          s.x += v[q].x; s.y += v[q].y; s.z += v[q].z; s.w += v[q].w;
        }
        *reinterpret_cast<float4*>(buf + e) = s;
        *reinterpret_cast<float4*>(mine + e) = s;
      } else {
        for (int64_t k = e; k < end; ++k) {
          float s = 0.f;
          for (int q = 0; q < W; ++q) s += (q == r ? buf : P.stg[q])[k];
          buf[k] = s;
          mine[k] = s;
        }
      }
    }
  }
  signal_peers(P, W, r, 1, b, G, epoch, mute);
  wait_peers(P, W, r, 1, b, G, epoch, timeout_ticks);

  // ---- phase 2: gather the other reduced chunks
#pragma unroll
  for (int p = 0; p < W; ++p) {
    if (p == r) continue;
    const int64_t base = p * c, end = base + c < n ? base + c : n;
    const float* src = P.stg[p];
    for (int64_t j = j0; j < c4; j += stride) {
      const int64_t e = base + 4 * j;
      if (e < end) copy_pos(buf, src, e, end);
    }
  }
  // nobody may overwrite a staging buffer (next call's phase 0/1) while a peer still reads it
  signal_peers(P, W, r, 2, b, G, epoch, mute);
  wait_peers(P, W, r, 2, b, G, epoch, timeout_ticks);
}

struct Ctx {
  int rank, world, G, device;
  int64_t cap;             // staging capacity in floats
  uint32_t epoch;
  float* stg;              // own staging (hipMalloc)
  uint32_t* flg;           // own signal page (uncached)
  size_t flg_bytes;
  Peers peers;
  bool opened[MAXW];
  double timeout_s;
};

#define HX_HIP(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      snprintf(g_err, sizeof(g_err), "%s failed: %s", #x, hipGetErrorString(e_));          \
      return -1;                                                                           \
    }                                                                                      \
  } while (0)

thread_local char g_err[256];

template <int W>
void launch_w(const Ctx& c, const Peers& P, int64_t n, int rank0, int ny, hipStream_t s, uint32_t epoch, int mute) {
  int64_t chunk = (n + W - 1) / W;
  chunk = (chunk + 63) & ~int64_t(63);          // 256-B aligned chunk starts
  const uint64_t ticks = (uint64_t)(c.timeout_s * 1e8);
  xar_k<W><<<dim3(c.G, ny), NT, 0, s>>>(P, n, chunk, rank0, epoch, ticks, mute);
}

void launch(const Ctx& c, const Peers& P, int64_t n, int rank0, int ny, hipStream_t s, uint32_t epoch,
            int mute = -1) {
  switch (c.world) {
    case 2: launch_w<2>(c, P, n, rank0, ny, s, epoch, mute); break;
    case 3: launch_w<3>(c, P, n, rank0, ny, s, epoch, mute); break;
    case 4: launch_w<4>(c, P, n, rank0, ny, s, epoch, mute); break;
    case 5: launch_w<5>(c, P, n, rank0, ny, s, epoch, mute); break;
    case 6: launch_w<6>(c, P, n, rank0, ny, s, epoch, mute); break;
    case 7: launch_w<7>(c, P, n, rank0, ny, s, epoch, mute); break;
    default: launch_w<8>(c, P, n, rank0, ny, s, epoch, mute); break;
  }
}

}  // namespace

const char* hx_xar_last_error() { return g_err; }

int hx_xar_create(int rank, int world, int64_t cap_floats, int nblocks, double timeout_s, void** out) {
  g_err[0] = 0;
  if (world < 2 || world > MAXW || rank < 0 || rank >= world || nblocks < 1 || nblocks > 1024 || cap_floats < 64) {
    snprintf(g_err, sizeof(g_err), "xgmi all-reduce: bad arguments (rank %d world %d blocks %d cap %lld)", rank, world,
             nblocks, (long long)cap_floats);
    return -1;
  }
  Ctx* c = new Ctx();
  memset(c, 0, sizeof(Ctx));
  c->rank = rank;
  c->world = world;
  c->G = nblocks;
  c->cap = (cap_floats + 63) & ~int64_t(63);
  c->timeout_s = timeout_s;
  HX_HIP(hipGetDevice(&c->device));
  HX_HIP(hipMalloc((void**)&c->stg, c->cap * sizeof(float)));
  c->flg_bytes = ((size_t)NPHASE * nblocks * MAXW + 64) * sizeof(uint32_t);
  HX_HIP(hipExtMallocWithFlags((void**)&c->flg, c->flg_bytes, hipDeviceMallocUncached));
  HX_HIP(hipMemset(c->flg, 0, c->flg_bytes));
  HX_HIP(hipDeviceSynchronize());
  c->peers.stg[rank] = c->stg;
  c->peers.flg[rank] = c->flg;
  *out = c;
  return 0;
}

int64_t hx_xar_capacity(void* ctx) { return static_cast<Ctx*>(ctx)->cap; }

// IPC handles of the staging buffer and the signal page (2 x 64 bytes)
int hx_xar_export(void* ctx, char* out128) {
  Ctx* c = static_cast<Ctx*>(ctx);
  hipIpcMemHandle_t h0, h1;
  HX_HIP(hipIpcGetMemHandle(&h0, c->stg));
  HX_HIP(hipIpcGetMemHandle(&h1, c->flg));
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
  memcpy(out128, &h0, 64);
  memcpy(out128 + 64, &h1, 64);
  return 0;
}

// map every peer's staging buffer and signal page (handles: world x 128 bytes)
int hx_xar_open(void* ctx, const char* handles) {
  Ctx* c = static_cast<Ctx*>(ctx);
  for (int q = 0; q < c->world; ++q) {
    if (q == c->rank) continue;
    hipIpcMemHandle_t h0, h1;
    memcpy(&h0, handles + 128 * q, 64);
    memcpy(&h1, handles + 128 * q + 64, 64);
    void *p0 = nullptr, *p1 = nullptr;
    HX_HIP(hipIpcOpenMemHandle(&p0, h0, hipIpcMemLazyEnablePeerAccess));
    HX_HIP(hipIpcOpenMemHandle(&p1, h1, hipIpcMemLazyEnablePeerAccess));
    c->peers.stg[q] = static_cast<float*>(p0);
    c->peers.flg[q] = static_cast<uint32_t*>(p1);
    c->opened[q] = true;
  }
  return 0;
}

// in-place SUM all-reduce of buf[0, n) with the peers (same call sequence on every rank);
// buckets larger than the staging capacity run as consecutive pieces
int hx_xar_allreduce(void* ctx, float* buf, int64_t n, hipStream_t s) {
  Ctx* c = static_cast<Ctx*>(ctx);
  for (int64_t off = 0; off < n; off += c->cap) {
    const int64_t m = n - off < c->cap ? n - off : c->cap;
    Peers P = c->peers;
    P.buf[c->rank] = buf + off;
    launch(*c, P, m, c->rank, 1, s, ++c->epoch);
  }
  HX_HIP(hipGetLastError());
  return 0;
}

// test-only: W simulated ranks in ONE grid on one device; ctxs[q] are W contexts created
// on this device, bufs[q] the rank-q buckets (all n floats)
int hx_xar_allreduce_sim(void** ctxs, float** bufs, int W, int64_t n, int mute, hipStream_t s) {
  Ctx* c0 = static_cast<Ctx*>(ctxs[0]);
  if (n > c0->cap) {
    snprintf(g_err, sizeof(g_err), "simulation bucket larger than the staging capacity");
    return -1;
  }
  Peers P;
  memset(&P, 0, sizeof(P));
  for (int q = 0; q < W; ++q) {
    Ctx* c = static_cast<Ctx*>(ctxs[q]);
    P.stg[q] = c->stg;
    P.flg[q] = c->flg;
    P.buf[q] = bufs[q];
  }
  const uint32_t epoch = ++c0->epoch;
  for (int q = 1; q < W; ++q) static_cast<Ctx*>(ctxs[q])->epoch = epoch;
  launch(*c0, P, n, 0, W, s, epoch, mute);
  HX_HIP(hipGetLastError());
  return 0;
}

// error word of the signal page (synchronising read): bit ph = a phase-ph wait timed out
int hx_xar_error(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  uint32_t e = 0;
  HX_HIP(hipMemcpy(&e, c->flg + (size_t)NPHASE * c->G * MAXW, sizeof(e), hipMemcpyDeviceToHost));
  return (int)e;
}

int hx_xar_error_async(void* ctx, int32_t* dst, hipStream_t s) {
  Ctx* c = static_cast<Ctx*>(ctx);
  HX_HIP(hipMemcpyAsync(dst, c->flg + (size_t)NPHASE * c->G * MAXW, sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  return 0;
}

void hx_xar_destroy(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return;
  (void)hipDeviceSynchronize();
  for (int q = 0; q < MAXW; ++q)
    if (c->opened[q]) {
      (void)hipIpcCloseMemHandle(c->peers.stg[q]);
      (void)hipIpcCloseMemHandle(c->peers.flg[q]);
    }
  (void)hipFree(c->stg);
  (void)hipFree(c->flg);
  delete c;
}
