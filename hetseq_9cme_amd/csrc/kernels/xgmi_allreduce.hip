// Intra-node gradient all-reduce over xGMI peer mappings.
//
// The reference hands every gradient bucket to NCCL through DDP
// (hetseq/controller.py:79-87, 25 MB buckets from options.py:215-216).  On a fully
// connected MI355X node each GPU has a direct xGMI link to each of its 7 peers, so the
// buckets are reduced by a kernel that drives all links at once instead of walking a ring.
//
// IN PLACE: every rank exports its whole flat gradient buffer ONCE (hx_xar_register + the
// IPC exchange); a bucket is a slice [off, off + n) of it on every rank, so peers read each
// other's buckets directly -- no staging copy, no staging allocation.
//
//   two-shot (large buckets)
//     phase 0  "my bucket is final" (its producing kernels have ended: their writes are in
//              memory) -> wait for every peer's;
//     phase 1  (reduce-scatter) rank r sums chunk r of every peer's bucket in RANK ORDER and
//              writes it into its own chunk r -> signal, wait;
//     phase 2  (all-gather) rank r copies every other chunk p from rank p's bucket ->
//              signal "done reading", wait: no rank overwrites its buffer (next step's
//              backward) while a peer still reads it.
//     Hazard-free in place: my chunk q (q != r) is read by peer q only in q's phase 1, and I
//     overwrite it only in my phase 2, after q's phase-1 signal; my chunk r is read by peers
//     only in their phase 2, after my phase-1 signal.  2 (W-1)/W n floats over the links.
//   one-shot (small buckets, latency-bound)
//     phase 0 as above; every rank sums the WHOLE bucket over all peers into registers (the
//     same rank-order sum, so every rank gets bit-identical values), signals "done reading",
//     waits, then stores the sums: two hand-offs instead of three, no second data pass.
//
// Each chunk / element is summed in rank order 0..W-1 everywhere, so every rank ends with
// bitwise identical gradients (the replicas never drift) and the result equals the
// reference's NCCL-free rank-order sum.
//
// Cross-GPU synchronisation is per workgroup, never grid-wide: workgroup b of every rank
// handles the same float4 positions of every chunk, so block b of rank r only ever needs
// block b of its peers.  A hand-off is
//   producer  every wave drains its stores (s_waitcnt vmcnt(0)), workgroup barrier, one
//             lane issues a system-scope release (L2 write-back) and stores the call's
//             epoch into flag[phase][b][r] of every peer (relaxed system-scope atomics
//             into the peer's uncached signal page);
//   consumer  one lane per peer polls its own signal page (system-scope relaxed loads,
//             bounded by a real-time deadline), one system-scope acquire, barrier, then
//             plain loads of the peer's buffer.
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
#include <stdlib.h>
#include <string.h>

#include "hx_launch.h"

namespace {

constexpr int MAXW = 8;     // one node: at most 8 GPUs on xGMI
constexpr int NT = 256;     // threads per workgroup
constexpr int NPHASE = 3;
constexpr int V1 = 4;       // one-shot: float4 positions held in registers per thread

struct Peers {
  float* reg[MAXW];       // registered gradient buffer of each rank (peer ones IPC-mapped)
  uint32_t* flg[MAXW];    // signal pages: [NPHASE][G][MAXW] epochs, then the error word
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

__device__ __forceinline__ void copy_pos(float* dst, const float* src, int64_t e, int64_t end) {
  if (e + 4 <= end) {
    *reinterpret_cast<float4*>(dst + e) = *reinterpret_cast<const float4*>(src + e);
  } else {
    for (int64_t k = e; k < end; ++k) dst[k] = src[k];
  }
}

template <int W>
__device__ __forceinline__ float4 sum_pos(const Peers& P, int64_t off, int64_t e) {
  float4 v[W];
#pragma unroll
  for (int q = 0; q < W; ++q) v[q] = *reinterpret_cast<const float4*>(P.reg[q] + off + e);
  float4 s = v[0];
#pragma unroll
  for (int q = 1; q < W; ++q) {
    s.x += v[q].x; s.y += v[q].y; s.z += v[q].z; s.w += v[q].w;
  }
  return s;
}
template <int W>
__device__ __forceinline__ void sum_tail(const Peers& P, int64_t off, float* dst, int64_t e, int64_t end) {
  for (int64_t k = e; k < end; ++k) {
    float s = 0.f;
    for (int q = 0; q < W; ++q) s += P.reg[q][off + k];
    dst[k] = s;
  }
}

template <int W>
__global__ __launch_bounds__(NT) void xar2_k(Peers P, int64_t off, int64_t n, int64_t c, int rank0, uint32_t epoch,
                                             uint64_t timeout_ticks, int mute) {
  const int G = gridDim.x, b = blockIdx.x;
  const int r = rank0 + (int)blockIdx.y;
  float* buf = P.reg[r] + off;
  const int64_t c4 = (c + 3) >> 2;
  const int64_t stride = (int64_t)G * NT;
  const int64_t j0 = (int64_t)b * NT + threadIdx.x;

  signal_peers(P, W, r, 0, b, G, epoch, mute);
  wait_peers(P, W, r, 0, b, G, epoch, timeout_ticks);

  // ---- phase 1: reduce chunk r in place (rank order, identical on every rank)
  {
    const int64_t base = (int64_t)r * c, end = base + c < n ? base + c : n;
    for (int64_t j = j0; j < c4; j += stride) {
      const int64_t e = base + 4 * j;
      if (e >= end) break;
      if (e + 4 <= end) *reinterpret_cast<float4*>(buf + e) = sum_pos<W>(P, off, e);
      else sum_tail<W>(P, off, buf, e, end);
    }
  }
  signal_peers(P, W, r, 1, b, G, epoch, mute);
  wait_peers(P, W, r, 1, b, G, epoch, timeout_ticks);

  // ---- phase 2: gather the other reduced chunks from their owners
#pragma unroll
  for (int p = 0; p < W; ++p) {
    if (p == r) continue;
    const int64_t base = p * c, end = base + c < n ? base + c : n;
    const float* src = P.reg[p] + off;
    for (int64_t j = j0; j < c4; j += stride) {
      const int64_t e = base + 4 * j;
      if (e < end) copy_pos(buf, src, e, end);
    }
  }
  // nobody may overwrite its buffer (next step's backward) while a peer still reads it
  signal_peers(P, W, r, 2, b, G, epoch, mute);
  wait_peers(P, W, r, 2, b, G, epoch, timeout_ticks);
}

// one-shot: n <= gridDim.x * NT * 4 * V1 floats
template <int W>
__global__ __launch_bounds__(NT) void xar1_k(Peers P, int64_t off, int64_t n, int rank0, uint32_t epoch,
                                             uint64_t timeout_ticks, int mute) {
  const int G = gridDim.x, b = blockIdx.x;
  const int r = rank0 + (int)blockIdx.y;
  float* buf = P.reg[r] + off;
  const int64_t stride = (int64_t)G * NT;
  const int64_t j0 = (int64_t)b * NT + threadIdx.x;

  signal_peers(P, W, r, 0, b, G, epoch, mute);
  wait_peers(P, W, r, 0, b, G, epoch, timeout_ticks);
  float4 s[V1];
  float tail[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int v = 0; v < V1; ++v) {
    const int64_t e = 4 * (j0 + v * stride);
    if (e + 4 <= n) {
      s[v] = sum_pos<W>(P, off, e);
    } else if (e < n) {
      for (int64_t k = e; k < n; ++k) {
        float t = 0.f;
        for (int q = 0; q < W; ++q) t += P.reg[q][off + k];
        tail[k - e] = t;
      }
    }
  }
  signal_peers(P, W, r, 1, b, G, epoch, mute);     // done reading every peer's bucket
  wait_peers(P, W, r, 1, b, G, epoch, timeout_ticks);
#pragma unroll
  for (int v = 0; v < V1; ++v) {
    const int64_t e = 4 * (j0 + v * stride);
    if (e + 4 <= n) *reinterpret_cast<float4*>(buf + e) = s[v];
    else if (e < n)
      for (int64_t k = e; k < n; ++k) buf[k] = tail[k - e];
  }
}

struct Ctx {
  int rank, world, G, device;
  uint32_t epoch;
  float* reg;              // own registered buffer (the flat gradients), not owned
  int64_t reg_n;
  uint32_t* flg;           // own signal page (uncached)
  size_t flg_bytes;
  Peers peers;
  void* opened_base[MAXW];   // IPC mappings to close (peer allocation bases)
  bool opened_flg[MAXW];
  double timeout_s;
  int64_t oneshot_max;     // floats
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
void launch_w(const Ctx& c, const Peers& P, int64_t off, int64_t n, int rank0, int ny, hipStream_t s, uint32_t epoch,
              int mute) {
  const uint64_t ticks = (uint64_t)(c.timeout_s * 1e8);
  if (n <= c.oneshot_max) {
    const int64_t need = (n + 4 * NT * V1 - 1) / (4 * NT * V1);   // workgroups holding n in registers
    const int g = (int)(need < c.G ? (need < 1 ? 1 : need) : c.G);
    xar1_k<W><<<dim3(g, ny), NT, 0, s>>>(P, off, n, rank0, epoch, ticks, mute);
    return;
  }
  int64_t chunk = (n + W - 1) / W;
  chunk = (chunk + 63) & ~int64_t(63);          // 256-B aligned chunk starts
  xar2_k<W><<<dim3(c.G, ny), NT, 0, s>>>(P, off, n, chunk, rank0, epoch, ticks, mute);
}

void launch(const Ctx& c, const Peers& P, int64_t off, int64_t n, int rank0, int ny, hipStream_t s, uint32_t epoch,
            int mute = -1) {
  switch (c.world) {
    case 2: launch_w<2>(c, P, off, n, rank0, ny, s, epoch, mute); break;
    case 3: launch_w<3>(c, P, off, n, rank0, ny, s, epoch, mute); break;
    case 4: launch_w<4>(c, P, off, n, rank0, ny, s, epoch, mute); break;
    case 5: launch_w<5>(c, P, off, n, rank0, ny, s, epoch, mute); break;
    case 6: launch_w<6>(c, P, off, n, rank0, ny, s, epoch, mute); break;
    case 7: launch_w<7>(c, P, off, n, rank0, ny, s, epoch, mute); break;
    default: launch_w<8>(c, P, off, n, rank0, ny, s, epoch, mute); break;
  }
}

}  // namespace

const char* hx_xar_last_error() { return g_err; }

int hx_xar_create(int rank, int world, int nblocks, double timeout_s, int64_t oneshot_max_bytes, void** out) {
  g_err[0] = 0;
  if (world < 2 || world > MAXW || rank < 0 || rank >= world || nblocks < 1 || nblocks > 1024) {
    snprintf(g_err, sizeof(g_err), "xgmi all-reduce: bad arguments (rank %d world %d blocks %d)", rank, world,
             nblocks);
    return -1;
  }
  Ctx* c = new Ctx();
  memset(c, 0, sizeof(Ctx));
  c->rank = rank;
  c->world = world;
  c->G = nblocks;
  c->timeout_s = timeout_s;
  const int64_t cap1 = (int64_t)nblocks * NT * 4 * V1;   // what the one-shot grid holds in registers
  const int64_t want = oneshot_max_bytes / 4;
  c->oneshot_max = want < cap1 ? want : cap1;
  HX_HIP(hipGetDevice(&c->device));
  c->flg_bytes = ((size_t)NPHASE * nblocks * MAXW + 64) * sizeof(uint32_t);
  HX_HIP(hipExtMallocWithFlags((void**)&c->flg, c->flg_bytes, hipDeviceMallocUncached));
  HX_HIP(hipMemset(c->flg, 0, c->flg_bytes));
  HX_HIP(hipDeviceSynchronize());
  c->peers.flg[rank] = c->flg;
  *out = c;
  return 0;
}

int64_t hx_xar_oneshot_max(void* ctx) { return static_cast<Ctx*>(ctx)->oneshot_max; }

// the buffer every bucket lives in (this rank's flat gradients); before export / open
int hx_xar_register(void* ctx, float* base, int64_t n) {
  Ctx* c = static_cast<Ctx*>(ctx);
  c->reg = base;
  c->reg_n = n;
  c->peers.reg[c->rank] = base;
  return 0;
}

// IPC handle of the registered buffer's allocation + the buffer's byte offset in it, and of
// the signal page: kXarRecord bytes
int hx_xar_export(void* ctx, char* out) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c->reg) {
    snprintf(g_err, sizeof(g_err), "xgmi all-reduce: export before register");
    return -1;
  }
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
  void* base = nullptr;
  size_t size = 0;
  HX_HIP(hipMemGetAddressRange(&base, &size, c->reg));
  hipIpcMemHandle_t h0, h1;
  HX_HIP(hipIpcGetMemHandle(&h0, base));
  HX_HIP(hipIpcGetMemHandle(&h1, c->flg));
  const int64_t offset = (int64_t)((char*)c->reg - (char*)base);
  memset(out, 0, kXarRecord);
  memcpy(out, &h0, 64);
  memcpy(out + 64, &offset, 8);
  memcpy(out + 72, &c->reg_n, 8);
  memcpy(out + 80, &h1, 64);
  return 0;
}

// map every peer's registered buffer and signal page (records: world x kXarRecord bytes)
int hx_xar_open(void* ctx, const char* recs) {
  Ctx* c = static_cast<Ctx*>(ctx);
  for (int q = 0; q < c->world; ++q) {
    if (q == c->rank) continue;
    const char* rec = recs + (size_t)kXarRecord * q;
    hipIpcMemHandle_t h0, h1;
    int64_t offset = 0, n = 0;
    memcpy(&h0, rec, 64);
    memcpy(&offset, rec + 64, 8);
    memcpy(&n, rec + 72, 8);
    memcpy(&h1, rec + 80, 64);
    if (n != c->reg_n) {
      snprintf(g_err, sizeof(g_err), "xgmi all-reduce: rank %d registered %lld floats, rank %d %lld", q,
               (long long)n, c->rank, (long long)c->reg_n);
      return -1;
    }
    void *p0 = nullptr, *p1 = nullptr;
    HX_HIP(hipIpcOpenMemHandle(&p0, h0, hipIpcMemLazyEnablePeerAccess));
    c->opened_base[q] = p0;
    HX_HIP(hipIpcOpenMemHandle(&p1, h1, hipIpcMemLazyEnablePeerAccess));
    c->opened_flg[q] = true;
    c->peers.reg[q] = reinterpret_cast<float*>(static_cast<char*>(p0) + offset);
    c->peers.flg[q] = static_cast<uint32_t*>(p1);
  }
  return 0;
}

// in-place SUM all-reduce of buf[0, n), a slice of the registered buffer (same call sequence,
// same slices on every rank)
int hx_xar_allreduce(void* ctx, float* buf, int64_t n, hipStream_t s) {
  Ctx* c = static_cast<Ctx*>(ctx);
  const int64_t off = buf - c->reg;
  if (!c->reg || off < 0 || off + n > c->reg_n || (off & 3)) {
    snprintf(g_err, sizeof(g_err), "xgmi all-reduce: bucket [%lld, +%lld) is not a 16-B aligned slice of the "
             "registered buffer (%lld floats)", (long long)off, (long long)n, (long long)c->reg_n);
    return -1;
  }
  if (n == 0) return 0;
  launch(*c, c->peers, off, n, c->rank, 1, s, ++c->epoch);
  HX_HIP(hipGetLastError());
  return 0;
}

// test-only: W simulated ranks in ONE grid on one device; ctxs[q] are W contexts created
// on this device, bufs[q] the rank-q buckets (all n floats)
int hx_xar_allreduce_sim(void** ctxs, float** bufs, int W, int64_t n, int mute, hipStream_t s) {
  Ctx* c0 = static_cast<Ctx*>(ctxs[0]);
  Peers P;
  memset(&P, 0, sizeof(P));
  for (int q = 0; q < W; ++q) {
    Ctx* c = static_cast<Ctx*>(ctxs[q]);
    P.reg[q] = bufs[q];
    P.flg[q] = c->flg;
  }
  const uint32_t epoch = ++c0->epoch;
  for (int q = 1; q < W; ++q) static_cast<Ctx*>(ctxs[q])->epoch = epoch;
  launch(*c0, P, 0, n, 0, W, s, epoch, mute);
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
  for (int q = 0; q < MAXW; ++q) {
    if (c->opened_base[q]) (void)hipIpcCloseMemHandle(c->opened_base[q]);
    if (c->opened_flg[q]) (void)hipIpcCloseMemHandle(c->peers.flg[q]);
  }
  (void)hipFree(c->flg);
  delete c;
}
