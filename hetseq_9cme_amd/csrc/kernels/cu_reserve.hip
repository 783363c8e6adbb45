// Compute units reserved for communication kernels.
//
// The gradient all-reduce (RCCL ring kernels, or the hand-written xGMI kernel) runs on its own
// stream WHILE the backward's GEMMs run.  The GEMM / weight-gradient plans size their grids to
// whole rounds of one workgroup per CU (126-144 KiB of LDS each: no co-residence), so a comm
// kernel holding R CUs pushes R workgroups of a one-round plan into a second round -- the
// kernel takes up to twice as long while the comm is in flight.  With ``hx_set_reserved_cus(R)``
// the plans count only the CUs the comm leaves free (wgrad: split count sized to
// n_cu - R slots; piece GEMM: the tile shape whose tiles fill whole rounds of n_cu - R), and the
// comm side is confined to R CUs: a CU-masked HIP stream for the xGMI kernel, RCCL's channel cap
// (NCCL_MAX_NCHANNELS, one workgroup per channel) for the library.
//
// Also here: a spin kernel that occupies a given number of CUs for a given time on such a
// stream -- the stand-in comm load of the one-GPU contention A/B
// (tools/probe/comm_contention_probe.py).
#include <atomic>
#include <vector>

#include "hx_launch.h"

namespace {
std::atomic<int> g_reserved{0};
int g_ncu = 0;

__global__ __launch_bounds__(256) void spin_k(uint64_t ticks, uint32_t* sink) {
  // wall time from s_memrealtime (100 MHz): every wave busy-waits `ticks` and exits; the dynamic
  // LDS of the launch (like an RCCL kernel's) keeps a GEMM workgroup off its CU meanwhile
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t n = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(2);
    ++n;
  }
  if (n == 0xffffffffu) sink[threadIdx.x] = n;   // (never true: keeps the loop)
}
}  // namespace

int hx_num_cus() {
  if (!g_ncu) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                 hipSuccess && n > 0)
      g_ncu = n;
    else
      g_ncu = 256;
  }
  return g_ncu;
}

void hx_set_reserved_cus(int r) { g_reserved.store(r < 0 ? 0 : r); }
int hx_reserved_cus() { return g_reserved.load(); }

// workgroup slots of one round for one-workgroup-per-CU kernels
int hx_cu_slots() {
  const int n = hx_num_cus(), r = g_reserved.load();
  return r > 0 && r < n / 2 ? n - r : n;
}

// A stream whose kernels run only on CUs first_cu .. first_cu + count - 1 (logical CU mask
// bits); returns 0 on failure.  The caller owns it (hx_destroy_stream).
hipStream_t hx_cu_masked_stream(int first_cu, int count) {
  const int n = hx_num_cus();
  std::vector<uint32_t> mask((n + 31) / 32, 0u);
  for (int c = first_cu; c < first_cu + count && c < n; ++c) mask[c / 32] |= 1u << (c % 32);
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) return nullptr;
  return s;
}

// A non-blocking stream at HIP priority `prio` (clamped to the device range: least = the lowest,
// e.g. 1 below the default 0; greatest = the highest, -1); returns 0 on failure.  The caller owns it.
hipStream_t hx_priority_stream(int prio) {
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return nullptr;
  const int p = prio > least ? least : (prio < greatest ? greatest : prio);
  hipStream_t s = nullptr;
  if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, p) != hipSuccess) return nullptr;
  return s;
}

void hx_stream_priority_range(int* least, int* greatest) {
  *least = *greatest = 0;
  (void)hipDeviceGetStreamPriorityRange(least, greatest);
}

void hx_destroy_stream(hipStream_t s) {
  if (s) (void)hipStreamDestroy(s);
}

// `blocks` 256-thread workgroups holding `lds_bytes` of LDS each that spin for `us` microseconds
// on stream s (a stand-in for a comm kernel's footprint)
void hx_spin(int blocks, double us, int lds_bytes, uint32_t* sink, hipStream_t s) {
  if (blocks < 1) return;
  static int attr = 0;
  if (lds_bytes > 65536 && attr < lds_bytes) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&spin_k), hipFuncAttributeMaxDynamicSharedMemorySize,
                              lds_bytes);
    attr = lds_bytes;
  }
  spin_k<<<blocks, 256, lds_bytes, s>>>((uint64_t)(us * 100.0), sink);
}
