// MFMA shape vs clock under load: every wave of a full-chip grid runs a long chain of fp16 MFMAs
// on random register operands (8 independent accumulators), v_mfma_f32_32x32x16_f16 vs
// v_mfma_f32_16x16x32_f16 (same flops per instruction pair).  The guide (MI355X_MICROARCH.md,
// DVFS item 7) measured the 16x16x32 bf16 loop ~1.12-1.15x faster in FLOP/s at equal cycles per
// FLOP on random data: the shape changes the clock the chip holds.  This checks it for f16.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_shape_probe tools/probe/mfma_shape_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int SHAPE>
__global__ __launch_bounds__(256) void loop_k(const f16x8* __restrict__ in, float* __restrict__ out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  f16x8 a = in[t & 4095], b = in[(t + 77) & 4095];
  if constexpr (SHAPE == 32) {
    f32x16 acc[4];
    for (int j = 0; j < 4; ++j) acc[j] = f32x16{0};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[j], 0, 0, 0);
    }
    float s = 0.f;
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 16; ++k) s += acc[j][k];
    out[t] = s;
  } else {
    f32x4 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = f32x4{0};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[j], 0, 0, 0);
    }
    float s = 0.f;
    for (int j = 0; j < 8; ++j)
      for (int k = 0; k < 4; ++k) s += acc[j][k];
    out[t] = s;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  const int blocks = 256 * 8;   // 8 waves per SIMD... 2048 workgroups of 4 waves
  f16x8* in;
  float* out;
  hipMalloc(&in, 4096 * sizeof(f16x8));
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
  f16x8* h = (f16x8*)malloc(4096 * sizeof(f16x8));
  srand(1);
  for (int i = 0; i < 4096; ++i)
    for (int k = 0; k < 8; ++k) h[i][k] = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 2e-3f);
  hipMemcpy(in, h, 4096 * sizeof(f16x8), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    for (int shape : {32, 16}) {
      // warm for ~1 s so the clock settles
      for (int w = 0; w < 3; ++w) {
        if (shape == 32) loop_k<32><<<blocks, 256>>>(in, out, iters);
        else loop_k<16><<<blocks, 256>>>(in, out, iters);
      }
      hipEventRecord(e0);
      for (int w = 0; w < 5; ++w) {
        if (shape == 32) loop_k<32><<<blocks, 256>>>(in, out, iters);
        else loop_k<16><<<blocks, 256>>>(in, out, iters);
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      // flops: per wave per iter 4 x (2 32 32 16) or 8 x (2 16 16 32), equal
      const double fl = 5.0 * blocks * 4.0 * iters * 4 * 2.0 * 32 * 32 * 16;
      printf("shape %dx%d: %.3f ms for 5 launches, %.1f TF/s f16\n", shape, shape, ms, fl / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
