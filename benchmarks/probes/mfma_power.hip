// Sustained matrix-core throughput and power of the two bf16 MFMA shapes, register operands only (no memory traffic
// in the loop, four random operand pairs rotated): v_mfma_f32_32x32x16_bf16 vs v_mfma_f32_16x16x32_bf16 on independent accumulator chains, 2 waves per
// SIMD.  Run under benchmarks/probes/mfma_power.py, which samples clock / power / energy while it runs.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_power benchmarks/probes/mfma_power.hip
//   /tmp/mfma_power {16|32} SECONDS
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int ITERS = 4096;

// Four operand pairs of pseudo-random bf16 values (normal-range exponents, random mantissas and signs), rotated over
// the unrolled MFMAs so the multiplier inputs toggle as they do on real data.
__device__ void init_operands(bf16x8 (&a)[4], bf16x8 (&b)[4], float seed) {
  unsigned x = threadIdx.x * 2654435761u + (unsigned)(seed * 1e6f);
  for (int p = 0; p < 4; ++p)
    for (int i = 0; i < 8; ++i) {
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      a[p][i] = (__bf16)((float)(int)(x & 0xffff) * (1.f / 32768.f) - 1.f);
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      b[p][i] = (__bf16)((float)(int)(x & 0xffff) * (1.f / 32768.f) - 1.f);
    }
}

// 128 accumulator registers per wave in both forms (8 x 16 or 32 x 4), the operand count of a 128 x 64 wave tile.
__global__ __launch_bounds__(512, 1) void mfma32_k(float* out, float seed) {
  bf16x8 a[4], b[4];
  init_operands(a, b, seed);
  f32x16 acc[8] = {};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[j & 3], b[(j >> 1) & 3], acc[j], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[j][r];
  if (s == 1234.5f) out[threadIdx.x] = s;   // keeps the chains live
}

__global__ __launch_bounds__(512, 1) void mfma16_k(float* out, float seed) {
  bf16x8 a[4], b[4];
  init_operands(a, b, seed);
  f32x4 acc[32] = {};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < 32; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j & 3], b[(j >> 2) & 3], acc[j], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 32; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) s += acc[j][r];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int shape = argc > 1 ? atoi(argv[1]) : 32;
  const double secs = argc > 2 ? atof(argv[2]) : 3.0;
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  float* out = nullptr;
  hipMalloc(&out, 4096);
  const dim3 grid(cus), block(512);
  // flops per launch: every wave does ITERS x (8 x 32x32x16 = 131072 MACs, or 32 x 16x16x32 = 262144 MACs)
  const double macs = shape == 16 ? 32.0 * 16 * 16 * 32 : 8.0 * 32 * 32 * 16;
  const double flops = 2.0 * cus * 8 * (double)ITERS * macs;
  auto launch = [&] {
    if (shape == 16) hipLaunchKernelGGL(mfma16_k, grid, block, 0, 0, out, 1e-3f);
    else hipLaunchKernelGGL(mfma32_k, grid, block, 0, 0, out, 1e-3f);
  };
  launch();
  hipDeviceSynchronize();
  const auto t0 = std::chrono::steady_clock::now();
  long n = 0;
  double el = 0.0;
  while (el < secs) {
    for (int i = 0; i < 10; ++i) launch();
    hipDeviceSynchronize();
    n += 10;
    el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  printf("{\"shape\": %d, \"launches\": %ld, \"seconds\": %.3f, \"tflops\": %.1f}\n", shape, n, el,
         flops * n / el / 1e12);
  hipFree(out);
  return 0;
}
