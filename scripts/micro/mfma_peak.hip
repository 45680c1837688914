// Attainable f32 MFMA rate on this part: independent v_mfma_f32_16x16x4_f32 chains from
// registers (no memory), 1..4 waves per SIMD. Build: hipcc -O3 --offload-arch=gfx950
// mfma_peak.hip -o mfma_peak; prints TFLOP/s per configuration.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int CHAINS>
__global__ __launch_bounds__(256) void k_mfma(float *out, int iters, float seed) {
  f32x4 acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a = seed * threadIdx.x, b = seed + threadIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int s = 0; s < 16; ++s)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c)
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
  }
  float r = 0.f;
  for (int c = 0; c < CHAINS; ++c) r += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  if (r == 12345.f) out[threadIdx.x] = r;
}

int main() {
  float *out;
  hipMalloc(&out, 1024 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 4000;
  for (int wps = 1; wps <= 4; ++wps) {
    const int blocks = cus * wps;  // 4 waves per block = one per SIMD
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      k_mfma<2><<<blocks, 256>>>(out, iters, 1e-3f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double flops = 2.0 * 16 * 16 * 4 * 16 * 2 * (double)iters * blocks * 4;
      if (rep) printf("waves/SIMD %d (2 chains): %.1f TFLOP/s (%.3f ms)\n", wps, flops / ms / 1e9, ms);
    }
  }
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    k_mfma<4><<<cus * 2, 256>>>(out, iters, 1e-3f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 16 * 16 * 4 * 16 * 4 * (double)iters * cus * 2 * 4;
    if (rep) printf("waves/SIMD 2 (4 chains): %.1f TFLOP/s (%.3f ms)\n", flops / ms / 1e9, ms);
  }
  return 0;
}
