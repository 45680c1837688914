// LDS scatter-add rates on this part: each wave adds to random columns of its own 2048-entry
// accumulator (the K3s walk's acc), as ds_add_f64 / ds_add_u64 / ds_add_f32 / plain
// ds_write_b64, with 2..16 waves per CU. Build: hipcc -O3 --offload-arch=gfx950
// lds_atomic.hip -o lds_atomic; prints G adds/s chip-wide and LDS cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int kCols = 2048;

// MODE 0 / 4 / 5: ds_add_f64 with all lanes at random columns / ~45 % of the lanes active
// (random mask, the walk's slot density) / all lanes at consecutive columns (conflict-free)
template <int MODE>
__global__ __launch_bounds__(1024) void k_scatter(double *out, int iters, uint32_t seed) {
  extern __shared__ double lds[];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  double *acc = lds + wave * kCols;
  for (int j = lane; j < kCols; j += 64) acc[j] = 0.0;
  __syncthreads();
  uint32_t x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
  const double v = 1.0 + lane;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      x = x * 1664525u + 1013904223u;
      const uint32_t c = (x >> 8) & (kCols - 1);
      if constexpr (MODE == 0)
        __hip_atomic_fetch_add(&acc[c], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else if constexpr (MODE == 4) {
        if (((x >> 3) & 15) < 7)  // 7 / 16 of the lanes
          __hip_atomic_fetch_add(&acc[c], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if constexpr (MODE == 5)
        __hip_atomic_fetch_add(&acc[(lane + 64 * s) & (kCols - 1)], v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      else if constexpr (MODE == 1)
        __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(acc) + c, 3ull,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else if constexpr (MODE == 2)
        __hip_atomic_fetch_add(reinterpret_cast<float *>(acc) + c, 1.5f, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      else
        acc[c] = v;
    }
  }
  __syncthreads();
  double r = 0.0;
  for (int j = lane; j < kCols; j += 64) r += acc[j];
  if (r == 1.2345) out[threadIdx.x] = r;
}

template <int MODE>
static void run(const char *name, double *out, int cus) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 2000;
  for (int w = 2; w <= 16; w *= 2) {
    const size_t lds = (size_t)w * kCols * 8;
    if (lds > 160 * 1024) break;
    hipFuncSetAttribute((const void *)k_scatter<MODE>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      k_scatter<MODE><<<cus, 64 * w, lds>>>(out, iters, 1234u + rep);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double adds = (double)cus * w * 64 * iters * 16;
    const double winstr = (double)w * iters * 16;  // per CU
    printf("%-12s waves/CU %2d: %8.1f G adds/s, %6.1f cycles per wave-instruction per CU "
           "(2.4 GHz)\n", name, w, adds / best / 1e6, best * 1e-3 * 2.4e9 / winstr);
  }
}

int main() {
  double *out;
  hipMalloc(&out, 1024 * sizeof(double));
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  run<0>("ds_add_f64", out, cus);
  run<4>("add_f64 45%", out, cus);
  run<5>("add_f64 seq", out, cus);
  run<1>("ds_add_u64", out, cus);
  run<2>("ds_add_f32", out, cus);
  run<3>("ds_write_b64", out, cus);
  return 0;
}
