// Semantics of v_cvt_pk_u8_f32 on the box (clamping and rounding), for the score-bound
// kernel's per-column 8-bit bounds (csrc/gbound.hip): prints each input and its byte.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(const float *x, unsigned *y, int n) {
  const int i = threadIdx.x;
  if (i < n) y[i] = __builtin_amdgcn_cvt_pk_u8_f32(x[i], 0, 0u);
}

int main() {
  const float h[] = {-5.f, -0.4f, -0.6f, 0.f, 0.3f, 0.5f, 0.7f, 1.5f, 2.5f, 3.5f, 254.4f, 254.5f,
                     254.6f, 255.f, 255.4f, 255.6f, 256.f, 300.f, 1e9f, __builtin_nanf(""),
                     __builtin_inff(), -__builtin_inff(), 1e-30f, 7.999999f};
  const int n = sizeof(h) / sizeof(h[0]);
  float *dx;
  unsigned *dy, hy[64];
  if (hipMalloc(&dx, sizeof(h)) != hipSuccess || hipMalloc(&dy, 64 * 4) != hipSuccess) return 1;
  if (hipMemcpy(dx, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
  k<<<1, 64>>>(dx, dy, n);
  if (hipMemcpy(hy, dy, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int i = 0; i < n; ++i) printf("cvt_pk_u8(%.7g) = %u\n", h[i], hy[i] & 0xFF);
  return 0;
}
