// Exhaustive check of the walk's VALU reciprocal (v_rcp_f64 + Newton + Markstein step)
// against the correctly rounded 1.0 / k for every k in [1, 65535]: prints the mismatches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
__global__ void k_recip(double *out, int n) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (k > n) return;
  const double b = (double)k;
  double y = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-b, y, 1.0);
  out[k - 1] = __builtin_fma(y, e, y);
}
int main() {
  const int n = 65535;
  double *d;
  if (hipMalloc(&d, n * 8) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_recip, dim3((n + 255) / 256), dim3(256), 0, 0, d, n);
  double *h = new double[n];
  if (hipMemcpy(h, d, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int bad = 0;
  for (int k = 1; k <= n; ++k) {
    const double r = 1.0 / (double)k;  // host: IEEE correctly rounded
    if (std::memcmp(&r, &h[k - 1], 8) != 0) {
      if (bad < 10) printf("k=%d gpu=%.17g ref=%.17g\n", k, h[k - 1], r);
      ++bad;
    }
  }
  printf("recip_f64: %d of %d differ from 1.0/k\n", bad, n);
  hipFree(d);
  return bad != 0;
}
