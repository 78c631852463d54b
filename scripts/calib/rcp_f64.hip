// Accuracy of v_rcp_f64 (__builtin_amdgcn_rcp on double) on gfx950 against the correctly rounded
// 1/x, over x = vd0 = v * d values of the distance cuts' range (v in (0, 10], d ~ 0.23-0.71 min)
// and over random doubles in [1, 2). Prints the max relative error in units of 2^-52.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

__global__ void k(const double* x, double* r, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) r[i] = __builtin_amdgcn_rcp(x[i]);
}

int main() {
  const int n = 1 << 22;
  std::vector<double> x(n), r(n);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const double u = (double)(s >> 11) * 0x1p-53;
    x[i] = i < n / 2 ? 1.0 + u : (1e-3 + 10.0 * u) * (0.23 + 0.48 * ((i * 2654435761u) % 1000) / 1000.0);
  }
  double *dx, *dr;
  hipMalloc(&dx, n * 8); hipMalloc(&dr, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  k<<<(n + 255) / 256, 256>>>(dx, dr, n);
  hipMemcpy(r.data(), dr, n * 8, hipMemcpyDeviceToHost);
  double worst = 0.0;
  long exact = 0;
  for (int i = 0; i < n; ++i) {
    const double want = 1.0 / x[i];
    const double e = fabs(r[i] - want) / want;
    if (r[i] == want) ++exact;
    if (e > worst) worst = e;
  }
  printf("{\"samples\": %d, \"max_rel_err\": %.3e, \"max_rel_err_ulps_2^-52\": %.1f, \"correctly_rounded_frac\": %.4f}\n",
         n, worst, worst / 0x1p-52, (double)exact / n);
  hipFree(dx); hipFree(dr);
  return 0;
}
