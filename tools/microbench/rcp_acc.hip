// Accuracy of v_rcp_f64 (__builtin_amdgcn_rcp on double) over [1, 4): max error in ulps
// of the raw instruction and after one / two Newton steps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
__global__ void k(const double* x, double* r0, double* r1, double* r2, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double d = x[i];
  double r = __builtin_amdgcn_rcp(d);
  r0[i] = r;
  double e = __builtin_fma(-d, r, 1.0);
  double ra = __builtin_fma(r, e, r);
  r1[i] = ra;
  e = __builtin_fma(-d, ra, 1.0);
  r2[i] = __builtin_fma(ra, e, ra);
}
int main() {
  const int n = 1 << 22;
  std::vector<double> x(n), a(n), b(n), c(n);
  for (int i = 0; i < n; ++i) x[i] = 1.0 + 3.0 * (i + 0.5) / n;
  double *dx, *d0, *d1, *d2;
  hipMalloc(&dx, n * 8); hipMalloc(&d0, n * 8); hipMalloc(&d1, n * 8); hipMalloc(&d2, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, d0, d1, d2, n);
  hipMemcpy(a.data(), d0, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), d1, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(c.data(), d2, n * 8, hipMemcpyDeviceToHost);
  double m0 = 0, m1 = 0, m2 = 0;
  for (int i = 0; i < n; ++i) {
    long double ex = 1.0L / (long double)x[i];
    double ulp = std::nextafter((double)ex, 2.0) - (double)ex;
    m0 = std::fmax(m0, std::fabs((double)(a[i] - ex)) / ulp);
    m1 = std::fmax(m1, std::fabs((double)(b[i] - ex)) / ulp);
    m2 = std::fmax(m2, std::fabs((double)(c[i] - ex)) / ulp);
  }
  printf("v_rcp_f64 max err: raw %.3g ulp, 1 NR %.3g ulp, 2 NR %.3g ulp\n", m0, m1, m2);
  return 0;
}
