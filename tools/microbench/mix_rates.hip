// Does fp32 / int32 VALU work overlap fp64 MFMA on gfx950? Each SIMD gets one
// MFMA-f64 wave and one VALU wave (fp64 FMA, fp32 FMA or int32 mad).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int KIND>  // 0 fp64 fma, 1 fp32 fma, 2 int32 mad, 3 none
__global__ void __launch_bounds__(512) k(int im, int iv, double a, double b, double* out) {
  const int wave = threadIdx.x >> 6;
  double* o = out + blockIdx.x * blockDim.x + threadIdx.x;
  if (wave < 4) {
    d4 acc[4];
    for (int i = 0; i < 4; ++i) acc[i] = d4{0, 0, 0, 0};
    for (int it = 0; it < im; ++it)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    *o = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
  } else if (KIND == 0) {
    double r[16];
    for (int i = 0; i < 16; ++i) r[i] = a * i;
    for (int it = 0; it < iv; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) r[i] = __builtin_fma(r[i], b, a);
    double s = 0; for (int i = 0; i < 16; ++i) s += r[i]; *o = s;
  } else if (KIND == 1) {
    float r[16]; float fa = (float)a, fb = (float)b;
    for (int i = 0; i < 16; ++i) r[i] = fa * i;
    for (int it = 0; it < iv; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) r[i] = __builtin_fmaf(r[i], fb, fa);
    float s = 0; for (int i = 0; i < 16; ++i) s += r[i]; *o = s;
  } else if (KIND == 2) {
    unsigned r[16]; unsigned ua = (unsigned)threadIdx.x | 1u, ub = 2654435761u;
    for (int i = 0; i < 16; ++i) r[i] = ua * i;
    for (int it = 0; it < iv; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) r[i] = r[i] * ub + ua;
    unsigned s = 0; for (int i = 0; i < 16; ++i) s += r[i]; *o = s;
  }
}
template <int KIND> float run(int im, int iv, double* out) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  k<KIND><<<256, 512>>>(im, iv, 1.0000001, 0.9999999, out);
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) k<KIND><<<256, 512>>>(im, iv, 1.0000001, 0.9999999, out);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); return ms / 5;
}
int main() {
  double* out; hipMalloc(&out, 256 * 512 * 8);
  const int im = 4000;
  float t_m = run<3>(im, 0, out);
  printf("MFMA alone: %.3f ms (%.1f TF)\n", t_m, 256.0 * 4 * im * 4 * 2048 / t_m / 1e9);
  for (int iv : {1000, 4000, 16000}) {
    float t0 = run<0>(im, iv, out), t1 = run<1>(im, iv, out), t2 = run<2>(im, iv, out);
    float v0 = run<0>(0, iv, out), v1 = run<1>(0, iv, out), v2 = run<2>(0, iv, out);
    printf("iv=%d: +fp64 VALU %.3f ms (valu alone %.3f) | +fp32 VALU %.3f (alone %.3f) | +int32 %.3f (alone %.3f)\n",
           iv, t0, v0, t1, v1, t2, v2);
  }
  return 0;
}
