// Microbenchmark: fp64 MFMA throughput vs the number of independent
// accumulator chains per wave and the number of waves per SIMD. Decides how
// many chains the Y stage of the fused pass needs (each extra chain costs
// VALU adds to combine).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

template <int NACC>
__global__ void __launch_bounds__(512) k_chain(int iters, double a, double b, double* out) {
  d4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8 / NACC; ++k)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
static void run(int cus, int threads, double* out) {
  const int iters = 4000;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  k_chain<NACC><<<cus, threads>>>(iters, 1.0000001, 0.9999999, out);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) k_chain<NACC><<<cus, threads>>>(iters, 1.0000001, 0.9999999, out);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 5;
  const double flops = (double)cus * threads / 64 * iters * 8 * 2048.0;
  printf("chains=%d waves/SIMD=%d: %.3f ms  %.1f TF\n", NACC, threads / 256, ms, flops / ms / 1e9);
}

int main() {
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  double* out; CHECK(hipMalloc(&out, sizeof(double) * cus * 512));
  for (int threads : {256, 512}) {
    run<1>(cus, threads, out);
    run<2>(cus, threads, out);
    run<4>(cus, threads, out);
    run<8>(cus, threads, out);
  }
  return 0;
}
