// Do fp64 vector instructions ride in the shadow of the issuing wave's own i8 MFMAs on gfx950?
// (chain_coexec.hip measured fp32 fillers only; the fused pass's vector work is mostly fp64.)
// One wave per SIMD (4 waves, waves go round-robin over the SIMDs), a stream of 1 MFMA + K
// independent vector instructions of one kind, 4 MFMA accumulators in rotation:
//   KIND 0: v_fma_f64   KIND 1: v_cvt_f64_i32   KIND 2: v_fma_f32   KIND 3: v_mul_f64
//   OP 0: v_mfma_i32_16x16x64_i8   OP 1: v_mfma_i32_32x32x32_i8
// Cycles per MFMA of wave 0 (clock64 bracketing its loop, block 0); one workgroup per CU.
// build: hipcc -O3 --offload-arch=gfx950 tools/microbench/f64_fill32.hip -o tools/microbench/f64_fill32
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int OP, int KIND, int K>
__global__ void __launch_bounds__(256) k(int iters, int seed, double da, double db, long long* cyc, double* out) {
  const int tid = threadIdx.x;
  v4i a = {seed + tid, seed + 1, seed + 2, seed + 3}, acc[4];
  v16i bacc[4];
  for (int i = 0; i < 4; ++i) {
    acc[i] = v4i{0, 0, 0, 0};
    for (int j = 0; j < 16; ++j) bacc[i][j] = 0;
  }
  double r[4 * (K > 0 ? K : 1)];
  float rf[4 * (K > 0 ? K : 1)];
  int ri[4 * (K > 0 ? K : 1)];
  for (int i = 0; i < 4 * (K > 0 ? K : 1); ++i) {
    r[i] = da * i * 1e-3 + tid;
    rf[i] = (float)r[i];
    ri[i] = seed * i + tid;
  }
  const float fa = (float)da, fb = (float)db;
  __syncthreads();
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if constexpr (OP == 0) asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %1, %0" : "+v"(acc[m & 3]) : "v"(a));
      else asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %1, %0" : "+v"(bacc[m & 3]) : "v"(a));
#pragma unroll
      for (int f = 0; f < K; ++f) {
        const int j = (m & 3) * K + f;  // each register reused 4 MFMAs later
        if constexpr (KIND == 0) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(r[j]) : "v"(db), "v"(da));
        else if constexpr (KIND == 1) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(r[j]) : "v"(ri[j]));
        else if constexpr (KIND == 2) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(rf[j]) : "v"(fb), "v"(fa));
        else asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r[j]) : "v"(db));
      }
    }
  }
  const long long t1 = clock64();
  double s = 0;
  for (int i = 0; i < 4; ++i) s += acc[i][0] + bacc[i][3];
  for (int i = 0; i < 4 * (K > 0 ? K : 1); ++i) s += r[i] + rf[i];
  out[blockIdx.x * blockDim.x + tid] = s;
  if (blockIdx.x == 0 && tid == 0) *cyc = t1 - t0;
}

template <int OP, int KIND, int K>
void run(const char* what) {
  long long* cyc;
  double* out;
  hipMalloc(&cyc, sizeof(long long));
  hipMalloc(&out, 256 * 256 * sizeof(double));
  const int iters = 2000;
  hipLaunchKernelGGL((k<OP, KIND, K>), dim3(256), dim3(256), 0, 0, iters, 3, 1.0000001, 0.9999999, cyc, out);
  hipLaunchKernelGGL((k<OP, KIND, K>), dim3(256), dim3(256), 0, 0, iters, 3, 1.0000001, 0.9999999, cyc, out);
  long long c = 0;
  hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
  std::printf("%-16s + %d %-14s: %.2f cycles per MFMA\n", OP == 0 ? "i8 16x16x64" : "i8 32x32x32", K, what,
              (double)c / (iters * 8.0));
  hipFree(cyc);
  hipFree(out);
}

template <int OP>
void sweep() {
  run<OP, 0, 0>("none");
  run<OP, 0, 2>("fma_f64");
  run<OP, 0, 4>("fma_f64");
  run<OP, 0, 6>("fma_f64");
  run<OP, 0, 8>("fma_f64");
  run<OP, 1, 4>("cvt_f64_i32");
  run<OP, 1, 8>("cvt_f64_i32");
  run<OP, 3, 4>("mul_f64");
  run<OP, 2, 4>("fma_f32");
  run<OP, 2, 8>("fma_f32");
}

int main() {
  sweep<0>();
  sweep<1>();
  return 0;
}
