// The shader clock the chip holds under a sustained MFMA stream on every SIMD (power), by MFMA
// kind: cycles (clock64 of wave 0 of block 0) over wall time (HIP events) of a ≈ 0.2–0.5 s launch,
// 256 workgroups × 256 threads (one wave per SIMD) or × 512 (two). Also i8 MFMAs with vector
// fillers and an fp64 + i8 mix (what a G-on-digits fused pass would run).
// build: hipcc -O3 --offload-arch=gfx950 tools/microbench/mfma_clock.hip -o tools/microbench/mfma_clock
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef double v4d __attribute__((ext_vector_type(4)));

// KIND 0: i8 16x16x64; 1: fp64 16x16x4; 2: i8 16x16x64 + 2 fp32 FMA fillers; 3: fp64 and i8
// alternating (1 : 4, the MAC-time ratio of the fused pass's G and Y stages)
template <int KIND>
__global__ void __launch_bounds__(512) k(int iters, int seed, long long* cyc, int* out) {
  const int tid = threadIdx.x;
  // random-looking operands that change every iteration (multiplier toggling, as real digits do)
  unsigned h = (unsigned)(tid + 1) * 2654435761u ^ (unsigned)blockIdx.x * 40503u;
  v4i a = {(int)h, (int)(h * 2246822519u), (int)(h * 3266489917u), (int)(h * 668265263u)}, acc[4];
  v4d dacc[4];
  double da = 1.0 + (h & 0xffff) * 1e-5;
  float r0 = tid * 1e-3f, r1 = r0 + 1.f;
  for (int i = 0; i < 4; ++i) {
    acc[i] = v4i{0, 0, 0, 0};
    dacc[i] = v4d{0, 0, 0, 0};
  }
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    const unsigned u = (unsigned)it;
    a ^= v4i{(int)(u * 0x9E3779B1u), (int)(u * 0x85EBCA77u), (int)(u * 0xC2B2AE3Du), (int)(u * 0x27D4EB2Fu)};
    if constexpr (KIND == 1 || KIND == 3) da = __builtin_fma(da, 0.9999999, 1e-7 * (it & 7));
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if constexpr (KIND == 1) {
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %1, %0" : "+v"(dacc[m & 3]) : "v"(da));
      } else if constexpr (KIND == 3) {
        if (m == 0) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %1, %0" : "+v"(dacc[0]) : "v"(da));
        else asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %1, %0" : "+v"(acc[m & 3]) : "v"(a));
      } else {
        asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %1, %0" : "+v"(acc[m & 3]) : "v"(a));
        if constexpr (KIND == 2) {
          asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(r0) : "v"(r1));
          asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(r1) : "v"(r0));
        }
      }
    }
  }
  const long long t1 = clock64();
  int s = 0;
  for (int i = 0; i < 4; ++i) s += acc[i][0] + (int)dacc[i][0];
  out[blockIdx.x * blockDim.x + tid] = s + (int)(r0 + r1);
  if (blockIdx.x == 0 && tid == 0) *cyc = t1 - t0;
}

template <int KIND>
void run(int threads, int iters, long long* dcyc, int* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<KIND><<<256, threads>>>(iters / 10, 1, dcyc, out);  // warm up
  hipDeviceSynchronize();
  hipEventRecord(e0);
  k<KIND><<<256, threads>>>(iters, 1, dcyc, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  long long c = 0;
  hipMemcpy(&c, dcyc, sizeof c, hipMemcpyDeviceToHost);
  static const char* nm[] = {"i8 16x16x64", "f64 16x16x4", "i8 16x16x64 + 2 fp32 FMA", "f64 : i8 = 1 : 7 instructions"};
  printf("%-32s %d waves/SIMD: %8.2f ms, %.3e cycles of wave 0 -> %.2f GHz\n", nm[KIND], threads / 256, ms, (double)c,
         c / (ms * 1e-3) / 1e9);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  int* out;
  long long* dcyc;
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&dcyc, 8);
  for (int th : {256}) {
    run<0>(th, 1500000 / (th / 256), dcyc, out);
    run<1>(th, 400000 / (th / 256), dcyc, out);
    run<2>(th, 1200000 / (th / 256), dcyc, out);
    run<3>(th, 800000 / (th / 256), dcyc, out);
  }
  return 0;
}
