// Why a real kernel does not get the co-issue fill_coexec.hip measures: the fillers there are
// independent; a kernel's row terms are dependency chains, and the SIMD may also hold a second
// wave with MFMAs of its own. One wave per SIMD (or two, ROLE below), a stream of
// 1 MFMA + K fp32 vector instructions:
//   DEP 0: K independent FMAs (each register reused 4 MFMAs later, as in fill_coexec);
//   DEP 1: ONE chain — every filler reads the previous one's result (r = r·a + b), across gaps;
//   DEP 2: two chains interleaved (a, b, a, b, …);
//   DEP 3: ONE chain of v_exp_f32 (transcendental latency).
//   ROLE 0: one wave per SIMD; ROLE 1: a second wave per SIMD issues only v_mfma_f64_16x16x4 (a G
//   wave of the fused pass); ROLE 2: a second wave issuing the same i8 MFMA stream without fillers.
// Cycles per MFMA of wave 0 (s_memtime bracketing its loop, block 0).
//   OP 0: v_mfma_i32_16x16x64_i8   OP 2: v_mfma_i32_32x32x32_i8
// build: hipcc -O3 --offload-arch=gfx950 tools/microbench/chain_coexec.hip -o tools/microbench/chain_coexec
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef double v4d __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int OP, int DEP, int K, int ROLE>
__global__ void __launch_bounds__(512) k(int iters, int seed, float fa, float fb, long long* cyc, int* out) {
  const int tid = threadIdx.x, wave = tid >> 6;
  const bool second = ROLE != 0 && wave >= 4;  // waves 4–7: the second wave of SIMDs 0–3 (waves go round-robin)
  v4i a = {seed + tid, seed + 1, seed + 2, seed + 3}, acc[4];
  v16i bacc[4];
  v4d dacc[4];
  const double da = 1.0 + seed * 1e-9 + tid * 1e-12;
  for (int i = 0; i < 4; ++i) {
    acc[i] = v4i{0, 0, 0, 0};
    dacc[i] = v4d{0, 0, 0, 0};
    for (int j = 0; j < 16; ++j) bacc[i][j] = 0;
  }
  fa += tid * 1e-9f;
  fb -= tid * 1e-9f;
  float r[4 * (K > 0 ? K : 1)];
  for (int i = 0; i < 4 * (K > 0 ? K : 1); ++i) r[i] = fa * i * 1e-3f;
  float c0 = fa, c1 = fb;
  __syncthreads();
  const long long t0 = clock64();
  if (second) {  // outlasts wave 0's stream
    for (int it = 0; it < (ROLE == 1 ? iters : 3 * iters); ++it)
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        if constexpr (ROLE == 1) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %1, %0" : "+v"(dacc[m & 3]) : "v"(da));
        else if constexpr (OP == 0) asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %1, %0" : "+v"(acc[m & 3]) : "v"(a));
        else asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %1, %0" : "+v"(bacc[m & 3]) : "v"(a));
      }
  } else {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        if constexpr (OP == 0) asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %1, %0" : "+v"(acc[m & 3]) : "v"(a));
        else asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %1, %0" : "+v"(bacc[m & 3]) : "v"(a));
#pragma unroll
        for (int f = 0; f < K; ++f) {
          if constexpr (DEP == 0) {
            const int j = (m & 3) * K + f;
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[j]) : "v"(fb), "v"(fa));
          } else if constexpr (DEP == 1) {
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(c0) : "v"(fb), "v"(fa));
          } else if constexpr (DEP == 2) {
            if (f & 1) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(c1) : "v"(fb), "v"(fa));
            else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(c0) : "v"(fb), "v"(fa));
          } else {
            asm volatile("v_exp_f32 %0, %0" : "+v"(c0));
          }
        }
      }
    }
  }
  const long long t1 = clock64();
  int s = 0;
  for (int i = 0; i < 4; ++i) s += acc[i][0] + bacc[i][3] + (int)dacc[i][1];
  float fs = c0 + c1;
  for (int i = 0; i < 4 * (K > 0 ? K : 1); ++i) fs += r[i];
  out[blockIdx.x * blockDim.x + tid] = s + (int)fs;
  if (blockIdx.x == 0 && tid == 0) *cyc = t1 - t0;
}

template <int OP, int DEP, int K, int ROLE>
void run(long long* dcyc, int* out) {
  const int iters = OP == 0 ? 2000 : 1000;
  const int threads = ROLE == 0 ? 256 : 512;  // 1 or 2 waves per SIMD (one workgroup per CU)
  for (int rep = 0; rep < 2; ++rep) {
    k<OP, DEP, K, ROLE><<<256, threads>>>(iters, 3, 1.0000001f, 0.9999999f, dcyc, out);
    (void)hipDeviceSynchronize();
  }
  long long c = 0;
  (void)hipMemcpy(&c, dcyc, sizeof c, hipMemcpyDeviceToHost);
  static const char* dep[] = {"independent", "one chain", "two chains", "exp chain"};
  static const char* role[] = {"alone", "beside an f64-MFMA wave", "beside an i8-MFMA wave"};
  printf("%s + %d %s fillers, wave %s: %.2f cycles per MFMA of wave 0\n", OP == 0 ? "i8 16x16x64" : "i8 32x32x32", K,
         dep[DEP], role[ROLE], (double)c / (iters * 8.0));
}

template <int OP, int ROLE>
void sweep(long long* dcyc, int* out) {
  run<OP, 0, 0, ROLE>(dcyc, out);
  run<OP, 0, 4, ROLE>(dcyc, out);
  run<OP, 1, 2, ROLE>(dcyc, out);
  run<OP, 1, 4, ROLE>(dcyc, out);
  run<OP, 2, 4, ROLE>(dcyc, out);
  run<OP, 3, 2, ROLE>(dcyc, out);
}

int main() {
  int* out;
  long long* dcyc;
  (void)hipMalloc(&out, 256 * 512 * 4);
  (void)hipMalloc(&dcyc, 8);
  sweep<0, 0>(dcyc, out);
  sweep<2, 0>(dcyc, out);
  sweep<0, 1>(dcyc, out);
  sweep<2, 1>(dcyc, out);
  sweep<0, 2>(dcyc, out);
  sweep<2, 2>(dcyc, out);
  return 0;
}
