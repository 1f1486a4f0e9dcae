// How many VALU instructions hide inside the gap of an MFMA when they come from the SAME wave
// (interleaved with __builtin_amdgcn_sched_group_barrier: 1 MFMA, then K fillers), against the
// cross-wave case of agpr_coexec.hip (an MFMA wave beside a VALU wave: fully serialised).
// W waves per SIMD (W = 1: 256 threads, W = 2: 512, W = 4: 1024), every wave runs the same
// stream; cycles per MFMA per SIMD from s_memtime (shader clock) of wave 0 of block 0.
//   OP 0: v_mfma_i32_16x16x64_i8 (16 cyc)   OP 1: v_mfma_f64_16x16x4_f64 (64 cyc)
//   OP 2: v_mfma_i32_32x32x32_i8 (32 cyc, the same MACs as two 16x16x64)
//   F 0: v_fma_f32 fillers   F 1: v_exp_f32 fillers   F 2: v_fma_f64 fillers
// build: hipcc -O3 --offload-arch=gfx950 tools/microbench/fill_coexec.hip -o tools/microbench/fill_coexec
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef double v4d __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int OP, int F, int K>
__global__ void __launch_bounds__(1024) k(int iters, int seed, float fa, float fb, long long* cyc, int* out) {
  int* o = out + blockIdx.x * blockDim.x + threadIdx.x;
  const int tid = threadIdx.x;  // lane-varying operands stay in VGPRs (no re-materialisation)
  v4i a = {seed + tid, seed + 1, seed + 2, seed + 3}, acc[4];
  fa += tid * 1e-9f;
  fb -= tid * 1e-9f;
  v4d dacc[4];
  v16i bacc[4];
  const double da = 1.0 + seed * 1e-9 + tid * 1e-12;
  const double dfa = fa, dfb = fb;
  for (int i = 0; i < 4; ++i) {
    acc[i] = v4i{0, 0, 0, 0};
    dacc[i] = v4d{0, 0, 0, 0};
    for (int j = 0; j < 16; ++j) bacc[i][j] = 0;
  }
  float r[4 * (K > 0 ? K : 1)];
  double rd[4 * (K > 0 ? K : 1)];
  for (int i = 0; i < 4 * (K > 0 ? K : 1); ++i) {
    r[i] = fa * i * 1e-3f;
    rd[i] = fa * i;
  }
  __syncthreads();
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      // inline asm keeps the program order exactly (volatile asm is not reordered); the
      // accumulators rotate over 4 (each reused 4 MFMAs later: no hazard padding needed)
      if constexpr (OP == 0) asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %1, %0" : "+v"(acc[m & 3]) : "v"(a));
      else if constexpr (OP == 1) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %1, %0" : "+v"(dacc[m & 3]) : "v"(da));
      else asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %1, %0" : "+v"(bacc[m & 3]) : "v"(a));
#pragma unroll
      for (int f = 0; f < K; ++f) {
        const int j = (m & 3) * K + f;  // reused 4 MFMAs later (independent in between)
        if constexpr (F == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[j]) : "v"(fb), "v"(fa));
        else if constexpr (F == 1) asm volatile("v_exp_f32 %0, %0" : "+v"(r[j]));
        else asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(rd[j]) : "v"(dfb), "v"(dfa));
      }
    }
  }
  const long long t1 = clock64();
  int s = 0;
  for (int i = 0; i < 4; ++i) s += acc[i][0] + (int)dacc[i][0] + bacc[i][5];
  float fs = 0;
  for (int i = 0; i < 4 * (K > 0 ? K : 1); ++i) fs += r[i] + (float)rd[i];
  *o = s + (int)fs;
  if (blockIdx.x == 0 && threadIdx.x == 0) *cyc = t1 - t0;
}

template <int OP, int F, int K>
void run(int waves, long long* dcyc, int* out) {
  const int iters = OP == 0 ? 2000 : OP == 2 ? 1000 : 500;
  k<OP, F, K><<<256, 256 * waves>>>(iters, 3, 1.0000001f, 0.9999999f, dcyc, out);
  (void)hipDeviceSynchronize();
  k<OP, F, K><<<256, 256 * waves>>>(iters, 3, 1.0000001f, 0.9999999f, dcyc, out);
  (void)hipDeviceSynchronize();
  long long c = 0;
  (void)hipMemcpy(&c, dcyc, sizeof c, hipMemcpyDeviceToHost);
  const double per = (double)c / (iters * 8.0 * waves);  // cycles per MFMA on the SIMD
  printf("%s W=%d filler=%s K=%d: %.2f cyc per MFMA per SIMD (%.2f per MFMA+%d fillers of one wave)\n",
         OP == 0 ? "i8 16x16x64" : OP == 1 ? "f64 16x16x4" : "i8 32x32x32", waves, F == 0 ? "fma_f32" : F == 1 ? "exp_f32" : "fma_f64", K, per,
         per * waves, K);
}

template <int OP, int F>
void sweep(long long* dcyc, int* out) {
  for (int w : {1, 2, 4}) {
    run<OP, F, 0>(w, dcyc, out);
    run<OP, F, 1>(w, dcyc, out);
    run<OP, F, 2>(w, dcyc, out);
    run<OP, F, 3>(w, dcyc, out);
    run<OP, F, 4>(w, dcyc, out);
    run<OP, F, 6>(w, dcyc, out);
    if (OP == 2) run<OP, F, 8>(w, dcyc, out);
  }
}

int main() {
  int* out;
  long long* dcyc;
  (void)hipMalloc(&out, 256 * 1024 * 4);
  (void)hipMalloc(&dcyc, 8);
  if (getenv("FILL_ONLY_32")) {
    sweep<2, 0>(dcyc, out);
    sweep<2, 1>(dcyc, out);
    return 0;
  }
  sweep<0, 0>(dcyc, out);
  sweep<0, 1>(dcyc, out);
  sweep<1, 0>(dcyc, out);
  sweep<1, 2>(dcyc, out);
  sweep<2, 0>(dcyc, out);
  sweep<2, 1>(dcyc, out);
  return 0;
}
