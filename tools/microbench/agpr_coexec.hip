// Does an MFMA accumulating in AGPRs (the accumulation register file) leave more vector issue
// to a co-resident VALU wave than the same MFMA accumulating in VGPRs? (tools/microbench/
// i8_hold.hip measured ≈ 11.5 of the 16 cycles of v_mfma_i32_16x16x64_i8 held with VGPR
// accumulators.) One MFMA wave and one VALU wave per SIMD; times in shader cycles (s_memtime
// deltas of wave 0 of block 0) and wall ms.
//   MODE 0: i8 MFMA, VGPR acc      MODE 1: i8 MFMA, AGPR acc (inline asm, "+a")
//   MODE 2: f64 MFMA, VGPR acc     MODE 3: f64 MFMA, AGPR acc
//   MODE 4: no MFMA
//   V 0: none, 1: fp32 FMA stream (16 chains), 2: v_exp_f32 stream, 3: fp64 FMA stream
// build: hipcc -O3 --offload-arch=gfx950 tools/microbench/agpr_coexec.hip -o tools/microbench/agpr_coexec
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef double v4d __attribute__((ext_vector_type(4)));

template <int MODE, int V>
__global__ void __launch_bounds__(512) k(int im, int iv, int seed, float fa, float fb, long long* cyc, int* out) {
  const int wave = threadIdx.x >> 6;
  int* o = out + blockIdx.x * blockDim.x + threadIdx.x;
  const long long t0 = clock64();
  if (wave < 4) {
    if constexpr (MODE == 0 || MODE == 1) {
      v4i a = {seed, seed + 1, seed + 2, seed + 3}, acc[8];
      for (int i = 0; i < 8; ++i) acc[i] = v4i{0, 0, 0, 0};
      for (int it = 0; it < im; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if constexpr (MODE == 0) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, acc[i], 0, 0, 0);
          else asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %1, %0" : "+a"(acc[i]) : "v"(a));
        }
      int s = 0;
      for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][3];
      *o = s;
    } else if constexpr (MODE == 2 || MODE == 3) {
      double a = 1.0 + seed * 1e-9;
      v4d acc[8];
      for (int i = 0; i < 8; ++i) acc[i] = v4d{0, 0, 0, 0};
      for (int it = 0; it < im / 4; ++it)  // 64-cycle MFMA: a quarter as many for the same matrix time
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if constexpr (MODE == 2) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, acc[i], 0, 0, 0);
          else asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %1, %0" : "+a"(acc[i]) : "v"(a));
        }
      double s = 0;
      for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][3];
      *o = (int)s;
    }
  } else if (V == 1) {
    float r[16];
    for (int i = 0; i < 16; ++i) r[i] = fa * i;
    for (int it = 0; it < iv; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) r[i] = __builtin_fmaf(r[i], fb, fa);
    float s = 0;
    for (int i = 0; i < 16; ++i) s += r[i];
    *o = (int)s;
  } else if (V == 2) {
    float r[16];
    for (int i = 0; i < 16; ++i) r[i] = -fa * i * 1e-3f;
    for (int it = 0; it < iv; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) r[i] = __builtin_amdgcn_exp2f(r[i]) - 1.0f;
    float s = 0;
    for (int i = 0; i < 16; ++i) s += r[i];
    *o = (int)s;
  } else if (V == 3) {
    double r[16];
    for (int i = 0; i < 16; ++i) r[i] = fa * i;
    for (int it = 0; it < iv / 2; ++it)  // fp64 FMA: half rate
#pragma unroll
      for (int i = 0; i < 16; ++i) r[i] = __builtin_fma(r[i], (double)fb, (double)fa);
    double s = 0;
    for (int i = 0; i < 16; ++i) s += r[i];
    *o = (int)s;
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) *cyc = clock64() - t0;
}

template <int MODE, int V>
void run(const char* name, int im, int iv, long long* dcyc, int* out) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  k<MODE, V><<<256, 512>>>(im, iv, 3, 1.0000001f, 0.9999999f, dcyc, out);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int r = 0; r < 5; ++r) k<MODE, V><<<256, 512>>>(im, iv, 3, 1.0000001f, 0.9999999f, dcyc, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  long long c = 0;
  (void)hipMemcpy(&c, dcyc, sizeof c, hipMemcpyDeviceToHost);
  printf("%-34s %8.4f ms  %10lld cycles  %.2f GHz\n", name, ms / 5, c, c / (ms / 5 * 1e-3) / 1e9);
}

int main() {
  int* out;
  long long* dcyc;
  (void)hipMalloc(&out, 256 * 512 * 4);
  (void)hipMalloc(&dcyc, 8);
  const int im = 2000;  // i8: 16000 MFMAs per wave (256,000 matrix cycles); f64: 4000 (256,000)
  const int iv = 4000;  // 64,000 VALU instructions per wave (fp64 stream: 32,000 at half rate)
  run<0, 0>("i8 MFMA (VGPR acc) alone", im, 0, dcyc, out);
  run<1, 0>("i8 MFMA (AGPR acc) alone", im, 0, dcyc, out);
  run<2, 0>("f64 MFMA (VGPR acc) alone", im, 0, dcyc, out);
  run<3, 0>("f64 MFMA (AGPR acc) alone", im, 0, dcyc, out);
  run<4, 1>("fp32 FMA alone", 0, iv, dcyc, out);
  run<4, 2>("v_exp_f32 alone", 0, iv, dcyc, out);
  run<4, 3>("fp64 FMA alone", 0, iv, dcyc, out);
  run<0, 1>("i8 VGPR acc + fp32 FMA", im, iv, dcyc, out);
  run<1, 1>("i8 AGPR acc + fp32 FMA", im, iv, dcyc, out);
  run<0, 2>("i8 VGPR acc + v_exp_f32", im, iv, dcyc, out);
  run<1, 2>("i8 AGPR acc + v_exp_f32", im, iv, dcyc, out);
  run<2, 1>("f64 VGPR acc + fp32 FMA", im, iv, dcyc, out);
  run<3, 1>("f64 AGPR acc + fp32 FMA", im, iv, dcyc, out);
  run<2, 3>("f64 VGPR acc + fp64 FMA", im, iv, dcyc, out);
  run<3, 3>("f64 AGPR acc + fp64 FMA", im, iv, dcyc, out);
  return 0;
}
