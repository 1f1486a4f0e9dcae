// How much vector issue does an i8 MFMA hold on gfx950, 16x16x64 vs 32x32x32?
// Each SIMD gets one MFMA wave (M = 0: v_mfma_i32_16x16x64_i8, 1: v_mfma_i32_32x32x32_i8,
// 2: none) and one VALU wave (fp32 FMA stream, V = 1; v_exp_f32 stream, V = 2; none, V = 0).
// Same MACs per MFMA wave for both shapes (one 32x32x32 = two 16x16x64).
// build: hipcc -O3 --offload-arch=gfx950 tools/microbench/i8_hold.hip -o tools/microbench/i8_hold
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
template <int M, int V>
__global__ void __launch_bounds__(512) k(int im, int iv, int seed, float fa, float fb, int* out) {
  const int wave = threadIdx.x >> 6;
  int* o = out + blockIdx.x * blockDim.x + threadIdx.x;
  if (wave < 4) {
    if (M == 0) {
      v4i a = {seed, seed + 1, seed + 2, seed + 3}, acc[8];
      for (int i = 0; i < 8; ++i) acc[i] = v4i{0, 0, 0, 0};
      for (int it = 0; it < im; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, acc[i], 0, 0, 0);
      int s = 0;
      for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][3];
      *o = s;
    } else if (M == 1) {
      v4i a = {seed, seed + 1, seed + 2, seed + 3};
      v16i acc[4];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 16; ++j) acc[i][j] = 0;
      for (int it = 0; it < im; ++it)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, acc[i], 0, 0, 0);
      int s = 0;
      for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][15];
      *o = s;
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
  }
}
template <int M, int V>
float run(int im, int iv, int* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k<M, V><<<256, 512>>>(im, iv, 3, 1.0000001f, 0.9999999f, out);
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) k<M, V><<<256, 512>>>(im, iv, 3, 1.0000001f, 0.9999999f, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}
int main() {
  int* out;
  hipMalloc(&out, 256 * 512 * 4);
  const int im = 2000;  // 16x16x64: 16000 MFMAs per wave; 32x32x32: 8000 (same MACs)
  const float m0 = run<0, 0>(im, 0, out), m1 = run<1, 0>(im, 0, out);
  printf("MFMA alone: 16x16x64 %.3f ms, 32x32x32 %.3f ms\n", m0, m1);
  for (int iv : {500, 1000, 2000, 4000}) {
    const float f = run<2, 1>(0, iv, out), e = run<2, 2>(0, iv, out);
    const float f0 = run<0, 1>(im, iv, out), f1 = run<1, 1>(im, iv, out);
    const float e0 = run<0, 2>(im, iv, out), e1 = run<1, 2>(im, iv, out);
    printf("iv=%d (%d VALU/wave): fma alone %.3f | +16x16 %.3f +32x32 %.3f || exp alone %.3f | +16x16 %.3f +32x32 %.3f\n",
           iv, iv * 16, f, f0, f1, e, e0, e1);
  }
  return 0;
}
