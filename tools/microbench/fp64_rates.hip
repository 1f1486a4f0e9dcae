// Microbenchmark: fp64 MFMA vs fp64 VALU FMA throughput on gfx950, alone and
// co-resident, plus an HBM streaming-read roof. Used to pick the design of
// the fused Picard evaluation pass (see DESIGN.md "Measured roofs").
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

template <int NACC>
__device__ __forceinline__ void mfma_loop(int iters, double a, double b, double* out) {
  d4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  *out = s;
}

__device__ __forceinline__ void valu_loop(int iters, double a, double b, double* out) {
  double r[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = a * (i + 1);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int i = 0; i < 16; ++i) r[i] = __builtin_fma(r[i], b, a);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += r[i];
  *out = s;
}

// mode 0: all waves MFMA; 1: all waves VALU; 2: half waves MFMA, half VALU;
// 3: each wave interleaves both.
__global__ void __launch_bounds__(512) k_rates(int mode, int iters_m, int iters_v, double a, double b, double* out) {
  int wave = threadIdx.x >> 6;
  int nw = blockDim.x >> 6;
  double* o = out + blockIdx.x * blockDim.x + threadIdx.x;
  if (mode == 0) {
    mfma_loop<4>(iters_m, a, b, o);
  } else if (mode == 1) {
    valu_loop(iters_v, a, b, o);
  } else if (mode == 2) {
    if (wave < nw / 2) mfma_loop<4>(iters_m, a, b, o);
    else valu_loop(iters_v, a, b, o);
  } else {
    double t1, t2;
    mfma_loop<4>(iters_m, a, b, &t1);
    valu_loop(iters_v, a, b, &t2);
    *o = t1 + t2;
  }
}

// Interleaved in one loop body: 4 MFMA + 16*K VALU FMAs per iteration.
template <int KV>
__global__ void __launch_bounds__(256) k_inter(int iters, double a, double b, double* out) {
  d4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = d4{0, 0, 0, 0};
  double r[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = a * (i + 1);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
#pragma unroll
      for (int k = 0; k < KV; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) r[i * 4 + j] = __builtin_fma(r[i * 4 + j], b, a);
    }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
#pragma unroll
  for (int i = 0; i < 16; ++i) s += r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_stream(const double2* __restrict__ x, size_t n2, double* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  double2 s = {0, 0};
  for (; i < n2; i += stride) { double2 v = x[i]; s.x += v.x; s.y += v.y; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}

static float time_launch(void (*f)(void*), void* ctx, int reps) {
  hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  f(ctx); CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f(ctx);
  CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

struct RatesCtx { int mode, im, iv, blocks, threads; double* out; };
static void run_rates(void* p) {
  RatesCtx* c = (RatesCtx*)p;
  k_rates<<<c->blocks, c->threads>>>(c->mode, c->im, c->iv, 1.0000001, 0.9999999, c->out);
}
template <int KV> struct InterCtx { int iters, blocks; double* out; };
template <int KV> static void run_inter(void* p) {
  InterCtx<KV>* c = (InterCtx<KV>*)p;
  k_inter<KV><<<c->blocks, 256>>>(c->iters, 1.0000001, 0.9999999, c->out);
}
struct StreamCtx { const double2* x; size_t n2; double* out; };
static void run_stream(void* p) {
  StreamCtx* c = (StreamCtx*)p;
  k_stream<<<256 * 8, 256>>>(c->x, c->n2, c->out);
}

int main() {
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  int cus = prop.multiProcessorCount;
  double* out; CHECK(hipMalloc(&out, sizeof(double) * 4096 * 1024));
  const int threads = 512;
  for (int bpc = 1; bpc <= 2; ++bpc) {
    int blocks = cus * bpc;
    int im = 2000, iv = 1000;
    // flops: MFMA wave-iter = 4 * 2048 flop; VALU thread-iter = 64 FMA = 128 flop
    for (int mode = 0; mode < 4; ++mode) {
      RatesCtx c{mode, im, iv, blocks, threads, out};
      float ms = time_launch(run_rates, &c, 5);
      double waves = (double)blocks * threads / 64;
      double mf = 0, vf = 0;
      if (mode == 0) mf = waves * im * 4 * 2048.0;
      if (mode == 1) vf = waves * 64 * iv * 128.0;
      if (mode == 2) { mf = waves / 2 * im * 4 * 2048.0; vf = waves / 2 * 64 * iv * 128.0; }
      if (mode == 3) { mf = waves * im * 4 * 2048.0; vf = waves * 64 * iv * 128.0; }
      printf("rates bpc=%d mode=%d: %.3f ms  mfma %.1f TF  valu %.1f TF  total %.1f TF\n", bpc, mode, ms,
             mf / ms / 1e9, vf / ms / 1e9, (mf + vf) / ms / 1e9);
    }
  }
  {
    int blocks = cus * 2, iters = 2000;
    InterCtx<0> c0{iters, blocks, out};
    float ms0 = time_launch(run_inter<0>, &c0, 5);
    double w = blocks * 4.0;
    printf("inter KV=0: %.3f ms mfma %.1f TF\n", ms0, w * iters * 4 * 2048.0 / ms0 / 1e9);
    InterCtx<1> c1{iters, blocks, out};
    float ms1 = time_launch(run_inter<1>, &c1, 5);
    printf("inter KV=1: %.3f ms mfma %.1f TF valu %.1f TF\n", ms1, w * iters * 4 * 2048.0 / ms1 / 1e9,
           w * 64 * iters * 16 * 2.0 / ms1 / 1e9);
    InterCtx<2> c2{iters, blocks, out};
    float ms2 = time_launch(run_inter<2>, &c2, 5);
    printf("inter KV=2: %.3f ms mfma %.1f TF valu %.1f TF\n", ms2, w * iters * 4 * 2048.0 / ms2 / 1e9,
           w * 64 * iters * 32 * 2.0 / ms2 / 1e9);
    InterCtx<4> c4{iters, blocks, out};
    float ms4 = time_launch(run_inter<4>, &c4, 5);
    printf("inter KV=4: %.3f ms mfma %.1f TF valu %.1f TF\n", ms4, w * iters * 4 * 2048.0 / ms4 / 1e9,
           w * 64 * iters * 64 * 2.0 / ms4 / 1e9);
  }
  {
    size_t bytes = (size_t)4 << 30;
    double2* x; CHECK(hipMalloc(&x, bytes)); CHECK(hipMemset(x, 0, bytes));
    StreamCtx c{x, bytes / 16, out};
    float ms = time_launch(run_stream, &c, 5);
    printf("stream read 4 GiB: %.3f ms  %.1f GB/s\n", ms, bytes / ms / 1e6);
    CHECK(hipFree(x));
  }
  return 0;
}
