// Streaming read bandwidth of the screen's staging pattern: each workgroup (512 threads, 8 waves)
// reads its own contiguous range of a large buffer in steps; per step every wave issues P
// 1-KiB pieces (64 lanes x 16 B), into LDS by raw buffer loads (MODE 0, the screen kernels'
// staging) or into registers by 16-B global loads (MODE 1), keeping D steps in flight (a ring
// of D + 1 LDS slots, counted vmcnt). Question answered: is ~3 TB/s (the screens' rate,
// profiles/r04_b) the ceiling of this access pattern, and how much in flight does HBM need?
// build: hipcc -O3 --offload-arch=gfx950 tools/microbench/dma_stream.hip -o tools/microbench/dma_stream
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr;

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else static_assert(N < 0, "vmcnt");
}

// bytes per workgroup step: 8 waves x P KiB
template <int MODE, int P, int D>
__global__ void __launch_bounds__(512) k_stream(const uint8_t* buf, uint64_t per_wg, int* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr uint32_t STEP = 8u * P * 1024u;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint8_t* base = buf + (uint64_t)blockIdx.x * per_wg;
  const uint32_t nsteps = (uint32_t)(per_wg / STEP);
  int acc = 0;
  if constexpr (MODE == 0) {
    // raw buffer resource over this workgroup's range (offsets < 2^31), uniform in SGPRs
    uint64_t bp = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bp), hi = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    const uint8_t* ub = (const uint8_t*)(((uint64_t)hi << 32) | lo);
    __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)ub, 0, (int)per_wg, 0x00020000);
    auto issue = [&](uint32_t k) {
      const uint32_t slot = k % (D + 1);
#pragma unroll
      for (int q = 0; q < P; ++q) {
        const uint32_t off = k * STEP + (uint32_t)(w * P + q) * 1024u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr)(smem + slot * STEP + (w * P + q) * 1024), 16,
                                                 off + lane * 16, 0, 0, 0);
      }
    };
#pragma unroll
    for (int k = 0; k < D; ++k) issue(k);
    for (uint32_t k = 0; k < nsteps; ++k) {
      if (k + D < nsteps) {
        issue(k + D);
        wait_vm<P * D>();
      } else {
        wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      // touch one word of the slot (keeps the data "used"; no LDS bandwidth to speak of)
      acc ^= *(const int*)(smem + (k % (D + 1)) * STEP + threadIdx.x * 4);
      __builtin_amdgcn_s_barrier();
    }
  } else {
    v4i r[D][P];
#pragma unroll
    for (int k = 0; k < D; ++k)
#pragma unroll
      for (int q = 0; q < P; ++q)
        r[k][q] = __builtin_nontemporal_load((const v4i*)(base + (uint64_t)k * STEP + (w * P + q) * 1024 + lane * 16));
    for (uint32_t k = 0; k < nsteps; k += D) {
#pragma unroll
      for (int j = 0; j < D; ++j)
#pragma unroll
        for (int q = 0; q < P; ++q) {
          acc ^= r[j][q][0] ^ r[j][q][1] ^ r[j][q][2] ^ r[j][q][3];
          if (k + D + j < nsteps)
            r[j][q] = __builtin_nontemporal_load(
                (const v4i*)(base + (uint64_t)(k + D + j) * STEP + (w * P + q) * 1024 + lane * 16));
        }
    }
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

template <int MODE, int P, int D>
void run(const uint8_t* buf, uint64_t bytes, int wg_per_cu, int n_cu, int* out) {
  const int nwg = wg_per_cu * n_cu;
  constexpr uint64_t STEP = 8ull * P * 1024;
  const uint64_t per_wg = bytes / nwg / STEP * STEP;
  const int lds = MODE == 0 ? (int)((D + 1) * STEP) : 0;
  if (lds > 160 * 1024 / wg_per_cu) {
    std::printf("MODE %d P %d D %d wg/CU %d: LDS %d KiB does not fit\n", MODE, P, D, wg_per_cu, lds / 1024);
    return;
  }
  CK(hipFuncSetAttribute((const void*)k_stream<MODE, P, D>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  k_stream<MODE, P, D><<<nwg, 512, lds>>>(buf, per_wg, out);
  CK(hipDeviceSynchronize());
  const int reps = 5;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) k_stream<MODE, P, D><<<nwg, 512, lds>>>(buf, per_wg, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  const double gb = (double)per_wg * nwg / 1e9;
  std::printf("%s P=%d KiB/wave D=%d wg/CU=%d: in flight %3d KiB/CU  %.3f ms  %.0f GB/s\n",
              MODE == 0 ? "lds-dma" : "regs   ", P, D, wg_per_cu, (int)(wg_per_cu * D * STEP / 1024), ms,
              gb / (ms * 1e-3));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main() {
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int n_cu = pr.multiProcessorCount;
  const uint64_t bytes = 8ull << 30;
  uint8_t* buf;
  int* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 1, bytes));
  std::printf("%d CUs, %.1f GiB streamed per launch\n", n_cu, bytes / double(1 << 30));
  for (int wpc = 1; wpc <= 2; ++wpc) {
    run<0, 1, 1>(buf, bytes, wpc, n_cu, out);
    run<0, 1, 2>(buf, bytes, wpc, n_cu, out);
    run<0, 1, 4>(buf, bytes, wpc, n_cu, out);
    run<0, 2, 1>(buf, bytes, wpc, n_cu, out);
    run<0, 2, 2>(buf, bytes, wpc, n_cu, out);
    run<0, 2, 3>(buf, bytes, wpc, n_cu, out);
    run<0, 4, 1>(buf, bytes, wpc, n_cu, out);
    run<0, 4, 2>(buf, bytes, wpc, n_cu, out);
    run<0, 4, 3>(buf, bytes, wpc, n_cu, out);
    run<0, 8, 1>(buf, bytes, wpc, n_cu, out);
    run<1, 1, 2>(buf, bytes, wpc, n_cu, out);
    run<1, 2, 2>(buf, bytes, wpc, n_cu, out);
    run<1, 4, 2>(buf, bytes, wpc, n_cu, out);
  }
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
