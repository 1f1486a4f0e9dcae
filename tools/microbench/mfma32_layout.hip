// Operand / result layout of v_mfma_i32_32x32x32_i8 (gfx950), measured: for an A operand with a
// single 1 at (lane la, byte ba) and a B operand of all ones, which (lane, register) outputs are
// 1 (→ the row that A position feeds); the same for B (→ its column); and which B position
// (lane lb, byte bb) pairs with a given A position on k (A one-hot × B one-hot ≠ 0).
// build: hipcc -O3 --offload-arch=gfx950 tools/microbench/mfma32_layout.hip -o tools/microbench/mfma32_layout
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// mode 0: A one-hot at (p / 16, p % 16), B all ones; mode 1: B one-hot, A all ones;
// mode 2: A one-hot at p0, B one-hot at p (p0 fixed)
__global__ void k(int mode, int p0, int* out) {
  const int p = blockIdx.x;  // one-hot position of this block: lane p / 16, byte p % 16
  const int l = threadIdx.x;
  auto onehot = [&](int q) {
    v4i v = {0, 0, 0, 0};
    if (l == q / 16) v[(q % 16) / 4] = 1 << (8 * (q % 4));
    return v;
  };
  const v4i ones = {0x01010101, 0x01010101, 0x01010101, 0x01010101};
  v4i a, b;
  if (mode == 0) { a = onehot(p); b = ones; }
  else if (mode == 1) { a = ones; b = onehot(p); }
  else { a = onehot(p0); b = onehot(p); }
  v16i c;
  for (int r = 0; r < 16; ++r) c[r] = 0;
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) out[(p * 64 + l) * 16 + r] = c[r];
}

int main() {
  int* d;
  const size_t n = 1024 * 64 * 16;
  hipMalloc(&d, n * sizeof(int));
  int* h = (int*)malloc(n * sizeof(int));
  // mode 0 / 1: per one-hot position, the set of (lane, reg) outputs that are nonzero
  for (int mode = 0; mode < 2; ++mode) {
    k<<<1024, 64>>>(mode, 0, d);
    hipMemcpy(h, d, n * sizeof(int), hipMemcpyDeviceToHost);
    printf("mode %d (%s one-hot): position (lane, byte) -> nonzero outputs (lane:reg)\n", mode, mode ? "B" : "A");
    for (int p = 0; p < 1024; p += (p < 64 ? 1 : 97)) {
      printf("  (%2d,%2d):", p / 16, p % 16);
      int cnt = 0;
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r)
          if (h[(p * 64 + l) * 16 + r]) {
            if (cnt < 6) printf(" %d:%d", l, r);
            ++cnt;
          }
      printf("  [%d nonzero]\n", cnt);
    }
  }
  // mode 2: for a few A positions, the B positions that pair with them on k
  const int probes[] = {0, 1, 5, 8, 9, 15, 16, 17, 31 * 16 + 3, 32 * 16, 32 * 16 + 8, 33 * 16 + 15, 63 * 16 + 7};
  for (int p0 : probes) {
    k<<<1024, 64>>>(2, p0, d);
    hipMemcpy(h, d, n * sizeof(int), hipMemcpyDeviceToHost);
    printf("A (%2d,%2d) pairs with B:", p0 / 16, p0 % 16);
    for (int p = 0; p < 1024; ++p) {
      bool nz = false;
      for (int i = 0; i < 64 * 16; ++i) nz |= h[p * 64 * 16 + i] != 0;
      if (nz) printf(" (%d,%d)", p / 16, p % 16);
    }
    printf("\n");
  }
  hipFree(d);
  free(h);
  return 0;
}
