// Host interface of the second line-search screen kernel (screen.hip, k_screen_oz2), called by
// DeviceCtx::screen_at (device.hip). Same statistics and bound as k_screen_oz (ozaki.inc).
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace pcamd {

typedef __attribute__((address_space(3))) void* lds_vptr2;

struct Screen2Args {
  const uint8_t* xsl;  // the digit image (ozaki.inc layout)
  const float* xsf;    // per-sample fp32 scales 2^(e_t − E0), lane-permuted (screen2_build_xsf)
  const uint8_t* wsl;  // the W digit image
  const double* wsc;   // W row scales 2^(f_i − 12)
  float c32;           // fl32(−2α·log2 e)
  int e0;              // E0: the image's largest sample exponent
  double ln2_alpha;    // ln 2 / α
  uint32_t bpw;        // 16-sample blocks per workgroup (a multiple of the blocks per step)
  uint32_t n_blocks;   // 16-sample blocks of the shard
  int nwg;             // workgroups (two per CU)
  double* partials;    // [nwg][nw][2·16·NB]: [Σℓ raw | Σ|ỹ|] per row
  int nw = 1;          // tries per pass: 2 = the second W in row blocks NB … 2·NB − 1 of the W image
  bool form32 = false; // k_screen_oz32 (NB = 8, nw = 1): 32x32x32 MFMAs, 2 blocks per step, 1 WG per CU
  int dmax = 3;        // diagonals a + b ≤ dmax of the digit products (2: 6 products on planes 0–2; 3: 10 on 0–3)
};

int screen2_blocks_per_step(int nb);   // 16-sample blocks per loop step (NB = 8: 1, NB = 4: 2)
uint64_t screen2_tile_bytes(int nb);   // bytes of one block's digit image
hipError_t screen2_launch(int nb, const Screen2Args& a, hipStream_t stream);
hipError_t screen2_build_xsf(const double* xsc, uint64_t n, int e0, float* xsf, hipStream_t stream);

}  // namespace pcamd
