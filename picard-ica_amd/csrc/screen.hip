// The orthogonal line-search screen, second form (k_screen_oz2): the same bound as
// k_screen_oz (ozaki.inc) — diagonals D ≤ 3 (or D ≤ 2, DeviceCtx::screen_at) of the exact int8 digit stage, the fp32 combine
// and fp32 ℓ with the error terms DeviceCtx::screen_at adds — on a schedule built from the
// issue costs measured on MI355X (tools/microbench/fill_coexec.hip, profiles/r04_a):
//
//   * an i8 MFMA (v_mfma_i32_16x16x64_i8) holds its SIMD's vector issue for ≈ 12 of its 16
//     cycles, and vector instructions co-issue beside it only from the SAME wave (an MFMA wave
//     beside a VALU wave runs serialised: tools/microbench/agpr_coexec.hip). So each wave
//     interleaves the row terms of its previous step between the MFMAs of its current step
//     (sched_group_barrier: one MFMA, then one vector instruction), instead of 20 MFMAs
//     followed by a block of VALU;
//   * fewer vector instructions per element: the sample scale 2^(e_t − E0) comes in fp32 from
//     a per-image array (k_build_xsf, 4 B per sample, laid out so one ds_read_b128 gives a
//     lane its 4 samples) and the row scale 2^(f_i + E0 − 20) is folded into the exp argument
//     and the final row sums — both powers of two, so every rounding is the old kernel's;
//   * the LDS-DMA staging is raw buffer loads (one 1-KiB piece per wave and step, the step
//     offset in the lane offset: no 64-bit address arithmetic in the loop), and a piece past
//     the workgroup's last block reads zeros (buffer range check): a zero digit block gives
//     y = 0 exactly, whose row terms vanish (|0| = 0, 2^0 = 1, log2 1 = 0), so the loop needs
//     no per-step bounds tests;
//   * 8 waves per workgroup, two workgroups per CU (the two barrier streams interleave).
//
// Not a standalone translation unit for the library's host code: device.hip calls
// screen2_launch / screen2_build_xsf through the declarations in screen2.hpp.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "screen2.hpp"

namespace pcamd {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int SLICES = 7;  // digits per value (ozaki.inc OZ_SLICES)
constexpr int RSRC_DW3 = 0x00020000;  // raw buffer descriptor word 3 (gfx9 family)

__device__ __forceinline__ void* uniform_ptr(const void* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (void*)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ v4i mfma_i8(v4i a, v4i b, v4i c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

// One step's row terms of a lane (4 samples lk + 4r of row lr): the D ≤ 3 diagonal sums
// acc[0..3] → y' = fl(fl(R23)·2^-16 + fl(Q01)) (oz_combine_screen_f32's arithmetic), u = y'·sf
// (sf = 2^(e_t − E0), exact), z = fl(|u|·cz) (cz = |c32|·2^(f_i + E0 − 20): the same fl(|ỹ|·c32)
// as loss_acc4_f32y, negated), then Σ|u| in fp32 ((|u0| + |u1|) + (|u2| + |u3|)) into l and
// log2 Π (1 + 2^−z)/2 into g — every rounding of loss_acc4_f32y's per-element arithmetic, on
// values scaled by exact powers of two.
template <int DM>
__device__ __forceinline__ void row_terms(const v4i (&acc)[4], const f4v& sf, float cz, double& l, double& g) {
  static_assert(DM == 2 || DM == 3, "screen diagonals");
  float u[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q01 = acc[0][r] * 256 + acc[1][r];
    if constexpr (DM == 3) {
      const int r23 = acc[2][r] * 256 + acc[3][r];
      u[r] = __builtin_fmaf((float)r23, 0x1p-16f, (float)q01) * sf[r];
    } else {  // |P_2| < 2^24: exact in fp32, so the fma is the only rounding after fl(Q01)
      u[r] = __builtin_fmaf((float)acc[2][r], 0x1p-8f, (float)q01) * sf[r];
    }
  }
  float f[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = __builtin_fmaf(__builtin_amdgcn_exp2f(-(__builtin_fabsf(u[r]) * cz)), 0.5f, 0.5f);
  const float s = (__builtin_fabsf(u[0]) + __builtin_fabsf(u[1])) + (__builtin_fabsf(u[2]) + __builtin_fabsf(u[3]));
  l += (double)s;
  g += (double)__builtin_amdgcn_logf((f[0] * f[1]) * (f[2] * f[3]));
}

template <int NB, int DM = 3>
struct S2 {
  static constexpr int KSO = NB == 8 ? 2 : 1;          // k-steps of 64 features
  static constexpr int U = 8 / NB;                     // 16-sample blocks per step
  static constexpr int NCP = 16 * NB;                  // rows of the partials
  static constexpr int TILE = SLICES * KSO * 1024;     // bytes of one block's digit image
  static constexpr int PL = DM + 1;                    // digit planes the screen reads (D ≤ DM)
  static constexpr int SLOT = PL * KSO * 1024;         // LDS bytes of one block's planes
  static constexpr int PIECES = PL * KSO;              // 1-KiB pieces per block (U·PIECES ≤ 8)
  static constexpr int NPROD = (DM + 1) * (DM + 2) / 2;  // digit products per k-step (a + b ≤ DM)
  static constexpr int NBUF = 3, SCB = 256;
  template <int NW>
  static constexpr int lds() { return NBUF * U * SLOT + NBUF * SCB + NW * U * NCP * 2 * 8; }
};

// FILL: vector instructions scheduled after each MFMA (0: no schedule groups, the compiler's order).
// NW = 2: two tries at once (the W image's row blocks NB … 2·NB − 1 and row scales 16·NB … hold
// the second W): every X operand read and staged once for both, each W's row terms in the
// arithmetic and order of NW = 1 (so each W's sums are bit-identical to its own screen), partials
// [nwg][NW][2·NCP]. Half the HBM bytes per try: the screen's clock is held down by the memory
// side's power (profiles/r04_e/screen_clock.txt), and two tries per pass relieve it.
template <int NB, int FILL, int NW, int DM>
__global__ void __launch_bounds__(512, NW == 1 ? 2 : 1)
k_screen_oz2(const uint8_t* __restrict__ xsl, const float* __restrict__ xsf, const uint8_t* __restrict__ wsl_g,
             const double* __restrict__ wsc, float c32, int e0, double ln2_alpha, uint32_t bpw, uint32_t n_blocks,
             double* __restrict__ partials) {
  using S = S2<NB, DM>;
  constexpr int KSO = S::KSO, U = S::U, NCP = S::NCP, TILE = S::TILE, SLOT = S::SLOT, NBUF = S::NBUF, PL = S::PL;
  static_assert(U * S::PIECES <= 8, "at most one piece per wave and step");
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int lr = lane & 15, lk = lane >> 4;
  const int yi = wv % NB, h = wv / NB;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tiles = smem;                            // [NBUF][U][SLOT]
  uint8_t* scl = tiles + NBUF * U * SLOT;           // [NBUF][SCB]: U·16 fp32 scales (+ DMA overhang)
  double* red = (double*)(scl + NBUF * S::SCB);     // [U][NCP][2]
  const uint32_t b_begin = blockIdx.x * bpw;
  const uint32_t b_end = b_begin + bpw < n_blocks ? b_begin + bpw : n_blocks;
  const uint32_t nb = b_begin < b_end ? b_end - b_begin : 0u;
  const uint32_t nsteps = (nb + U - 1) / U;
  // buffer resources over this workgroup's blocks only: a piece past its last block reads 0
  // (the operands are wave-uniform; readfirstlane keeps the descriptors in SGPRs, else every
  // buffer load becomes a waterfall loop)
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(xsl + (size_t)b_begin * TILE), 0, __builtin_amdgcn_readfirstlane((int)(nb * TILE)), RSRC_DW3);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(xsf + (size_t)b_begin * 16), 0, __builtin_amdgcn_readfirstlane((int)(nb * 64)), RSRC_DW3);
  // this wave's piece of every step: block bp of the step, piece q (planes 0 … DM are the first
  // PL·KSO KiB of a block image; D ≤ 2: waves 6, 7 stage no piece); wave 7 also moves the
  // step's U·16 scales (lanes repeat)
  const bool piece_wave = wv < U * S::PIECES;
  const int bp = piece_wave ? wv / S::PIECES : 0, q = piece_wave ? wv % S::PIECES : 0;
  const uint32_t voff_x = (uint32_t)(bp * TILE + q * 1024 + lane * 16);
  const uint32_t voff_s = (uint32_t)((lane & (16 * U - 1)) * 4);
  const bool scale_wave = wv == 7;
  auto stage = [&](uint32_t step, int buf) {
    if (piece_wave)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_vptr2)(tiles + (buf * U + bp) * SLOT + q * 1024), 16,
                                               (int)(voff_x + step * (uint32_t)(U * TILE)), 0, 0, 0);
    if (scale_wave)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_vptr2)(scl + buf * S::SCB), 4,
                                               (int)(voff_s + step * (uint32_t)(U * 64)), 0, 0, 0);
  };
  // end of a step: this wave's piece(s) of the NEXT step landed (the ones just issued for the
  // step after may still fly: counted vmcnt), then every wave meets
  // (lgkmcnt(0): this step's scale read has returned before the next step's DMA may overwrite
  // its buffer)
  // (loads this wave issues per step: its piece and / or the scales)
  const int per_step = (piece_wave ? 1 : 0) + (scale_wave ? 1 : 0);
  auto step_barrier = [&]() {
    if (per_step == 2) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
    else if (per_step == 1) asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  v4i wsl[NW][4][KSO];
  double rowscale[NW];
  float cz[NW];
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int rb = yi + NB * w;  // this try's row block in the W image
#pragma unroll
    for (int a = 0; a <= DM; ++a)
#pragma unroll
      for (int s = 0; s < KSO; ++s)
        wsl[w][a][s] = *(const v4i*)(wsl_g + (size_t)(((rb * SLICES + a) * 2 + s) * 64 + lane) * 16);
    rowscale[w] = __builtin_ldexp(wsc[rb * 16 + lr], e0 - 8);  // 2^(f_i + E0 − 20)
    cz[w] = __builtin_fabsf(c32) * (float)rowscale[w];          // exact: a power-of-2 scaling
  }
  double l[NW], g[NW];
  v4i acc[2][NW][4];
  f4v sf[2];
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    l[w] = g[w] = 0.0;
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[1][w][d] = v4i{0, 0, 0, 0};  // the "previous step" of step 0: zero terms
  }
  sf[1] = f4v{0.f, 0.f, 0.f, 0.f};
  stage(0, 0);
  stage(1, 1);
  if (per_step == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (per_step == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // step k: stage k + 2; the MFMAs of step k with the row terms of step k − 1 between them
  auto body = [&](uint32_t k, int buf, auto cur_c) {
    constexpr int cur = decltype(cur_c)::value, prv = cur ^ 1;
    stage(k + 2, buf == 0 ? 2 : buf - 1);  // (k + 2) mod 3; past the end: zeros, never read
    const uint8_t* tile = tiles + (buf * U + h) * SLOT + lane * 16;
    v4i xa[2][KSO];
#pragma unroll
    for (int s = 0; s < KSO; ++s) xa[0][s] = *(const v4i*)(tile + s * 1024);
#pragma unroll
    for (int b = 0; b < PL; ++b) {
      if (b < PL - 1)
#pragma unroll
        for (int s = 0; s < KSO; ++s) xa[(b + 1) & 1][s] = *(const v4i*)(tile + ((b + 1) * KSO + s) * 1024);
#pragma unroll
      for (int s = 0; s < KSO; ++s)
#pragma unroll
        for (int a = 0; a <= DM - b; ++a)
#pragma unroll
          for (int w = 0; w < NW; ++w) {
            const int d = a + b;
            acc[cur][w][d] = (b == 0 && s == 0) ? mfma_i8(xa[b & 1][s], wsl[w][a][s], v4i{0, 0, 0, 0})
                                                : mfma_i8(xa[b & 1][s], wsl[w][a][s], acc[cur][w][d]);
          }
    }
#pragma unroll
    for (int w = 0; w < NW; ++w) row_terms<DM>(acc[prv][w], sf[prv], cz[w], l[w], g[w]);
    sf[cur] = *(const f4v*)(scl + buf * S::SCB + h * 64 + lk * 16);
    // one MFMA, then FILL vector instructions, over the NPROD·KSO·NW MFMAs of the step
    if constexpr (FILL > 0) {
#pragma unroll
      for (int i = 0; i < S::NPROD * KSO * NW; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, FILL, 0);
      }
    }
    // the row sums are complete here: keeps the row terms in this block (between the MFMAs)
    // instead of sunk past the barrier's wait
#pragma unroll
    for (int w = 0; w < NW; ++w) asm volatile("" ::"v"(l[w]), "v"(g[w]));
    step_barrier();
  };
  uint32_t k = 0;
  int buf = 0;
  for (; k + 1 < nsteps; k += 2) {
    body(k, buf, std::integral_constant<int, 0>{});
    buf = buf == 2 ? 0 : buf + 1;
    body(k + 1, buf, std::integral_constant<int, 1>{});
    buf = buf == 2 ? 0 : buf + 1;
  }
  if (k < nsteps) {
    body(k, buf, std::integral_constant<int, 0>{});
#pragma unroll
    for (int w = 0; w < NW; ++w) row_terms<DM>(acc[0][w], sf[0], cz[w], l[w], g[w]);
  } else {
#pragma unroll
    for (int w = 0; w < NW; ++w) row_terms<DM>(acc[1][w], sf[1], cz[w], l[w], g[w]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero pieces past the end: drained
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    double rs_y = l[w] * rowscale[w];  // Σ|ỹ| (exact scaling)
    double rs_ll = __builtin_fma(g[w], ln2_alpha, rs_y);
    rs_ll += __shfl_xor(rs_ll, 16); rs_ll += __shfl_xor(rs_ll, 32);
    rs_y += __shfl_xor(rs_y, 16);   rs_y += __shfl_xor(rs_y, 32);
    if (lk == 0) {
      red[((w * U + h) * NCP + yi * 16 + lr) * 2 + 0] = rs_ll;
      red[((w * U + h) * NCP + yi * 16 + lr) * 2 + 1] = rs_y;
    }
  }
  __syncthreads();
  double* out = partials + (size_t)blockIdx.x * NW * 2 * NCP;  // [NW][Σℓ raw | Σ|ỹ|]
  for (int e = threadIdx.x; e < NW * 2 * NCP; e += 512) {
    const int w = e / (2 * NCP), c = (e / NCP) % 2, row = e % NCP;
    double v = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) v += red[((w * U + u) * NCP + row) * 2 + c];
    out[e] = v;
  }
}

// The same screen on v_mfma_i32_32x32x32_i8 (NB = 8, one try; PICARD_SCREEN32=1): an i8 MFMA of
// this shape holds its SIMD's vector issue for ≈ 8 of its 32 cycles, so the row terms of step
// k − 1 (≈ 190 VALU per wave and step) fit in the gaps of step k's 40 MFMAs (1280 cycles), where
// the 16x16x64 form leaves ≈ 40 % of its row terms exposed (profiles/r05_m: the screen returns
// about half of a VALU cut as time). One wave per SIMD (4 waves, 256 threads): wave w owns W rows
// 32w … 32w + 31 of a 32-sample step (two 16-sample image blocks); the diagonal accumulators
// (4 × 16 int32, double-buffered) take the AGPRs. A operands come from the unchanged digit image:
// lane l reads the 16-byte item of sample row r = l & 31 (block r >> 4, A-row r & 15) and features
// 32k + 16(l >> 5) … +15; B operands (W's D ≤ 3 digits) likewise from the W image, once. Output:
// lane l holds W row 32w + (l & 31) and the 16 sample rows (i & 3) + 8(i >> 2) + 4(l >> 5); the
// fp32 scale of sample row r of the step is xsf[32·step + r] (k_build_xsf's order is the A-row
// order). Row terms: row_terms' per-element arithmetic on 4 groups of 4 samples per lane — the
// grouping the bound's per-4-sample constants assume — so DeviceCtx::screen_at's bound holds as
// for k_screen_oz2 (the estimate's grouping differs: not bit-identical to it).
constexpr int S32_U = 2, S32_SLOT = 4 * 2 * 1024, S32_NBUF = 3, S32_SCB = 256;
constexpr int S32_TILE = SLICES * 2 * 1024;
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ __forceinline__ v16i mfma_i8_32(v4i a, v4i b, v16i c) {
  return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void row_terms32(const v16i (&acc)[4], const float (&sf)[16], float cz, double& l,
                                            double& g) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float u[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * q + e;
      const int q01 = acc[0][i] * 256 + acc[1][i], r23 = acc[2][i] * 256 + acc[3][i];
      u[e] = __builtin_fmaf((float)r23, 0x1p-16f, (float)q01) * sf[i];
    }
    float f[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = __builtin_fmaf(__builtin_amdgcn_exp2f(-(__builtin_fabsf(u[e]) * cz)), 0.5f, 0.5f);
    const float sm = (__builtin_fabsf(u[0]) + __builtin_fabsf(u[1])) + (__builtin_fabsf(u[2]) + __builtin_fabsf(u[3]));
    l += (double)sm;
    g += (double)__builtin_amdgcn_logf((f[0] * f[1]) * (f[2] * f[3]));
  }
}

template <int FILL>
__global__ void __launch_bounds__(256, 1)
k_screen_oz32(const uint8_t* __restrict__ xsl, const float* __restrict__ xsf, const uint8_t* __restrict__ wsl_g,
              const double* __restrict__ wsc, float c32, int e0, double ln2_alpha, uint32_t bpw, uint32_t n_blocks,
              double* __restrict__ partials) {
  constexpr int NCP = 128;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int h = lane >> 5, n = lane & 15, rb16 = 2 * wv + ((lane & 31) >> 4);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tiles = smem;                                 // [NBUF][U][SLOT]: planes 0–3 of 2 blocks
  uint8_t* scl = tiles + S32_NBUF * S32_U * S32_SLOT;    // [NBUF][SCB]: 32 fp32 scales
  const uint32_t b_begin = blockIdx.x * bpw;
  const uint32_t b_end = b_begin + bpw < n_blocks ? b_begin + bpw : n_blocks;
  const uint32_t nb = b_begin < b_end ? b_end - b_begin : 0u;
  const uint32_t nsteps = (nb + S32_U - 1) / S32_U;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(xsl + (size_t)b_begin * S32_TILE), 0, __builtin_amdgcn_readfirstlane((int)(nb * S32_TILE)), RSRC_DW3);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(xsf + (size_t)b_begin * 16), 0, __builtin_amdgcn_readfirstlane((int)(nb * 64)), RSRC_DW3);
  // wave w stages pieces 4w … 4w + 3 of every step: block p >> 3, 1-KiB piece p & 7 (planes 0–3 ×
  // 2 k-steps are the first 8 KiB of a block image); wave 3 also the step's 32 scales
  const bool scale_wave = wv == 3;
  auto stage = [&](uint32_t step, int buf) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = 4 * wv + u, bp = p >> 3, q = p & 7;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_vptr2)(tiles + (buf * S32_U + bp) * S32_SLOT + q * 1024), 16,
                                               (int)((uint32_t)(bp * S32_TILE + q * 1024 + lane * 16) +
                                                     step * (uint32_t)(S32_U * S32_TILE)),
                                               0, 0, 0);
    }
    if (scale_wave)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_vptr2)(scl + buf * S32_SCB), 4,
                                               (int)((uint32_t)((lane & 31) * 4) + step * (uint32_t)(S32_U * 64)), 0,
                                               0, 0);
  };
  auto step_barrier = [&]() {
    if (scale_wave) asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  // W's D ≤ 3 digits as B operands: lane l = W row 32w + (l & 31), features 32k + 16h … +15
  v4i wb[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int s2 = k >> 1, g = 2 * (k & 1) + h;
      wb[a][k] = *(const v4i*)(wsl_g + (size_t)(((rb16 * SLICES + a) * 2 + s2) * 64 + n + 16 * g) * 16);
    }
  const double rowscale = __builtin_ldexp(wsc[rb16 * 16 + n], e0 - 8);  // 2^(f_i + E0 − 20)
  const float cz = __builtin_fabsf(c32) * (float)rowscale;
  double l = 0.0, g = 0.0;
  v16i acc[2][4];
  float sf[2][16];
#pragma unroll
  for (int d = 0; d < 4; ++d) acc[1][d] = v16i{};
#pragma unroll
  for (int i = 0; i < 16; ++i) sf[1][i] = 0.f;
  stage(0, 0);
  stage(1, 1);
  if (scale_wave) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // A item of lane l for (plane b, k-step k): sample row l & 31 → block (l & 31) >> 4, A-row l & 15
  const int a_off = ((lane & 31) >> 4) * S32_SLOT + n * 16;
  auto body = [&](uint32_t k, int buf, auto cur_c) {
    constexpr int cur = decltype(cur_c)::value, prv = cur ^ 1;
    stage(k + 2, buf == 0 ? 2 : buf - 1);  // (k + 2) mod 3; past the end: zeros, never read
    const uint8_t* tb = tiles + buf * S32_U * S32_SLOT + a_off;
    v4i xa[2][4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) xa[0][kk] = *(const v4i*)(tb + (kk >> 1) * 1024 + (2 * (kk & 1) + h) * 256);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (b < 3)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          xa[(b + 1) & 1][kk] = *(const v4i*)(tb + ((b + 1) * 2 + (kk >> 1)) * 1024 + (2 * (kk & 1) + h) * 256);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int a = 0; a <= 3 - b; ++a) {
          const int d = a + b;
          acc[cur][d] = (b == 0 && kk == 0) ? mfma_i8_32(xa[b & 1][kk], wb[a][kk], v16i{})
                                            : mfma_i8_32(xa[b & 1][kk], wb[a][kk], acc[cur][d]);
        }
    }
    row_terms32(acc[prv], sf[prv], cz, l, g);
    {  // this step's 16 scales: sample rows 8q + 4h + 0…3 (q = 0…3)
      const float* sp = (const float*)(scl + buf * S32_SCB);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *(const float4*)(sp + 8 * q + 4 * h);
        sf[cur][4 * q + 0] = v.x; sf[cur][4 * q + 1] = v.y; sf[cur][4 * q + 2] = v.z; sf[cur][4 * q + 3] = v.w;
      }
    }
    if constexpr (FILL > 0) {
#pragma unroll
      for (int i = 0; i < 40; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, FILL, 0);
      }
    }
    asm volatile("" ::"v"(l), "v"(g));
    step_barrier();
  };
  uint32_t k = 0;
  int buf = 0;
  for (; k + 1 < nsteps; k += 2) {
    body(k, buf, std::integral_constant<int, 0>{});
    buf = buf == 2 ? 0 : buf + 1;
    body(k + 1, buf, std::integral_constant<int, 1>{});
    buf = buf == 2 ? 0 : buf + 1;
  }
  if (k < nsteps) {
    body(k, buf, std::integral_constant<int, 0>{});
    row_terms32(acc[0], sf[0], cz, l, g);
  } else {
    row_terms32(acc[1], sf[1], cz, l, g);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero pieces past the end: drained
  double rs_y = l * rowscale;  // Σ|ỹ| (exact scaling)
  double rs_ll = __builtin_fma(g, ln2_alpha, rs_y);
  rs_ll += __shfl_xor(rs_ll, 32);
  rs_y += __shfl_xor(rs_y, 32);
  if (h == 0) {
    double* out = partials + (size_t)blockIdx.x * 2 * NCP;  // [Σℓ raw | Σ|ỹ|]
    out[32 * wv + (lane & 31)] = rs_ll;
    out[NCP + 32 * wv + (lane & 31)] = rs_y;
  }
}

// xsf[16·blk + 4·lk + r] = 2^(e_t − E0) in fp32 for sample t = 16·blk + lk + 4r (the lane's 4
// samples of k_screen_oz2 contiguous): exact for the image's exponent range (host-checked)
__global__ void __launch_bounds__(256) k_build_xsf(const double* __restrict__ xsc, uint64_t n, int e0,
                                                   float* __restrict__ xsf) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t blk = i >> 4;
    const int lk = (int)(i >> 2) & 3, r = (int)i & 3;
    xsf[i] = (float)__builtin_ldexp(xsc[blk * 16 + lk + 4 * r], -e0);
  }
}

template <int NB, int FILL, int NW, int DM>
hipError_t launch_fill(const Screen2Args& a, hipStream_t stream) {
  using S = S2<NB, DM>;
  constexpr int LDS = S::template lds<NW>();
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_screen_oz2<NB, FILL, NW, DM>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  k_screen_oz2<NB, FILL, NW, DM><<<a.nwg, 512, LDS, stream>>>(a.xsl, a.xsf, a.wsl, a.wsc, a.c32, a.e0, a.ln2_alpha,
                                                           a.bpw, a.n_blocks, a.partials);
  return hipGetLastError();
}
// PICARD_SCREEN2_FILL (measurement knob): vector instructions per MFMA gap, 0 = compiler order.
// Default 1: (128, 2e7) 3.20–3.26 ms against 3.29–3.31 for 2 and 3.30–3.32 for 0, alternating
// on one box (profiles/r04_e/screen_fill_ab.txt)
int fill_knob() {
  static const int v = [] {
    const char* e = std::getenv("PICARD_SCREEN2_FILL");
    return e ? std::atoi(e) : 1;
  }();
  return v;
}
template <int NB, int NW, int DM>
hipError_t launch_dm(const Screen2Args& a, hipStream_t stream) {
  switch (fill_knob()) {
    case 0: return launch_fill<NB, 0, NW, DM>(a, stream);
    case 2: return launch_fill<NB, 2, NW, DM>(a, stream);
    default: return launch_fill<NB, 1, NW, DM>(a, stream);
  }
}
template <int NB, int NW>
hipError_t launch(const Screen2Args& a, hipStream_t stream) {
  if (a.dmax == 2) return launch_dm<NB, NW, 2>(a, stream);
  if (a.dmax == 3) return launch_dm<NB, NW, 3>(a, stream);
  return hipErrorInvalidValue;
}

}  // namespace

int screen2_blocks_per_step(int nb) { return 8 / nb; }
uint64_t screen2_tile_bytes(int nb) { return nb == 8 ? S2<8>::TILE : S2<4>::TILE; }  // (all planes: DM-free)

template <int FILL>
hipError_t screen32_launch_fill(const Screen2Args& a, hipStream_t stream) {
  constexpr int LDS = S32_NBUF * S32_U * S32_SLOT + S32_NBUF * S32_SCB;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_screen_oz32<FILL>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  k_screen_oz32<FILL><<<a.nwg, 256, LDS, stream>>>(a.xsl, a.xsf, a.wsl, a.wsc, a.c32, a.e0, a.ln2_alpha, a.bpw,
                                                    a.n_blocks, a.partials);
  return hipGetLastError();
}
// PICARD_SCREEN32_FILL (measurement knob): vector instructions per MFMA gap, 0 = compiler order
hipError_t screen32_launch(const Screen2Args& a, hipStream_t stream) {
  static const int fill = [] {
    const char* e = std::getenv("PICARD_SCREEN32_FILL");
    return e ? std::atoi(e) : 5;
  }();
  switch (fill) {
    case 0: return screen32_launch_fill<0>(a, stream);
    case 3: return screen32_launch_fill<3>(a, stream);
    case 8: return screen32_launch_fill<8>(a, stream);
    default: return screen32_launch_fill<5>(a, stream);
  }
}

hipError_t screen2_launch(int nb, const Screen2Args& a, hipStream_t stream) {
  if (a.form32) return nb == 8 && a.nw == 1 && a.dmax == 3 ? screen32_launch(a, stream) : hipErrorInvalidValue;
  if (a.nw == 2) return nb == 8 ? launch<8, 2>(a, stream) : launch<4, 2>(a, stream);
  return nb == 8 ? launch<8, 1>(a, stream) : launch<4, 1>(a, stream);
}

hipError_t screen2_build_xsf(const double* xsc, uint64_t n, int e0, float* xsf, hipStream_t stream) {
  const unsigned grid = (unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  k_build_xsf<<<grid ? grid : 1, 256, 0, stream>>>(xsc, n, e0, xsf);
  return hipGetLastError();
}

}  // namespace pcamd
