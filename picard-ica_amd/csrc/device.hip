// MI355X (gfx950) device side of the Picard solver.
//
// The hot path is k_eval_fused: ONE pass over the resident X shard computes,
// for a candidate unmixing map W (nc × nf) and mean μ,
//     Y = W·(X − μ)                      (core.rs:124 / solver.rs:140, fp64 MFMA)
//     ψ, ψ′, ℓ = density(Y)              (density.rs:50-130, fp64 VALU, registers only)
//     G_raw += ψ·Yᵀ                      (core.rs:218, fp64 MFMA)
//     H_raw += ψ′·(Y∘Y)ᵀ   (non-ortho)   (core.rs:274, fp64 MFMA)
//     Σψ′, Σℓ, Σy² per row               (core.rs:226,264, :76,:79)
// Y never touches HBM: each 16×16 Yᵀ tile produced by v_mfma_f64_16x16x4_f64
// already sits in registers in the A/B operand layout of the next MFMA
// (lane l, reg r ↔ row l&15, sample 4r + (l>>4)), so ψ and Y are handed to
// the G-stage waves through LDS without any transpose. Per-workgroup partial
// sums are reduced by k_reduce in a fixed order (bit-reproducible; no atomics).
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <sched.h>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "collective.hpp"
#include "screen2.hpp"
#include "evaluator.hpp"
#include "host_linalg.hpp"
#include "expm_plan.hpp"

namespace pcamd {
size_t jade_max_pairs();  // host_solver.cpp (PICARD_JADE_MAX_PAIRS test hook)

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
// LDS-DMA (global_load_lds) operand address spaces
typedef __attribute__((address_space(3))) void* lds_vptr;
typedef __attribute__((address_space(1))) void* gbl_vptr;

// DENS_TANH_S / DENS_EXP_S: tanh / exp at any α (α ≤ 0 or NaN included — the
// reference does not restrict it, density.rs:33-103), by the reference's own
// formulas through libm instead of the α > 0 table paths; tiled path only.
enum { DENS_TANH = 0, DENS_EXP = 1, DENS_CUBE = 2, DENS_LINEAR = 3, DENS_NONE = 4, DENS_TANH_S = 5, DENS_EXP_S = 6 };

#define HIP_OK(expr)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      throw computation_error(std::string("HIP: ") + hipGetErrorString(e_) + " at " #expr); \
  } while (0)

// ---------------------------------------------------------------------------
// fp64 elementary functions for the fused pass. fp64 VALU issue and fp64 MFMA
// share one pipe on gfx950 (tools/microbench/fp64_rates.hip: 78 TF MFMA alone,
// 66 TF VALU alone, ~75 TF combined), so every VALU op here is paid for in
// MFMA time. Branch-free, argument ranges known, Chebyshev (near-minimax)
// coefficients generated with mpmath (tools/gen_coeffs.py): ≤ 2 ulp.
// ---------------------------------------------------------------------------
namespace fm {
constexpr double LOG2E = 0x1.71547652b82fep+0;
constexpr double LN2_HI = 0x1.62e42fee00000p-1;  // 32 trailing zero bits: k·LN2_HI exact
constexpr double LN2_LO = 0x1.a39ef35793c76p-33;
constexpr double LN2 = 0x1.62e42fefa39efp-1;
constexpr double SQRT2 = 0x1.6a09e667f3bcdp+0;

// x ∈ [-708, 0.35]: e^x = scale·(1 + em_r), scale = 2^k, em_r = e^r − 1, |r| ≤ ln2/2
__device__ __forceinline__ void exp_parts(double x, double& em_r, double& scale) {
  const double kf = __builtin_rint(x * LOG2E);
  double r = __builtin_fma(-kf, LN2_HI, x);
  r = __builtin_fma(-kf, LN2_LO, r);
  double p = 0x1.af389ecfc4b9cp-26;
  p = __builtin_fma(p, r, 0x1.28917c89a43a7p-22);
  p = __builtin_fma(p, r, 0x1.71de0db2f6b19p-19);
  p = __builtin_fma(p, r, 0x1.a019b9149a41cp-16);
  p = __builtin_fma(p, r, 0x1.a01a01a7c2efep-13);
  p = __builtin_fma(p, r, 0x1.6c16c17889ef1p-10);
  p = __builtin_fma(p, r, 0x1.11111111109b5p-7);
  p = __builtin_fma(p, r, 0x1.5555555553d68p-5);
  p = __builtin_fma(p, r, 0x1.5555555555556p-3);
  p = __builtin_fma(p, r, 0x1.0000000000001p-1);
  em_r = __builtin_fma(r * r, p, r);
  scale = __builtin_ldexp(1.0, (int)kf);
}

// v_rcp_f64 is good to ~2^-25 (tools/microbench/rcp_acc.hip: 2.4e8 ulp raw,
// 9.9 ulp after one Newton step, 0.5 ulp after two)
__device__ __forceinline__ double rcp_nr1(double d) {
  const double r = __builtin_amdgcn_rcp(d);
  return __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
}

// n / d: one Newton step on the reciprocal, then one residual correction of
// the quotient (error ≈ ε_r² + rounding: ≤ 1 ulp) — 6 fp64 ops
__device__ __forceinline__ double div_nr(double n, double d) {
  const double r = rcp_nr1(d);
  const double q = n * r;
  return __builtin_fma(__builtin_fma(-d, q, n), r, q);
}

// ln z for z ∈ [1, 2]: 2·atanh(s), s = (z'−1)/(z'+1), z' = z or z/2 (+ ln 2)
__device__ __forceinline__ double log_1_2(double z) {
  const bool big = z > SQRT2;
  const double zz = big ? 0.5 * z : z;
  const double s = div_nr(zz - 1.0, zz + 1.0);
  const double u = s * s;
  double q = 0x1.2f4d88c4fad06p-4;
  q = __builtin_fma(q, u, 0x1.3999bf614de60p-4);
  q = __builtin_fma(q, u, 0x1.7466994f20a7cp-4);
  q = __builtin_fma(q, u, 0x1.c71c50004ffddp-4);
  q = __builtin_fma(q, u, 0x1.2492494513f76p-3);
  q = __builtin_fma(q, u, 0x1.999999997aeaap-3);
  q = __builtin_fma(q, u, 0x1.55555555555aep-2);
  q = __builtin_fma(q, u, 0x1.0000000000000p+0);
  return __builtin_fma(s + s, q, big ? LN2 : 0.0);
}
}  // namespace fm

// ---------------------------------------------------------------------------
// density.rs:50-130 per element. psi = ψ(y), dpsi = ψ′(y), ll = ℓ(y).
// Tanh: one expm1 feeds both tanh(αy) = −em/(2+em)·sign and
// ℓ = |y| + ln(1 + e^{−2α|y|})/α = |y| + ln(2 + em)/α  (α > 0).
// inv_alpha = 1/α is precomputed (the reference divides; ≤ 1 ulp apart).
// ---------------------------------------------------------------------------
// Shared by every kernel so ℓ, ψ′ and y² are bit-identical across the fused,
// loss-only and completion passes (device code is built with -ffp-contract=on).
__device__ __forceinline__ double tanh_em(double y, double alpha) {  // e^{-2|αy|} − 1
  double em_r, sc;
  fm::exp_parts(fmax(-2.0 * fabs(alpha * y), -708.0), em_r, sc);
  return __builtin_fma(sc, em_r, sc - 1.0);
}
__device__ __forceinline__ double tanh_ll(double y, double em, double inv_alpha) {
  return __builtin_fma(fm::log_1_2(2.0 + em), inv_alpha, fabs(y));
}
__device__ __forceinline__ double exp_k(double y, double alpha) {  // e^{-α y²/2}
  double em_r, sc;
  fm::exp_parts(fmax(-alpha / 2.0 * (y * y), -708.0), em_r, sc);
  return __builtin_fma(sc, em_r, sc);
}

template <int DENS, bool FAST>
__device__ __forceinline__ void density_eval(double y, double alpha, double inv_alpha, double& psi, double& dpsi,
                                             double& ll) {
  if constexpr (DENS == DENS_TANH) {
    const double ay = fabs(y);
    const double a = alpha * y;
    if constexpr (FAST) {  // α > 0 (checked on the host)
      const double em = tanh_em(y, alpha);  // e^{-2|a|} − 1 ∈ (−1, 0]; 2 + em = 1 + e^{-2α|y|} ∈ (1, 2]
      const double th = copysign(fm::div_nr(-em, 2.0 + em), a);
      psi = th;
      dpsi = alpha * __builtin_fma(-th, th, 1.0);
      ll = tanh_ll(y, em, inv_alpha);
    } else {
      const double th = tanh(a);
      psi = th;
      dpsi = alpha * (1.0 - th * th);
      ll = ay + log(1.0 + exp(-2.0 * alpha * ay)) / alpha;
    }
  } else if constexpr (DENS == DENS_EXP) {
    const double y2 = y * y;
    const double x = -alpha / 2.0 * y2;
    double k;
    if constexpr (FAST) {  // α > 0: x ≤ 0
      (void)x;
      k = exp_k(y, alpha);
      ll = -k * inv_alpha;
    } else {
      k = exp(x);
      ll = -exp(-alpha * y * y / 2.0) / alpha;
    }
    psi = y * k;
    dpsi = (1.0 - alpha * y2) * k;
  } else if constexpr (DENS == DENS_CUBE) {
    const double y2 = y * y;
    psi = y2 * y;
    dpsi = 3.0 * y2;
    ll = y2 * y2 / 4.0;
  } else {  // LINEAR: ψ = y turns G_raw into the Gram Σ y yᵀ
    psi = y;
    dpsi = 1.0;
    ll = 0.0;
  }
}

// ℓ(y) alone (line-search tries only need Σℓ; core.rs:73-82)
template <int DENS>
__device__ __forceinline__ double density_loss(double y, double alpha, double inv_alpha) {
  if constexpr (DENS == DENS_TANH) {
    return tanh_ll(y, tanh_em(y, alpha), inv_alpha);
  } else if constexpr (DENS == DENS_EXP) {
    return -exp_k(y, alpha) * inv_alpha;
  } else if constexpr (DENS == DENS_CUBE) {
    const double y2 = y * y;
    return y2 * y2 / 4.0;
  } else {
    return 0.0;
  }
}

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// Per-lane row accumulators of the register-resident kernels (fused, loss-only,
// completion). Every term is arranged to vanish EXACTLY at y = 0, the value a
// padded sample (zero X̃ column) produces, so no per-element validity masks are
// needed; the per-sample constants are restored once per row in finalize_row:
//   tanh  Σψ′ = α·(n − Σ th²)               (ψ′ = α(1 − th²))
//         Σℓ  = Σ|y| + (n·ln2 + ln Π(1 + em/2))/α   (ℓ = |y| + ln(2 + em)/α)
//         the product replaces one fp64 log per element by one multiply; it is
//         accumulated as Π(2 + em) (the divisor of tanh's rcp, so no extra op),
//         kept as mantissa × 2^e (renormalised every 32 blocks: factors ∈ (1, 2])
//         and its log is taken once per lane, minus (#factors)·ln2 — the same
//         bits as Π(1 + em/2), since halving is exact
//   exp   Σψ′ = n + Σ(em − α y² k),  Σℓ = −(n + Σ em)/α   (k = e^{−αy²/2} = 1 + em)
//   cube  Σψ′ = 3·Σy²,  Σℓ = Σ y⁴/4
// All kernels of this family share these formulas and the sample → lane map,
// so their sums stay bit-identical to each other.
// ---------------------------------------------------------------------------
struct RowAcc {
  double d = 0.0, l = 0.0, q = 0.0;  // raw Σψ′ term, raw Σℓ term, Σy²
  double p = 1.0;                    // tanh: Π (2 + em), mantissa
  int e = 0;                         //       … and its binary exponent
  double g = 0.0;                    // tanh screen (fp32 ℓ): Σ log2 Π((1 + e^{−2α|y|})/2)
};

// e^x table for exp_n: T_j = 2^(j/32) (correctly rounded), with the high word
// pre-biased by −(j << 15) so that adding (m << 15) for m = 32k + j yields
// the high word of 2^k·T_j in ONE integer op (mod 2^32). Every kernel that
// calls exp_n copies it into its own LDS (exp_tab_load, before the first
// barrier): 32 doubles = the 64 LDS banks once, so any lane pattern is
// conflict-free.
__constant__ uint64_t c_exp_tab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
#define EXP_TAB_DECL __shared__ double s_exp_tab[32]
constexpr int EXP_TAB_BYTES = 32 * sizeof(double);  // static LDS: the dynamic limit is 160 KiB minus this
__device__ __forceinline__ void exp_tab_load(double* tab) {
  if (threadIdx.x < 32) tab[threadIdx.x] = __longlong_as_double((long long)c_exp_tab[threadIdx.x]);
}

// e^x for NW independent x ∈ [−708, 0] as s·(1 + emr), s = 2^(m/32) from the
// LDS table, |r| ≤ ln2/64, written step-interleaved so the NW dependent FMA
// chains overlap (left to itself the compiler emits them one after another).
// Rounding to m uses the 1.5·2^52 shifter (its low word IS m); the reduction
// r = x − m·ln2/32 is one fma (error ≤ |m|·2^-59·e^x ≤ 3e-17 absolute for
// x ≤ 0, 0 for m = 0); e^r − 1 = r + r²·p(r), p of degree 4 (near-minimax on
// |r| ≤ ln2/64, mpmath chebyfit: ≤ 2.2e-19 absolute). 15 VALU + 1 LDS read per
// element against 19 for a table-free degree-11 form.
template <int NW>
__device__ __forceinline__ void exp_n(const double* x, const double* tab, double* emr, double* sc) {
  constexpr double SHIFT = 0x1.8p52;
  constexpr double LOG2E_32 = 0x1.71547652b82fep+5, LN2_32 = 0x1.62e42fefa39efp-6;
  double t[NW], r[NW], p[NW], tj[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) t[i] = __builtin_fma(x[i], LOG2E_32, SHIFT);
#pragma unroll
  for (int i = 0; i < NW; ++i) tj[i] = tab[__double2loint(t[i]) & 31];
#pragma unroll
  for (int i = 0; i < NW; ++i) r[i] = __builtin_fma(-(t[i] - SHIFT), LN2_32, x[i]);
  constexpr double C[5] = {0x1.6c16ffe57d9c9p-10, 0x1.11114f8a7941cp-7, 0x1.555555555194dp-5,
                           0x1.555555554dd45p-3, 0x1.0000000000000p-1};
#pragma unroll
  for (int i = 0; i < NW; ++i) p[i] = __builtin_fma(C[0], r[i], C[1]);
#pragma unroll
  for (int c = 2; c < 5; ++c)
#pragma unroll
    for (int i = 0; i < NW; ++i) p[i] = __builtin_fma(p[i], r[i], C[c]);
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    emr[i] = __builtin_fma(r[i] * r[i], p[i], r[i]);
    const int m = __double2loint(t[i]);
    sc[i] = __hiloint2double(__double2hiint(tj[i]) + (m << 15), __double2loint(tj[i]));
  }
}

// DENS_TANH_S / DENS_EXP_S per element (any α): ψ, ψ′ (density.rs:58-63, 96-103),
// the raw Σψ′ term into dacc and the raw Σℓ term returned (density.rs:50-56,
// 91-94), in the same mask-free row-term forms as the table paths (every term
// vanishes at y = 0; finalize_row restores the per-sample constants).
template <int DENS>
__device__ __forceinline__ double safe_terms(double y, double alpha, double& dacc, double& psi, double& dpsi) {
  if constexpr (DENS == DENS_TANH_S) {
    const double th = tanh(alpha * y);
    psi = th;
    dacc = __builtin_fma(th, th, dacc);  // Σψ′ = α(n − Σ th²)
    dpsi = alpha * (1.0 - th * th);
    const double ay = fabs(y);
    return ay + (log(1.0 + exp(-2.0 * alpha * ay)) - fm::LN2) / alpha;  // Σℓ = Σ(·) + n·ln2/α
  } else {
    const double y2 = y * y;
    const double k = exp(-alpha / 2.0 * y2);
    const double em = k - 1.0;
    psi = y * k;
    dpsi = (1.0 - alpha * y2) * k;
    dacc += em - alpha * y2 * k;  // Σψ′ = n + Σ(k − 1 − αy²k)
    return em;                    // Σℓ = −(n + Σ(k − 1))/α
  }
}

// ψ (and ψ′ if NEED_D) of one 4-element fragment, NW elements interleaved at a
// time (register budget); accumulates the row terms in element order, so the
// sums do not depend on NW. Σy² only if NEED_Q (the reference uses Y∘Y only in
// non-orthogonal mode; cube needs it for Σψ′). m2a = −2α.
// th = −em/(2+em) uses one Newton step on v_rcp_f64 (≲ 10 ulp).
template <int DENS, bool NEED_D, bool NEED_Q, int NW = 4>
__device__ __forceinline__ void density_acc4(const d4& y, double alpha, double m2a, const double* tab, RowAcc& a,
                                             double (&psi)[4], double (&dpsi)[4]) {
  if constexpr (NEED_Q || DENS == DENS_CUBE)
#pragma unroll
    for (int i = 0; i < 4; ++i) a.q = __builtin_fma(y[i], y[i], a.q);
#pragma unroll
  for (int g = 0; g < 4; g += NW) {
    if constexpr (DENS == DENS_TANH) {
      double x[NW], emr[NW], sc[NW];
#pragma unroll
      for (int i = 0; i < NW; ++i) x[i] = fmax(m2a * fabs(y[g + i]), -708.0);  // = −2|αy| exactly (α > 0)
      exp_n<NW>(x, tab, emr, sc);
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        const double em = __builtin_fma(sc[i], emr[i], sc[i] - 1.0);  // e^{-2α|y|} − 1 ∈ (−1, 0]
        const double q = 2.0 + em;                                     // ∈ (1, 2], exactly 2 at y = 0
        const double th = copysign(-em * fm::rcp_nr1(q), y[g + i]);
        psi[g + i] = th;
        a.d = __builtin_fma(th, th, a.d);
        if constexpr (NEED_D) dpsi[g + i] = alpha * __builtin_fma(-th, th, 1.0);
        a.l += fabs(y[g + i]);
        a.p *= q;
      }
    } else if constexpr (DENS == DENS_EXP) {
      double x[NW], emr[NW], sc[NW];
#pragma unroll
      for (int i = 0; i < NW; ++i) x[i] = fmax(-alpha / 2.0 * (y[g + i] * y[g + i]), -708.0);
      exp_n<NW>(x, tab, emr, sc);
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        const double y2 = y[g + i] * y[g + i];
        const double k = __builtin_fma(sc[i], emr[i], sc[i]);
        const double em = k - 1.0;  // exactly 0 at y = 0
        const double ay2k = (alpha * y2) * k;
        psi[g + i] = y[g + i] * k;
        a.d += em - ay2k;
        if constexpr (NEED_D) dpsi[g + i] = k - ay2k;
        a.l += em;
      }
    } else if constexpr (DENS == DENS_CUBE) {
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        const double y2 = y[g + i] * y[g + i];
        psi[g + i] = y2 * y[g + i];
        if constexpr (NEED_D) dpsi[g + i] = 3.0 * y2;
        a.l = __builtin_fma(y2, y2, a.l);
      }
    } else if constexpr (DENS == DENS_TANH_S || DENS == DENS_EXP_S) {
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        double p, d;
        a.l += safe_terms<DENS>(y[g + i], alpha, a.d, p, d);
        psi[g + i] = p;
        if constexpr (NEED_D) dpsi[g + i] = d;
      }
    } else {  // LINEAR: ψ = y turns G_raw into the Gram Σ y yᵀ; row terms unused
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        psi[g + i] = y[g + i];
        if constexpr (NEED_D) dpsi[g + i] = 1.0;
      }
    }
  }
}

// ℓ terms only (line-search tries): identical arithmetic to density_acc4's ℓ part
template <int DENS, bool NEED_Q, int NW = 4, bool SCHED_FENCE = true>
__device__ __forceinline__ void loss_acc4(const d4& y, double alpha, double m2a, const double* tab, RowAcc& a) {
  if constexpr (NEED_Q || DENS == DENS_CUBE)  // as density_acc4 (cube's fused pass keeps Σy²)
#pragma unroll
    for (int i = 0; i < 4; ++i) a.q = __builtin_fma(y[i], y[i], a.q);
#pragma unroll
  for (int g = 0; g < 4; g += NW) {
    if constexpr (DENS == DENS_TANH) {
      double x[NW], emr[NW], sc[NW];
#pragma unroll
      for (int i = 0; i < NW; ++i) x[i] = fmax(m2a * fabs(y[g + i]), -708.0);
      exp_n<NW>(x, tab, emr, sc);
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        const double em = __builtin_fma(sc[i], emr[i], sc[i] - 1.0);
        a.l += fabs(y[g + i]);
        a.p *= 2.0 + em;
      }
      if constexpr (SCHED_FENCE) __builtin_amdgcn_sched_barrier(0);  // one group's chain live at a time
    } else if constexpr (DENS == DENS_EXP) {
      double x[NW], emr[NW], sc[NW];
#pragma unroll
      for (int i = 0; i < NW; ++i) x[i] = fmax(-alpha / 2.0 * (y[g + i] * y[g + i]), -708.0);
      exp_n<NW>(x, tab, emr, sc);
#pragma unroll
      for (int i = 0; i < NW; ++i) a.l += __builtin_fma(sc[i], emr[i], sc[i]) - 1.0;
    } else if constexpr (DENS == DENS_CUBE) {
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        const double y2 = y[g + i] * y[g + i];
        a.l = __builtin_fma(y2, y2, a.l);
      }
    } else if constexpr (DENS == DENS_TANH_S || DENS == DENS_EXP_S) {
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        double d_unused = 0.0, p, d;
        a.l += safe_terms<DENS>(y[g + i], alpha, d_unused, p, d);
      }
    }
  }
}

// ℓ terms of the line-search screen for tanh in fp32 (the screen's bound covers the error):
// Σ|y| in fp64 as the exact pass; the log term per lane and block as ONE v_log_f32 of the
// product of the 4 factors (1 + 2^z)/2 ∈ (1/2, 1], 2^z = e^{−2α|y|} by v_exp_f32 with
// z = fl32(|y|)·c32, c32 = fl32(−2α·log2 e). Every term vanishes at y = 0 (2^0 = 1,
// log2 1 = 0 exactly on the hardware, checked by k_check_f32_transc), so padding is free.
// Raw Σℓ = Σ|y| + (ln2/α)·g; finalize_row adds n·ln2/α as for the exact form.
// Error per block and lane (4 elements, in Σℓ units), DeviceCtx::screen_f32_block_bound.
__device__ __forceinline__ void loss_acc4_f32(const d4& y, float c32, RowAcc& a) {
  float pf = 1.0f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a.l += fabs(y[i]);
    const float z = (float)fabs(y[i]) * c32;
    pf *= __builtin_fmaf(__builtin_amdgcn_exp2f(z), 0.5f, 0.5f);
  }
  a.g += (double)__builtin_amdgcn_logf(pf);
}

// The same ℓ terms from the M waves' fp32 |ỹ| (k_eval_loss_oz, F32L): Σ|ỹ| of the 4 in fp32
// ((a0 + a2) + (a1 + a3): ≤ 2^-23·Σ relative) into the fp64 sum, z = ỹ·c32 (2 roundings: within
// the 3.0000002·2^-24 of screen_f32_block_bound), the rest as loss_acc4_f32; pairs of lanes go
// through the packed fp32 ops.
__device__ __forceinline__ void loss_acc4_f32y(const f4& y, float c32, RowAcc& a) {
  const f2 lo = {y[0], y[1]}, hi = {y[2], y[3]};
  const f2 s2 = lo + hi;
  a.l += (double)(s2[0] + s2[1]);
  const f2 zl = lo * c32, zh = hi * c32;
  f2 el = {__builtin_amdgcn_exp2f(zl[0]), __builtin_amdgcn_exp2f(zl[1])};
  f2 eh = {__builtin_amdgcn_exp2f(zh[0]), __builtin_amdgcn_exp2f(zh[1])};
  el = el * 0.5f + 0.5f;
  eh = eh * 0.5f + 0.5f;
  const f2 p2 = el * eh;
  a.g += (double)__builtin_amdgcn_logf(p2[0] * p2[1]);
}

// every ≤ 32 blocks (≤ 128 factors ∈ (1, 2] since the last call: no overflow);
// frexp is exact, so the cadence does not change any bits
constexpr int RENORM_BLOCKS = 32;
template <int DENS>
__device__ __forceinline__ void acc_renorm(RowAcc& a) {
  if constexpr (DENS == DENS_TANH) {
    int ex;
    a.p = frexp(a.p, &ex);
    a.e += ex;
  }
}

// per-lane raw Σℓ term (before the cross-lane sums)
// (nfac = number of factors in the tanh product: 4 per density call)
template <int DENS>
__device__ __forceinline__ double acc_ll(const RowAcc& a, double inv_alpha, int nfac) {
  if constexpr (DENS == DENS_TANH) {
    int ex;  // final renormalisation: (mantissa, exponent) no longer depends on the cadence
    const double m = frexp(a.p, &ex);
    return __builtin_fma(__builtin_fma((double)(a.e + ex - nfac), fm::LN2, log(m)), inv_alpha, a.l);
  }
  else
    return a.l;
}

// per-lane raw Σψ′ term (cube: ψ′ = 3y², so it is Σy² itself)
template <int DENS>
__device__ __forceinline__ double acc_dpsi(const RowAcc& a) {
  if constexpr (DENS == DENS_CUBE) return a.q;
  else return a.d;
}

// raw row sum → statistic (c: 0 Σψ′, 1 Σℓ, 2 Σy²), n = valid samples of this shard
__host__ __device__ inline double finalize_row(int dens, double alpha, double n, int c, double raw) {
  if (c == 2) return raw;
  if (dens == DENS_TANH_S) dens = DENS_TANH;
  if (dens == DENS_EXP_S) dens = DENS_EXP;
  if (dens == DENS_TANH) return c == 0 ? alpha * (n - raw) : raw + n * (0x1.62e42fefa39efp-1 / alpha);
  if (dens == DENS_EXP) return c == 0 ? n + raw : -(n + raw) / alpha;
  if (dens == DENS_CUBE) return c == 0 ? 3.0 * raw : 0.25 * raw;
  return c == 0 ? n : 0.0;  // LINEAR (Gram): unused
}

// density interleave widths (register budget: fused 256 VGPRs, split kernels 128)
constexpr int FUSED_NW = 2, LOSS_NW = 1, FROMY_NW = 1;

// End-of-block barrier of the store-epilogue kernels (k_ystore, k_tiled_yw):
// waits for this wave's LDS-DMA of the next block — issued BEFORE the block's
// NST global stores — but not for the stores themselves. vmcnt counts loads,
// stores and LDS-DMA together in issue order (MI355X_MICROARCH.md 's_waitcnt
// vmcnt(N)'), and __syncthreads() drains it to 0, which put every block's
// store round trip on the critical path. NST must be the exact number of
// vector-memory instructions this wave issued after its DMA (0 drains all).
template <int NST>
__device__ __forceinline__ void dma_barrier() {
  static_assert(NST >= 0 && NST < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
  __builtin_amdgcn_s_barrier();
}

#include "ozaki.inc"  // the int8-digit Y stage (k_eval_fused<4, …, OZ> uses it too)

// ---------------------------------------------------------------------------
// The fused pass. NB = 16-row blocks of Y (nc ≤ 16·NB), 8 waves.
// Block = TB = 16·(8/NB) samples; each wave owns one 16×16 Yᵀ tile of it.
// ---------------------------------------------------------------------------
constexpr int FUSED_THREADS = 512;
constexpr int KSMAX = 32;  // nf ≤ 128 (W fragments live in VGPRs)

template <int NB>
struct FusedShape {
  static constexpr int TS = 8 / NB;        // 16-sample sub-blocks per block
  static constexpr int TB = 16 * TS;       // samples per block
  static constexpr int NCP = 16 * NB;      // padded rows
  static constexpr int KK = 4 * TS;        // G-stage k-steps per block
  static constexpr int GI = NB == 8 ? 4 : 1;
  static constexpr int GJ = NB >= 4 ? 2 : 1;
  static constexpr int KSPL = NB == 2 ? 2 : (NB == 1 ? 8 : 1);
  static constexpr int KKW = KK / KSPL;
  static constexpr int FRAGS = KK * NB * 64;  // doubles per ψ / y LDS image
};

__host__ __device__ inline size_t fused_partial_stride(int ncp, bool need_h) {
  return (size_t)(need_h ? 2 : 1) * ncp * ncp + 3 * (size_t)ncp;
}

// Software-pipelined over blocks with ONE barrier per block: iteration b
// runs the Y stage of block b+1 (one MFMA accumulation chain) next to the G
// stage of block b (GI·GJ independent accumulators) in one basic block; X
// tiles and ψ/Y images are double-buffered. Loads of X use clamped block
// indices instead of branches (the last iteration is peeled); the row sums
// need no validity masks (RowAcc).
// X rows are padded to ldx ≡ 0 (mod 128) so a TB-sample tile never crosses a row end.
// OZ (NB = 4, nf ≤ 64, centred resident X): the Y stage runs on the int8 digit image
// (ozaki.inc: oz_ystage + oz_combine on 1 k-step, the arithmetic of k_eval_loss_oz<…, 4>,
// so the loss-only try and this pass give identical bits); the two 7-KiB digit images
// and the 32 scales of a block are staged by LDS-DMA in place of X.
template <int NB, bool NEED_H, int DENS, bool NEED_Q, bool OZ = false>
__global__ void __launch_bounds__(FUSED_THREADS, 2)
k_eval_fused(const double* __restrict__ X, uint64_t ldx, uint64_t n_local, int nf,
             const double* __restrict__ Wp, const double* __restrict__ mu, double alpha,
             uint64_t bpw, uint64_t n_blocks, double* __restrict__ partials,
             const uint8_t* __restrict__ xsl = nullptr, const double* __restrict__ xsc = nullptr,
             const uint8_t* __restrict__ wsl_g = nullptr, const double* __restrict__ wsc = nullptr) {
  static_assert(!OZ || NB == 4, "int8 Y stage of k_eval_fused: NB = 4");
  using S = FusedShape<NB>;
  constexpr int TS = S::TS, TB = S::TB, NCP = S::NCP, KKW = S::KKW, GI = S::GI, GJ = S::GJ;
  constexpr int NFP = 16 * NB;       // K of the Y stage, padded (zero X rows / zero W columns)
  constexpr int KS = NFP / 4;        // MFMA k-steps of the Y stage
  constexpr int XS = TS * NFP * 16;  // doubles per X tile (= 2048 for every NB)
  constexpr int N2 = XS / 2;         // double2 per X tile
  constexpr int PRE = N2 / FUSED_THREADS;
  static_assert(N2 % FUSED_THREADS == 0, "X tile must split evenly over the workgroup");
  constexpr int NIMG = NEED_H ? 3 : 2;  // ψ, y (, ψ′) images
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const int yi = wave % NB, yts = wave / NB;
  const double inv_alpha = 1.0 / alpha, m2a = -2.0 * alpha;

  extern __shared__ double smem[];
  EXP_TAB_DECL;
  exp_tab_load(s_exp_tab);
  double* xs0 = smem;             // [2][TS][NFP][16]
  double* img0 = smem + 2 * XS;   // [2][NIMG][KK][NB][64]

  double wf[OZ ? 1 : KS];
  v4i wsl[OZ ? OZ_SLICES : 1][1];
  double rsc = 0.0;
  if constexpr (OZ) {
#pragma unroll
    for (int a = 0; a < OZ_SLICES; ++a)
      wsl[a][0] = *(const v4i*)(wsl_g + (size_t)(((yi * OZ_SLICES + a) * 2 + 0) * 64 + lane) * 16);
    rsc = wsc[yi * 16 + lr];
  } else {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) wf[ks] = Wp[(yi * 16 + lr) * NFP + 4 * ks + lk];
  }

  int gi0, gj0, kk0;
  if constexpr (NB == 8) { gi0 = (wave >> 2) * 4; gj0 = (wave & 3) * 2; kk0 = 0; }
  else if constexpr (NB == 4) { gi0 = wave >> 1; gj0 = (wave & 1) * 2; kk0 = 0; }
  else if constexpr (NB == 2) { gi0 = (wave & 3) >> 1; gj0 = wave & 1; kk0 = (wave >> 2) * KKW; }
  else { gi0 = 0; gj0 = 0; kk0 = wave * KKW; }

  d4 accg[GI][GJ];
  d4 acch[GI][GJ];
#pragma unroll
  for (int i = 0; i < GI; ++i)
#pragma unroll
    for (int j = 0; j < GJ; ++j) { accg[i][j] = d4{0, 0, 0, 0}; acch[i][j] = d4{0, 0, 0, 0}; }
  RowAcc racc;

  const uint64_t b_begin = (uint64_t)blockIdx.x * bpw;
  const uint64_t b_end = b_begin + bpw < n_blocks ? b_begin + bpw : n_blocks;
  const uint64_t b_last = b_end - 1;

  // per-thread X staging slots: row k, sample pair t (fixed for the launch).
  // Rows k ≥ nf re-read row 0: their W columns are zero, so they add exactly 0.
  int xk[PRE], xt[PRE];
  double xmu[PRE];
  const double* xsrc[PRE];
#pragma unroll
  for (int p = 0; p < PRE; ++p) {
    const int e = tid + p * FUSED_THREADS;
    xk[p] = e / (TB / 2);
    xt[p] = 2 * (e % (TB / 2));
    const bool ok = xk[p] < nf;
    xmu[p] = (ok && mu) ? mu[xk[p]] : 0.0;
    xsrc[p] = X + (size_t)(ok ? xk[p] : 0) * ldx + xt[p];
  }
  // two register sets for the X prefetch: the set stored in iteration b was
  // loaded at the START of iteration b−1, a full iteration of latency hiding
  double2 preA[PRE], preB[PRE];
  auto load_x = [&](uint64_t b, double2 (&pre)[PRE]) {  // b ≤ b_last: always a valid address
#pragma unroll
    for (int p = 0; p < PRE; ++p) pre[p] = *reinterpret_cast<const double2*>(xsrc[p] + b * TB);
  };
  // X̃ = X − μ into LDS; samples past n_local become exact zeros (only the
  // grid's last block can hold any: a uniform branch, no per-element selects)
  auto store_x = [&](uint64_t b, double* xs, const double2 (&pre)[PRE]) {
    if (b * TB + TB <= n_local) {
#pragma unroll
      for (int p = 0; p < PRE; ++p) {
        const double2 v = double2{pre[p].x - xmu[p], pre[p].y - xmu[p]};
        *reinterpret_cast<double2*>(xs + ((xt[p] >> 4) * NFP + xk[p]) * 16 + (xt[p] & 15)) = v;
      }
    } else {
#pragma unroll
      for (int p = 0; p < PRE; ++p) {
        const uint64_t tg = b * TB + xt[p];
        double2 v;
        v.x = tg < n_local ? pre[p].x - xmu[p] : 0.0;
        v.y = tg + 1 < n_local ? pre[p].y - xmu[p] : 0.0;
        *reinterpret_cast<double2*>(xs + ((xt[p] >> 4) * NFP + xk[p]) * 16 + (xt[p] & 15)) = v;
      }
    }
  };
  // Y stage: Yᵀ tile (16 samples × 16 rows) = Xᵀ·Wᵀ over NFP as ONE accumulation
  // chain (back-to-back dependent fp64 MFMAs issue at full rate on gfx950:
  // tools/microbench/mfma_chain.hip), in the same order as k_eval_loss
  constexpr int OZT = oz_block_bytes<1>();  // OZ: one 16-sample sub-block's digit image
  static_assert(!OZ || 2 * OZT + 256 <= XS * (int)sizeof(double), "digit images fit the X tile");
  auto y_stage = [&](const double* xs) {
    if constexpr (OZ) {
      v4i acc[OZ_SLICES];
      const uint8_t* tile = (const uint8_t*)xs + yts * OZT;
      oz_ystage<OZ_SLICES - 1, 1>(tile, lane, wsl, acc);
      const double* scd = (const double*)((const uint8_t*)xs + 2 * OZT) + yts * 16;
      const double x4[4] = {scd[lk], scd[lk + 4], scd[lk + 8], scd[lk + 12]};
      return oz_combine(acc, rsc, x4);
    } else {
      d4 ya = d4{0, 0, 0, 0};
      const double* xrow = xs + (yts * NFP + lk) * 16 + lr;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) ya = mfma(xrow[(4 * ks) * 16], wf[ks], ya);
      return ya;
    }
  };
  // OZ: block b's 2 × 7 digit planes (1 KiB each) and its 32 scales → xs by LDS-DMA; wave w
  // moves items w and w + 8 of the 15 (item 14: the scales, 4 B per lane)
  auto stage_oz = [&](uint64_t b, double* xs) {
    uint8_t* dst = (uint8_t*)xs;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = wave + 8 * u;
      if (it < 14)
        __builtin_amdgcn_global_load_lds((gbl_vptr)(xsl + (2 * b) * OZT + it * 1024 + lane * 16),
                                         (lds_vptr)(dst + it * 1024), 16, 0, 0);
      else if (it == 14)
        __builtin_amdgcn_global_load_lds((gbl_vptr)((const uint32_t*)(xsc + b * 32) + lane),
                                         (lds_vptr)(dst + 2 * OZT), 4, 0, 0);
    }
  };
  // density on the tile, row terms, hand-off of the ψ / y (/ ψ′) fragments
  auto elementwise = [&](const d4& yv, double* img) {
    double psi[4], dpsi[4];
    density_acc4<DENS, NEED_H, NEED_Q, FUSED_NW>(yv, alpha, m2a, s_exp_tab, racc, psi, dpsi);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = ((yts * 4 + r) * NB + yi) * 64 + lane;
      img[f] = psi[r];
      img[S::FRAGS + f] = yv[r];
      if constexpr (NEED_H) img[2 * S::FRAGS + f] = dpsi[r];
    }
  };
  // G stage: G_raw[i-blocks][j-blocks] += ψ · Yᵀ (H_raw += ψ′ · (Y∘Y)ᵀ) over one block
  auto g_stage = [&](const double* img) {
#pragma unroll
    for (int q = 0; q < KKW; ++q) {
      const int kk = kk0 + q;
      double pa[GI], yf[GJ];
#pragma unroll
      for (int i = 0; i < GI; ++i) pa[i] = img[(kk * NB + gi0 + i) * 64 + lane];
#pragma unroll
      for (int j = 0; j < GJ; ++j) yf[j] = img[S::FRAGS + (kk * NB + gj0 + j) * 64 + lane];
#pragma unroll
      for (int i = 0; i < GI; ++i)
#pragma unroll
        for (int j = 0; j < GJ; ++j) accg[i][j] = mfma(pa[i], yf[j], accg[i][j]);
      if constexpr (NEED_H) {
#pragma unroll
        for (int i = 0; i < GI; ++i) {
          const double da = img[2 * S::FRAGS + (kk * NB + gi0 + i) * 64 + lane];
#pragma unroll
          for (int j = 0; j < GJ; ++j) acch[i][j] = mfma(da, yf[j] * yf[j], acch[i][j]);
        }
      }
    }
  };

  if (OZ && b_begin < b_end) {  // the same schedule with the digit images staged by DMA
    auto clampb = [&](uint64_t b) { return b < b_last ? b : b_last; };
    stage_oz(b_begin, xs0);
    __syncthreads();  // (also waits for this wave's LDS-DMA)
    elementwise(y_stage(xs0), img0);
    stage_oz(clampb(b_begin + 1), xs0 + XS);
    __syncthreads();
    // iteration b: block b+2 → xs[cur] (block b was consumed in iteration b−1) ‖ Y stage of
    // b+1 ‖ G stage of b
    auto iter = [&](uint64_t b, int cur) {
      stage_oz(clampb(b + 2), xs0 + cur * XS);
      const d4 yv = y_stage(xs0 + (cur ^ 1) * XS);     // block b+1
      g_stage(img0 + cur * NIMG * S::FRAGS);           // block b
      elementwise(yv, img0 + (cur ^ 1) * NIMG * S::FRAGS);
      __syncthreads();
    };
    uint64_t b = b_begin;
    while (b + 1 < b_last) {
      const uint64_t lim = b + RENORM_BLOCKS < b_last ? b + RENORM_BLOCKS : b_last;
      for (; b + 1 < lim; b += 2) {
        iter(b, 0);
        iter(b + 1, 1);
      }
      acc_renorm<DENS>(racc);
    }
    int cur = 0;
    if (b < b_last) {
      iter(b, 0);
      cur = 1;
    }
    g_stage(img0 + cur * NIMG * S::FRAGS);  // block b_last
    __syncthreads();
  } else if (b_begin < b_end) {
    auto clampb = [&](uint64_t b) { return b < b_last ? b : b_last; };
    // prologue: X(b0) → xs[0]; Y + density of b0 → img[0]; X(b0+1) → xs[1]; X(b0+2) → preA
    load_x(b_begin, preA);
    store_x(b_begin, xs0, preA);
    load_x(clampb(b_begin + 1), preA);
    __syncthreads();
    elementwise(y_stage(xs0), img0);
    store_x(clampb(b_begin + 1), xs0 + XS, preA);
    load_x(clampb(b_begin + 2), preA);
    __syncthreads();
    // iteration b: Y stage of b+1 ‖ G stage of b; X(b+2) (loaded a full iteration
    // ago) → xs[cur]; X(b+3) requested at the top. A clamped (repeated) block is
    // never consumed twice: its Y stage is the peeled tail's, which is skipped.
    auto iter = [&](uint64_t b, int cur, double2 (&use)[PRE], double2 (&fill)[PRE]) {
      load_x(clampb(b + 3), fill);
      const d4 yv = y_stage(xs0 + (cur ^ 1) * XS);     // block b+1
      g_stage(img0 + cur * NIMG * S::FRAGS);           // block b
      elementwise(yv, img0 + (cur ^ 1) * NIMG * S::FRAGS);
      store_x(clampb(b + 2), xs0 + cur * XS, use);
      __syncthreads();
    };
    uint64_t b = b_begin;
    while (b + 1 < b_last) {  // chunks of RENORM_BLOCKS blocks, renormalised after each
      const uint64_t lim = b + RENORM_BLOCKS < b_last ? b + RENORM_BLOCKS : b_last;
      for (; b + 1 < lim; b += 2) {
        iter(b, 0, preA, preB);
        iter(b + 1, 1, preB, preA);
      }
      acc_renorm<DENS>(racc);
    }
    int cur = 0;
    if (b < b_last) {
      iter(b, 0, preA, preB);
      cur = 1;
    }
    g_stage(img0 + cur * NIMG * S::FRAGS);  // block b_last
    __syncthreads();
  }

  // ---- epilogue: per-workgroup partials [G | H | Σψ′ | Σℓ | Σy²]
  double* out = partials + (size_t)blockIdx.x * fused_partial_stride(NCP, NEED_H);
  double* red = img0;  // scratch (all waves are past the last barrier)
  if constexpr (S::KSPL == 1) {
#pragma unroll
    for (int i = 0; i < GI; ++i)
#pragma unroll
      for (int j = 0; j < GJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = (gi0 + i) * 16 + lk + 4 * r, col = (gj0 + j) * 16 + lr;
          out[row * NCP + col] = accg[i][j][r];
          if constexpr (NEED_H) out[NCP * NCP + row * NCP + col] = acch[i][j][r];
        }
  } else {
    // waves that split one G block's k range meet in LDS, summed in wave order
    constexpr int NBLK = NB * NB;
    const int blk = gi0 * NB + gj0;
    const int sp = kk0 / KKW;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[(sp * NBLK + blk) * 256 + r * 64 + lane] = accg[0][0][r];
      if constexpr (NEED_H) red[(S::KSPL + sp) * NBLK * 256 + blk * 256 + r * 64 + lane] = acch[0][0][r];
    }
    __syncthreads();
    if (sp == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double g = 0.0, h = 0.0;
        for (int s2 = 0; s2 < S::KSPL; ++s2) {
          g += red[(s2 * NBLK + blk) * 256 + r * 64 + lane];
          if constexpr (NEED_H) h += red[(S::KSPL + s2) * NBLK * 256 + blk * 256 + r * 64 + lane];
        }
        const int row = gi0 * 16 + lk + 4 * r, col = gj0 * 16 + lr;
        out[row * NCP + col] = g;
        if constexpr (NEED_H) out[NCP * NCP + row * NCP + col] = h;
      }
    }
    __syncthreads();
  }
  // row sums: over the 4 lane groups, then over the TS waves of one row block
  const int nfac = b_begin < b_end ? 4 * (int)(b_end - b_begin) : 0;  // one density call per block
  double rs_dpsi = acc_dpsi<DENS>(racc), rs_ll = acc_ll<DENS>(racc, inv_alpha, nfac), rs_y2 = racc.q;
  rs_dpsi += __shfl_xor(rs_dpsi, 16); rs_dpsi += __shfl_xor(rs_dpsi, 32);
  rs_ll += __shfl_xor(rs_ll, 16);     rs_ll += __shfl_xor(rs_ll, 32);
  rs_y2 += __shfl_xor(rs_y2, 16);     rs_y2 += __shfl_xor(rs_y2, 32);
  double* rsb = xs0;  // [TS][NCP][3]
  if (lk == 0) {
    rsb[(yts * NCP + yi * 16 + lr) * 3 + 0] = rs_dpsi;
    rsb[(yts * NCP + yi * 16 + lr) * 3 + 1] = rs_ll;
    rsb[(yts * NCP + yi * 16 + lr) * 3 + 2] = rs_y2;
  }
  __syncthreads();
  double* orow = out + (size_t)(NEED_H ? 2 : 1) * NCP * NCP;
  for (int e = tid; e < NCP * 3; e += FUSED_THREADS) {
    const int row = e / 3, c = e % 3;
    double sum = 0.0;
    for (int ts = 0; ts < TS; ++ts) sum += rsb[(ts * NCP + row) * 3 + c];
    orow[c * NCP + row] = sum;
  }
}

// ---------------------------------------------------------------------------
// Warp-specialised fused pass for NB = 8 (64 < nc ≤ 128, no H), 16 waves:
//   waves 0-7  ("Y waves"): Y stage + density of row block w (W fragment in
//              VGPRs), ψ / y fragments → LDS images;
//   waves 8-15 ("G waves"): the G tiles of k_eval_fused<8> (GI = 4 × GJ = 2
//              accumulators in VGPRs) and the X staging (LDS-DMA of the centred
//              resident X, issued a full iteration ahead).
// k_eval_fused<8> holds both roles in every wave (256 VGPRs: 2 waves per SIMD,
// the barrier and MFMA → VALU latencies exposed); split, each role fits 128
// VGPRs and a CU runs 4 waves per SIMD. Each role runs its own loop (so the W
// fragments and the accumulators are never live at once) with the same number
// of barriers. Same block partition, G-tile map, k order, lane map and row-term
// formulas as k_eval_fused<8> / k_eval_loss<8> / k_eval_fromy<8>: identical sums.
// ---------------------------------------------------------------------------
#include "fused_ws.inc"
#include "fused_g8.inc"   // G = ψ·Yᵀ on int8 digits: the arithmetic
#include "fused_g8x.inc"  // … and the kernel (8 waves, G interleaved with the Y stage)

// ---------------------------------------------------------------------------
// Split evaluation for line-search tries (bit-identical sums to k_eval_fused):
//   k_eval_loss  — Y stage + Σℓ, Σy² only (half the MFMA work, no ψ/ψ′), and
//                  optionally Y written to HBM in MFMA-fragment order;
//   k_eval_fromy — reads that Y back (coalesced 512-B fragments), ψ, ψ′ and
//                  the G (H) stage: the rest of the statistics of an accepted try.
// A rejected try then costs ≈ half a fused pass.
// ---------------------------------------------------------------------------

template <int NB, int DENS, bool STORE, bool NEED_Q>
__global__ void __launch_bounds__(FUSED_THREADS, 4)
k_eval_loss(const double* __restrict__ X, uint64_t ldx, uint64_t n_local, int nf,
            const double* __restrict__ Wp, const double* __restrict__ mu, double alpha,
            uint64_t bpw, uint64_t n_blocks, double* __restrict__ partials, double* __restrict__ ybuf) {
  using S = FusedShape<NB>;
  constexpr int TS = S::TS, TB = S::TB, NCP = S::NCP;
  constexpr int NFP = 16 * NB, KS = NFP / 4, XS = TS * NFP * 16, N2 = XS / 2, PRE = N2 / FUSED_THREADS;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const int yi = wave % NB, yts = wave / NB;
  const double inv_alpha = 1.0 / alpha, m2a = -2.0 * alpha;
  extern __shared__ double smem[];
  EXP_TAB_DECL;
  exp_tab_load(s_exp_tab);
  double* xs0 = smem;  // [2][TS][NFP][16]
  double wf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) wf[ks] = Wp[(yi * 16 + lr) * NFP + 4 * ks + lk];
  RowAcc racc;
  // this workgroup's blocks b_begin + i, i < nb; block indices are 32-bit and
  // wave-uniform inside the loop (scalar compares, no 64-bit VALU compares
  // holding VGPRs); blocks i < nfull hold no padding
  const uint64_t b_begin = (uint64_t)blockIdx.x * bpw;
  const uint64_t b_end = b_begin + bpw < n_blocks ? b_begin + bpw : n_blocks;
  const uint32_t nb = b_begin < b_end ? (uint32_t)(b_end - b_begin) : 0u;
  const uint64_t nfull_g = n_local / TB;
  const uint32_t nfull = nfull_g > b_begin ? (uint32_t)(nfull_g - b_begin < nb ? nfull_g - b_begin : nb) : 0u;
  int xk[PRE], xt[PRE];
  double xmu[PRE];
  const double* xsrc[PRE];
#pragma unroll
  for (int p = 0; p < PRE; ++p) {  // same staging map as k_eval_fused (rows ≥ nf: zero W columns)
    const int e = tid + p * FUSED_THREADS;
    xk[p] = e / (TB / 2);
    xt[p] = 2 * (e % (TB / 2));
    const bool ok = xk[p] < nf;
    xmu[p] = (ok && mu) ? mu[xk[p]] : 0.0;
    xsrc[p] = X + (size_t)(ok ? xk[p] : 0) * ldx + xt[p] + b_begin * TB;
  }
  // one prefetch register set (128-VGPR budget): X(b+1) is requested at the top
  // of iteration b — pinned there by a scheduling barrier — and consumed after
  // the Y stage and the density math of block b, which hide its HBM latency
  double2 pre[PRE];
  auto load_x = [&](uint32_t i) {
#pragma unroll
    for (int p = 0; p < PRE; ++p) pre[p] = *reinterpret_cast<const double2*>(xsrc[p] + (size_t)i * TB);
  };
  auto store_x = [&](uint32_t i, double* xs) {
    if (i < nfull) {
#pragma unroll
      for (int p = 0; p < PRE; ++p) {
        const double2 v = double2{pre[p].x - xmu[p], pre[p].y - xmu[p]};
        *reinterpret_cast<double2*>(xs + ((xt[p] >> 4) * NFP + xk[p]) * 16 + (xt[p] & 15)) = v;
      }
    } else {
#pragma unroll
      for (int p = 0; p < PRE; ++p) {
        const uint64_t tg = (b_begin + i) * TB + xt[p];
        double2 v;
        v.x = tg < n_local ? pre[p].x - xmu[p] : 0.0;
        v.y = tg + 1 < n_local ? pre[p].y - xmu[p] : 0.0;
        *reinterpret_cast<double2*>(xs + ((xt[p] >> 4) * NFP + xk[p]) * 16 + (xt[p] & 15)) = v;
      }
    }
  };
  if (nb > 0) {
    load_x(0);
    store_x(0, xs0);
    __syncthreads();
    int cur = 0;
    // chunks of RENORM_BLOCKS blocks, the product renormalised after each (a
    // loop-level call, so it costs no per-block selects)
    for (uint32_t c0 = 0; c0 < nb; c0 += RENORM_BLOCKS) {
      const uint32_t c1 = c0 + RENORM_BLOCKS < nb ? c0 + RENORM_BLOCKS : nb;
      for (uint32_t i = c0; i < c1; ++i) {
        const uint32_t inext = i + 1 < nb ? i + 1 : nb - 1;  // clamped: always a valid address
        load_x(inext);
        __builtin_amdgcn_sched_barrier(0);
        d4 yv = d4{0, 0, 0, 0};  // one chain, same order as k_eval_fused's Y stage
        const double* xrow = xs0 + cur * XS + (yts * NFP + lk) * 16 + lr;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) yv = mfma(xrow[(4 * ks) * 16], wf[ks], yv);
        // X(i+1) → the other buffer before the density math (its load had the
        // whole MFMA chain to land), so nothing of the density is sunk past the
        // staging branch and no table value stays live across it
        store_x(inext, xs0 + (cur ^ 1) * XS);
        loss_acc4<DENS, NEED_Q, LOSS_NW>(yv, alpha, m2a, s_exp_tab, racc);
        if constexpr (STORE)
#pragma unroll
          for (int r = 0; r < 4; ++r) ybuf[(((b_begin + i) * 8 + wave) * 4 + r) * 64 + lane] = yv[r];
        __syncthreads();
        cur ^= 1;
      }
      acc_renorm<DENS>(racc);
    }
  }
  double rs_ll = acc_ll<DENS>(racc, inv_alpha, 4 * (int)nb), rs_y2 = racc.q;
  rs_ll += __shfl_xor(rs_ll, 16); rs_ll += __shfl_xor(rs_ll, 32);
  rs_y2 += __shfl_xor(rs_y2, 16); rs_y2 += __shfl_xor(rs_y2, 32);
  double* rsb = xs0;  // [TS][NCP][2]
  if (lk == 0) {
    rsb[(yts * NCP + yi * 16 + lr) * 2 + 0] = rs_ll;
    rsb[(yts * NCP + yi * 16 + lr) * 2 + 1] = rs_y2;
  }
  __syncthreads();
  double* out = partials + (size_t)blockIdx.x * 2 * NCP;  // [Σℓ | Σy²]
  for (int e = tid; e < NCP * 2; e += FUSED_THREADS) {
    const int row = e / 2, c = e % 2;
    double sum = 0.0;
    for (int ts = 0; ts < TS; ++ts) sum += rsb[(ts * NCP + row) * 2 + c];
    out[c * NCP + row] = sum;
  }
}

#include "loss2.inc"

template <int NB, bool NEED_H, int DENS>
__global__ void __launch_bounds__(FUSED_THREADS, 4)
k_eval_fromy(const double* __restrict__ ybuf, uint64_t n_local, double alpha, uint64_t bpw, uint64_t n_blocks,
             double* __restrict__ partials) {
  using S = FusedShape<NB>;
  constexpr int TS = S::TS, TB = S::TB, NCP = S::NCP, KKW = S::KKW, GI = S::GI, GJ = S::GJ;
  constexpr int NIMG = NEED_H ? 3 : 2;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const int yi = wave % NB, yts = wave / NB;
  const double inv_alpha = 1.0 / alpha;
  extern __shared__ double smem[];
  EXP_TAB_DECL;
  exp_tab_load(s_exp_tab);
  __syncthreads();  // the first density call precedes the pipeline's first barrier
  double* img0 = smem;  // [2][NIMG][KK][NB][64]
  int gi0, gj0, kk0;
  if constexpr (NB == 8) { gi0 = (wave >> 2) * 4; gj0 = (wave & 3) * 2; kk0 = 0; }
  else if constexpr (NB == 4) { gi0 = wave >> 1; gj0 = (wave & 1) * 2; kk0 = 0; }
  else if constexpr (NB == 2) { gi0 = (wave & 3) >> 1; gj0 = wave & 1; kk0 = (wave >> 2) * KKW; }
  else { gi0 = 0; gj0 = 0; kk0 = wave * KKW; }
  d4 accg[GI][GJ];
  d4 acch[GI][GJ];
#pragma unroll
  for (int i = 0; i < GI; ++i)
#pragma unroll
    for (int j = 0; j < GJ; ++j) { accg[i][j] = d4{0, 0, 0, 0}; acch[i][j] = d4{0, 0, 0, 0}; }
  RowAcc racc;
  (void)n_local;
  const uint64_t b_begin = (uint64_t)blockIdx.x * bpw;
  const uint64_t b_end = b_begin + bpw < n_blocks ? b_begin + bpw : n_blocks;
  const uint64_t b_last = b_end - 1;
  auto load_y = [&](uint64_t b) {
    d4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = ybuf[((b * 8 + wave) * 4 + r) * 64 + lane];
    return v;
  };
  auto elementwise = [&](const d4& yv, double* img) {
    double psi[4], dpsi[4];
    density_acc4<DENS, NEED_H, false, FROMY_NW>(yv, alpha, -2.0 * alpha, s_exp_tab, racc, psi, dpsi);  // ℓ, Σy² terms unused
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = ((yts * 4 + r) * NB + yi) * 64 + lane;
      img[f] = psi[r];
      img[S::FRAGS + f] = yv[r];
      if constexpr (NEED_H) img[2 * S::FRAGS + f] = dpsi[r];
    }
  };
  auto g_stage = [&](const double* img) {
#pragma unroll
    for (int q = 0; q < KKW; ++q) {
      const int kk = kk0 + q;
      double pa[GI], yf[GJ];
#pragma unroll
      for (int i = 0; i < GI; ++i) pa[i] = img[(kk * NB + gi0 + i) * 64 + lane];
#pragma unroll
      for (int j = 0; j < GJ; ++j) yf[j] = img[S::FRAGS + (kk * NB + gj0 + j) * 64 + lane];
#pragma unroll
      for (int i = 0; i < GI; ++i)
#pragma unroll
        for (int j = 0; j < GJ; ++j) accg[i][j] = mfma(pa[i], yf[j], accg[i][j]);
      if constexpr (NEED_H) {
#pragma unroll
        for (int i = 0; i < GI; ++i) {
          const double da = img[2 * S::FRAGS + (kk * NB + gi0 + i) * 64 + lane];
#pragma unroll
          for (int j = 0; j < GJ; ++j) acch[i][j] = mfma(da, yf[j] * yf[j], acch[i][j]);
        }
      }
    }
  };
  if (b_begin < b_end) {
    auto clampb = [&](uint64_t b) { return b < b_last ? b : b_last; };
    elementwise(load_y(b_begin), img0);
    d4 pre = load_y(clampb(b_begin + 1));
    __syncthreads();
    int cur = 0;
    for (uint64_t b = b_begin; b < b_last; ++b) {
      const d4 yv = pre;
      pre = load_y(clampb(b + 2));
      g_stage(img0 + cur * NIMG * S::FRAGS);
      elementwise(yv, img0 + (cur ^ 1) * NIMG * S::FRAGS);
      __syncthreads();
      cur ^= 1;
    }
    g_stage(img0 + cur * NIMG * S::FRAGS);
    __syncthreads();
  }
  double* out = partials + (size_t)blockIdx.x * fused_partial_stride(NCP, NEED_H);
  double* red = img0;
  if constexpr (S::KSPL == 1) {
#pragma unroll
    for (int i = 0; i < GI; ++i)
#pragma unroll
      for (int j = 0; j < GJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = (gi0 + i) * 16 + lk + 4 * r, col = (gj0 + j) * 16 + lr;
          out[row * NCP + col] = accg[i][j][r];
          if constexpr (NEED_H) out[NCP * NCP + row * NCP + col] = acch[i][j][r];
        }
  } else {
    constexpr int NBLK = NB * NB;
    const int blk = gi0 * NB + gj0;
    const int sp = kk0 / KKW;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[(sp * NBLK + blk) * 256 + r * 64 + lane] = accg[0][0][r];
      if constexpr (NEED_H) red[(S::KSPL + sp) * NBLK * 256 + blk * 256 + r * 64 + lane] = acch[0][0][r];
    }
    __syncthreads();
    if (sp == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double g = 0.0, h = 0.0;
        for (int s2 = 0; s2 < S::KSPL; ++s2) {
          g += red[(s2 * NBLK + blk) * 256 + r * 64 + lane];
          if constexpr (NEED_H) h += red[(S::KSPL + s2) * NBLK * 256 + blk * 256 + r * 64 + lane];
        }
        const int row = gi0 * 16 + lk + 4 * r, col = gj0 * 16 + lr;
        out[row * NCP + col] = g;
        if constexpr (NEED_H) out[NCP * NCP + row * NCP + col] = h;
      }
    }
    __syncthreads();
  }
  double rs_dpsi = acc_dpsi<DENS>(racc);
  rs_dpsi += __shfl_xor(rs_dpsi, 16); rs_dpsi += __shfl_xor(rs_dpsi, 32);
  double* rsb = img0 + 2 * NIMG * S::FRAGS - TS * NCP;  // [TS][NCP] at the end of the image area
  __syncthreads();
  if (lk == 0) rsb[yts * NCP + yi * 16 + lr] = rs_dpsi;
  __syncthreads();
  double* orow = out + (size_t)(NEED_H ? 2 : 1) * NCP * NCP;
  for (int row = tid; row < NCP; row += FUSED_THREADS) {
    double sum = 0.0;
    for (int ts = 0; ts < TS; ++ts) sum += rsb[ts * NCP + row];
    orow[row] = sum;
  }
}

// Fixed-order sum of per-workgroup partials, shared by every reduction of the
// register-resident kernels so their common statistics stay bit-identical: a
// 256-thread block reduces 64 outputs, each as 4 contiguous groups of workgroups
// summed in order, then ((g0 + g1) + (g2 + g3)).
constexpr int RED_OUT = 64;
__device__ __forceinline__ double reduce_partials(const double* __restrict__ p, int nwg, size_t pstride, bool ok,
                                                  double (*red)[RED_OUT]) {
  const int g = threadIdx.x / RED_OUT, o = threadIdx.x % RED_OUT;
  double s = 0.0;
  if (ok) {
    // loads 8 at a time (in flight together), added in the same order: the latency of a
    // serial chain of 128 L2/HBM loads was most of this kernel's time at small T
    const int w1 = nwg * (g + 1) / 4;
    int w = nwg * g / 4;
    for (; w + 8 <= w1; w += 8) {
      double v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = p[(size_t)(w + j) * pstride];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; w < w1; ++w) s += p[(size_t)w * pstride];
  }
  red[g][o] = s;
  __syncthreads();
  return (red[0][o] + red[1][o]) + (red[2][o] + red[3][o]);
}

// min, max and a NaN flag of the n sample scales 2^e_t, per workgroup: out[3·b + {0, 1, 2}]
// per workgroup: min, max, NaN flag and Σ v² of the sample scales v = 2^e_t (out[4·wg + c])
__global__ void __launch_bounds__(256) k_xsc_range(const double* __restrict__ xsc, uint64_t n, double* __restrict__ out) {
  __shared__ double s[4][256];
  double lo = INFINITY, hi = 0.0, nan = 0.0, sq = 0.0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const double v = xsc[i];
    if (v != v) nan = 1.0;
    else { lo = fmin(lo, v); hi = fmax(hi, v); sq = __builtin_fma(v, v, sq); }
  }
  s[0][threadIdx.x] = lo; s[1][threadIdx.x] = hi; s[2][threadIdx.x] = nan; s[3][threadIdx.x] = sq;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      s[0][threadIdx.x] = fmin(s[0][threadIdx.x], s[0][threadIdx.x + h]);
      s[1][threadIdx.x] = fmax(s[1][threadIdx.x], s[1][threadIdx.x + h]);
      s[2][threadIdx.x] = fmax(s[2][threadIdx.x], s[2][threadIdx.x + h]);
      s[3][threadIdx.x] += s[3][threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x < 4) out[4 * blockIdx.x + threadIdx.x] = s[threadIdx.x][0];
}

// out[c·nc + row] = Σ_w partials[w·pstride + poff + c·ncp + row], c < nsets,
// then finalize_row(dens, α, n, c0 + c, ·) unless dens < 0 (already final);
// c0 < 0: the sets alternate [Σℓ, Σy²] per try (multi-try layout)
__global__ void __launch_bounds__(256) k_reduce_rows(const double* __restrict__ partials, int nwg, size_t pstride,
                                                     size_t poff, int ncp, int nc, int nsets,
                                                     double* __restrict__ out, int dens, double alpha, double n,
                                                     int c0) {
  __shared__ double red[4][RED_OUT];
  const int e = blockIdx.x * RED_OUT + threadIdx.x % RED_OUT;
  const bool ok = e < nsets * nc;
  const int c = ok ? e / nc : 0, row = ok ? e % nc : 0;
  const double s = reduce_partials(partials + poff + (size_t)c * ncp + row, nwg, pstride, ok, red);
  if (ok && threadIdx.x < RED_OUT)
    out[e] = dens < 0 ? s : finalize_row(dens, alpha, n, c0 < 0 ? 1 + (c & 1) : c0 + c, s);
}

// ---------------------------------------------------------------------------
// Tiled two-phase pass for the shapes the register-resident fused kernel does
// not cover: any n_components (BASELINE C4: N = 256 non-ortho), H at nc > 64,
// any n_features (n_components < n_features), and tanh/exp at α ≤ 0.
//   phase 1 (k_tiled_yw): Y = W·X̃ per 16-sample block on MFMA with W in VGPRs,
//     density, row sums, and y, ψ (, ψ′) written to HBM in MFMA-fragment order
//     (512-B coalesced); features beyond 256 come in chunks of 256 whose
//     partial Y goes through the y buffer (MODE 2) and is picked up by the next
//     chunk's chain (yin);
//   phase 2 (k_tiled_gram2): G_raw (, H_raw) = Σ_t ψ_t y_tᵀ (ψ′_t (y_t∘y_t)ᵀ) on
//     MFMA, one 128×128 output tile per workgroup, T split over workgroups.
// ---------------------------------------------------------------------------
constexpr int TL_TT = 64;   // samples per tile (fragment layout unit: 4 blocks of 16)
constexpr int TL_TS = TL_TT / 16;
constexpr int TL_KMAX = 256;  // features per phase-1 chunk (W fragments in VGPRs)

__host__ __device__ inline size_t tl_frag(uint64_t tt, int ib, int ts, int r, int nib) {
  return ((((size_t)tt * nib + ib) * TL_TS + ts) * 4 + r) * 64;
}

// XCD-aware decode of a 1D grid into (sample range x, role): blocks b and b + 8
// land on one XCD (round-robin dispatch; MI355X_MICROARCH.md "Workgroup
// dispatch"), so the nroles roles of range x are consecutive slots of ONE XCD,
// start together and share that XCD's L2: X (or the fragments) is fetched from
// HBM once per range instead of once per role. Placement is a speed matter
// only; the grid is 8·⌈nx/8⌉·nroles blocks and those with x ≥ nx exit at once.
__device__ __forceinline__ bool xcd_decode(int nroles, uint64_t nx, uint64_t& x, int& role) {
  const unsigned i = blockIdx.x, slot = i >> 3;
  role = (int)(slot % (unsigned)nroles);
  x = (uint64_t)(slot / (unsigned)nroles) * 8 + (i & 7);
  return x < nx;
}
__host__ inline unsigned xcd_grid(uint64_t nx, int nroles) { return (unsigned)((nx + 7) / 8 * 8 * nroles); }

// Phase 1 with W in registers: the workgroup role blockIdx.y owns output rows
// [128·role, 128·role + 128); wave w owns row block ib = 8·role + w and keeps
// its W fragment (16 rows × 4·KS features of this chunk) in VGPRs for the whole
// launch, so W is read once. X̃ blocks of 16 samples × 4·KS features are staged
// by LDS-DMA (shared by the 8 waves; double-buffered, one barrier per block)
// and Yᵀ tiles come from ONE chain of KS MFMAs per wave, as in k_eval_fused.
// Row terms use the mask-free RowAcc (raw sums, finalized in k_reduce_tiled).
// MODE 0: y, ψ (, ψ′) fragments + all row terms; 1: Σℓ, Σy² terms only;
// 2: partial y of a feature chunk only. yin (MODE 0/1/2, may alias ybuf): the
// partial y of the earlier feature chunks, added at the start of each chain.
template <int KS, int DENS, int MODE, bool YIN>
__global__ void __launch_bounds__(FUSED_THREADS, 2)
k_tiled_yw(const double* __restrict__ X, uint64_t ldx, uint64_t n_in, int nf, int ncp,
           const double* __restrict__ WpT, const double* __restrict__ mu, double alpha, uint64_t bpw,
           uint64_t n_blocks, double* __restrict__ partials, int accumulate, double* ybuf,
           double* __restrict__ pbuf, double* __restrict__ dbuf, const double* yin, uint64_t nwgx) {
  constexpr int NFP = 4 * KS, XS = 16 * NFP, NU = NFP / 64;  // LDS-DMA instructions per wave per block
  static_assert(NFP % 64 == 0, "8 waves × 8 rows per instruction");
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const int nib = ncp / 16;
  uint64_t wx;
  int role;
  if (!xcd_decode((nib + 7) / 8, nwgx, wx, role)) return;
  const int ib = role * 8 + wave;
  const bool active = ib < nib;
  const int row = ib * 16 + lr;
  const double alpha_ = alpha, inv_alpha = 1.0 / alpha, m2a = -2.0 * alpha;
  extern __shared__ double smem[];
  EXP_TAB_DECL;
  exp_tab_load(s_exp_tab);
  double* xs0 = smem;  // [2][NFP][16]
  double wf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) wf[ks] = active ? WpT[(size_t)(4 * ks + lk) * ncp + row] : 0.0;
  RowAcc racc;
  const uint64_t b_begin = wx * bpw;
  const uint64_t b_end = b_begin + bpw < n_blocks ? b_begin + bpw : n_blocks;
  // X staged by LDS-DMA (the centred resident X: μ = null; samples past n_in are
  // the zero padding of X, rows ≥ nf read row 0 against zero W columns): wave w
  // moves rows [w·NFP/8, (w+1)·NFP/8), 8 rows × 16 samples per instruction
  (void)mu;
  (void)n_in;
  const double* src[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int xr = wave * (NFP / 8) + 8 * u + (lane >> 3);
    src[u] = X + (size_t)(xr < nf ? xr : 0) * ldx + 2 * (lane & 7);
  }
  auto stage = [&](uint64_t b, double* xs) {
#pragma unroll
    for (int u = 0; u < NU; ++u)
      __builtin_amdgcn_global_load_lds((gbl_vptr)(src[u] + b * 16),
                                       (lds_vptr)(xs + (wave * (NFP / 8) + 8 * u) * 16), 16, 0, 0);
  };
  if (b_begin < b_end) {
    stage(b_begin, xs0);
    __syncthreads();
    int cur = 0;
    for (uint64_t b = b_begin; b < b_end; ++b) {
      const size_t f0 = tl_frag(b >> 2, ib, (int)(b & 3), 0, nib) + lane;
      d4 yv = d4{0, 0, 0, 0};
      // partial y of the earlier feature chunks, loaded BEFORE the DMA so the wait
      // for it leaves the DMA in flight (a load issued after it drained both)
      if (YIN && active)
#pragma unroll
        for (int r = 0; r < 4; ++r) yv[r] = yin[f0 + 64 * r];
      if (b + 1 < b_end) stage(b + 1, xs0 + (cur ^ 1) * XS);
      __builtin_amdgcn_sched_barrier(0);  // the DMA stays ahead of this block's stores (dma_barrier)
      if (active) {
        const double* xrow = xs0 + cur * XS + lk * 16 + lr;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) yv = mfma(xrow[(4 * ks) * 16], wf[ks], yv);
        if constexpr (MODE == 0) {
          double psi[4], dpsi[4];
          density_acc4<DENS, true, true, 1>(yv, alpha_, m2a, s_exp_tab, racc, psi, dpsi);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ybuf[f0 + 64 * r] = yv[r];
            pbuf[f0 + 64 * r] = psi[r];
            if (dbuf) dbuf[f0 + 64 * r] = dpsi[r];
          }
        } else if constexpr (MODE == 1) {
          loss_acc4<DENS, true, 1>(yv, alpha_, m2a, s_exp_tab, racc);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) ybuf[f0 + 64 * r] = yv[r];
        }
        if constexpr (MODE != 2)
          if ((b & (RENORM_BLOCKS - 1)) == RENORM_BLOCKS - 1) acc_renorm<DENS>(racc);
      }
      // this wave's LDS-DMA of block b + 1 landed; its y / ψ (/ ψ′) stores may still be in flight
      if (!active || MODE == 1) dma_barrier<0>();
      else if (MODE == 2) dma_barrier<4>();
      else if (dbuf) dma_barrier<12>();
      else dma_barrier<8>();
      cur ^= 1;
    }
  }
  if constexpr (MODE == 2) return;
  // raw row terms → workgroup partials [Σψ′ | Σℓ | Σy²] (ncp each); the roles
  // of a slot write disjoint rows
  const int nfac = b_begin < b_end ? 4 * (int)(b_end - b_begin) : 0;  // one density call per block
  double rs_d = acc_dpsi<DENS>(racc), rs_l = acc_ll<DENS>(racc, inv_alpha, nfac), rs_q = racc.q;
  rs_d += __shfl_xor(rs_d, 16); rs_d += __shfl_xor(rs_d, 32);
  rs_l += __shfl_xor(rs_l, 16); rs_l += __shfl_xor(rs_l, 32);
  rs_q += __shfl_xor(rs_q, 16); rs_q += __shfl_xor(rs_q, 32);
  if (active && lk == 0) {
    double* out = partials + (size_t)wx * 3 * ncp;
    const double v[3] = {MODE == 0 ? rs_d : 0.0, rs_l, rs_q};
#pragma unroll
    for (int c = 0; c < 3; ++c) out[c * ncp + row] = accumulate ? out[c * ncp + row] + v[c] : v[c];
  }
}

// Phase 1 on the int8 digit stage (KSO k-steps of 64 features: nf ≤ 128 → 2, ≤ 256 → 4):
// the same roles, fragment layout, density, row terms and store/barrier schedule as
// k_tiled_yw (MODE 0 / 1, one feature chunk), with wave ib's Y tile formed by
// oz_ystage + oz_combine (ozaki.inc) from the digit image of X and the W digits held in
// VGPRs (7·KSO v4i per lane) — W read once per launch as k_tiled_yw's fragments are. Per
// 16-sample block the 7·KSO planes (1 KiB each) and 16 scales are staged by LDS-DMA,
// item w + 8u of wave w. Y has the accuracy of the fp64 stage (ozaki.inc); the full
// (MODE 0) and loss-only (MODE 1) passes run the same arithmetic, so their Σℓ, Σy² agree.
template <int KSO, int DENS, int MODE>
__global__ void __launch_bounds__(FUSED_THREADS, 2)
k_tiled_yw_oz(const uint8_t* __restrict__ xsl, const double* __restrict__ xsc, const uint8_t* __restrict__ wsl_g,
              const double* __restrict__ wsc, int ncp, double alpha, uint64_t bpw, uint64_t n_blocks,
              double* __restrict__ partials, int accumulate, double* ybuf, double* __restrict__ pbuf,
              double* __restrict__ dbuf, uint64_t nwgx) {
  static_assert(MODE == 0 || MODE == 1, "one feature chunk");
  constexpr int TILE = oz_block_bytes<KSO>(), NITEM = OZ_SLICES * KSO + 1, NU = (NITEM + 7) / 8;
  constexpr int SLOT = TILE + 256;  // bytes per staged block: digit planes, 16 scales
  constexpr int KSW = KSO < 2 ? 2 : KSO;  // k-step stride of the W digit image (DeviceCtx::wsl_ksw)
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const int nib = ncp / 16;
  uint64_t wx;
  int role;
  if (!xcd_decode((nib + 7) / 8, nwgx, wx, role)) return;
  const int ib = role * 8 + wave;
  const bool active = ib < nib;
  const int row = ib * 16 + lr;
  const double alpha_ = alpha, inv_alpha = 1.0 / alpha, m2a = -2.0 * alpha;
  extern __shared__ double smem[];
  EXP_TAB_DECL;
  exp_tab_load(s_exp_tab);
  uint8_t* xs0 = (uint8_t*)smem;  // [2][SLOT]
  v4i wsl[OZ_SLICES][KSO];
#pragma unroll
  for (int a = 0; a < OZ_SLICES; ++a)
#pragma unroll
    for (int k = 0; k < KSO; ++k)
      wsl[a][k] = active ? *(const v4i*)(wsl_g + (size_t)(((ib * OZ_SLICES + a) * KSW + k) * 64 + lane) * 16)
                         : v4i{0, 0, 0, 0};
  const double rsc = active ? wsc[row] : 0.0;
  RowAcc racc;
  const uint64_t b_begin = wx * bpw;
  const uint64_t b_end = b_begin + bpw < n_blocks ? b_begin + bpw : n_blocks;
  auto stage = [&](uint64_t b, uint8_t* xs) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int it = wave + 8 * u;
      if (it < NITEM - 1)
        __builtin_amdgcn_global_load_lds((gbl_vptr)(xsl + b * TILE + it * 1024 + lane * 16),
                                         (lds_vptr)(xs + it * 1024), 16, 0, 0);
      else if (it == NITEM - 1)
        __builtin_amdgcn_global_load_lds((gbl_vptr)((const uint32_t*)(xsc + b * 16) + (lane & 31)),
                                         (lds_vptr)(xs + TILE), 4, 0, 0);
    }
  };
  if (b_begin < b_end) {
    stage(b_begin, xs0);
    __syncthreads();
    int cur = 0;
    for (uint64_t b = b_begin; b < b_end; ++b) {
      const size_t f0 = tl_frag(b >> 2, ib, (int)(b & 3), 0, nib) + lane;
      if (b + 1 < b_end) stage(b + 1, xs0 + (cur ^ 1) * SLOT);
      __builtin_amdgcn_sched_barrier(0);  // the DMA stays ahead of this block's stores (dma_barrier)
      if (active) {
        const uint8_t* tile = xs0 + cur * SLOT;
        v4i acc[OZ_SLICES];
        oz_ystage<OZ_SLICES - 1, KSO>(tile, lane, wsl, acc);
        const double* scd = (const double*)(tile + TILE);
        const double x4[4] = {scd[lk], scd[lk + 4], scd[lk + 8], scd[lk + 12]};
        const d4 yv = oz_combine(acc, rsc, x4);
        if constexpr (MODE == 0) {
          double psi[4], dpsi[4];
          density_acc4<DENS, true, true, 1>(yv, alpha_, m2a, s_exp_tab, racc, psi, dpsi);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ybuf[f0 + 64 * r] = yv[r];
            pbuf[f0 + 64 * r] = psi[r];
            if (dbuf) dbuf[f0 + 64 * r] = dpsi[r];
          }
        } else {
          loss_acc4<DENS, true, 1>(yv, alpha_, m2a, s_exp_tab, racc);
        }
        if ((b & (RENORM_BLOCKS - 1)) == RENORM_BLOCKS - 1) acc_renorm<DENS>(racc);
      }
      // this wave's LDS-DMA of block b + 1 landed; its y / ψ (/ ψ′) stores may still be in flight
      if (!active || MODE == 1) dma_barrier<0>();
      else if (dbuf) dma_barrier<12>();
      else dma_barrier<8>();
      cur ^= 1;
    }
  }
  const int nfac = b_begin < b_end ? 4 * (int)(b_end - b_begin) : 0;  // one density call per block
  double rs_d = acc_dpsi<DENS>(racc), rs_l = acc_ll<DENS>(racc, inv_alpha, nfac), rs_q = racc.q;
  rs_d += __shfl_xor(rs_d, 16); rs_d += __shfl_xor(rs_d, 32);
  rs_l += __shfl_xor(rs_l, 16); rs_l += __shfl_xor(rs_l, 32);
  rs_q += __shfl_xor(rs_q, 16); rs_q += __shfl_xor(rs_q, 32);
  if (active && lk == 0) {
    double* out = partials + (size_t)wx * 3 * ncp;
    const double v[3] = {MODE == 0 ? rs_d : 0.0, rs_l, rs_q};
#pragma unroll
    for (int c = 0; c < 3; ++c) out[c * ncp + row] = accumulate ? out[c * ncp + row] + v[c] : v[c];
  }
}

// Phase 2 staged through LDS: blockIdx.x = 128×128 output tile (ti, tj),
// blockIdx.y = T split. Per 16-sample sub-block the workgroup copies the ψ
// (and ψ′) fragments of its 8 row blocks ti and the y fragments of row blocks
// tj (16 KB each, contiguous 2 KB runs) into LDS once — every fragment feeds 2
// or 4 waves — with the next sub-block prefetched into registers a full
// iteration ahead; one barrier per sub-block. Wave (gi, gj) accumulates a 64×32
// patch of G (and H) in registers.
// DFROMP (tanh, α > 0): ψ′ = α(1 − ψ²) is formed here from the staged ψ — the
// expression density_acc4 evaluates, so the same bits — instead of being
// written by phase 1 and read back (one array less each way).
template <bool NEED_H, bool DFROMP, int SBB = 2>
__global__ void __launch_bounds__(FUSED_THREADS, 1)
k_tiled_gram2(const double* __restrict__ ybuf, const double* __restrict__ pbuf, const double* __restrict__ dbuf,
              int ncp, uint64_t n_tiles, uint64_t tps, double* __restrict__ slabs, int accumulate, double alpha,
              uint64_t nsplit) {
  static_assert(NEED_H || !DFROMP, "ψ′ only feeds H");
  static_assert(SBB == 1 || SBB == 2 || SBB == 4, "sub-blocks per stage divide a 64-sample tile");
  constexpr int NARR = NEED_H && !DFROMP ? 3 : 2;  // staged arrays: ψ, y (, ψ′)
  constexpr int SUB = 8 * 256;          // doubles per array per sub-block (8 row blocks × 4 r × 64)
  constexpr int PRE = NARR * SUB / 2 / FUSED_THREADS;  // 2 slots per array
  constexpr int STG = SBB * NARR * SUB;  // doubles per stage (SBB sub-blocks, one barrier)
  static_assert(SUB == 4 * FUSED_THREADS, "slot map assumes 512 threads");
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const int nib = ncp / 16;
  const int nto = (nib + 7) / 8;
  uint64_t split;
  int tile;  // the nto² output tiles of one T split share an XCD: ψ / y fragments come from its L2
  if (!xcd_decode(nto * nto, nsplit, split, tile)) return;
  const int ti = tile / nto, tj = tile % nto;
  const int gi0 = (wave >> 2) * 4, gj0 = (wave & 3) * 2;  // local row blocks
  extern __shared__ double smem[];
  double* lds = smem;  // [2][SBB][NARR][8][4][64]
  d4 accg[4][2], acch[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) { accg[i][j] = d4{0, 0, 0, 0}; acch[i][j] = d4{0, 0, 0, 0}; }
  // staging slots: slot p of thread tid is double e = 2·tid + 1024·p of the
  // [NARR][8][256] sub-block image, i.e. array p/2 (ψ, y, ψ′), local row block
  // tid/128 + 4·(p&1), offset 2·tid mod 256 — all slots share one in-array offset
  const int lb0 = tid >> 7, off = (2 * tid) & 255;
  int soff[PRE];
  bool ok[PRE];
#pragma unroll
  for (int p = 0; p < PRE; ++p) {
    const int gb = ((p >> 1) == 1 ? tj : ti) * 8 + lb0 + 4 * (p & 1);  // y uses the tj row blocks
    ok[p] = gb < nib;
    soff[p] = (ok[p] ? gb : 0) * 1024 + off;  // + ((tt·nib)·4 + ts)·256 per sub-block
  }
  const uint64_t t_begin = split * tps;
  const uint64_t t_end = t_begin + tps < n_tiles ? t_begin + tps : n_tiles;
  const uint64_t s_begin = t_begin * 4, s_end = t_end * 4;  // sub-blocks (a multiple of SBB apart)
  double2 pre[SBB][PRE];
  auto load = [&](uint64_t sb0) {
#pragma unroll
    for (int q = 0; q < SBB; ++q) {
      const uint64_t sb = sb0 + q;
      const size_t o = ((sb >> 2) * (size_t)nib * 4 + (sb & 3)) * 256;
#pragma unroll
      for (int p = 0; p < PRE; ++p) {
        const double* base = (p >> 1) == 0 ? pbuf : (p >> 1) == 1 ? ybuf : dbuf;
        pre[q][p] = ok[p] ? *reinterpret_cast<const double2*>(base + o + soff[p]) : double2{0.0, 0.0};
      }
    }
  };
  auto store = [&](double* img) {
#pragma unroll
    for (int q = 0; q < SBB; ++q)
#pragma unroll
      for (int p = 0; p < PRE; ++p) *reinterpret_cast<double2*>(img + q * NARR * SUB + 2 * tid + 1024 * p) = pre[q][p];
  };
  if (s_begin < s_end) {
    load(s_begin);
    store(lds);
    __syncthreads();
    int cur = 0;
    for (uint64_t sb = s_begin; sb < s_end; sb += SBB) {
      load(sb + SBB < s_end ? sb + SBB : sb);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < SBB; ++q) {
        const double* img = lds + cur * STG + q * NARR * SUB;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          double pa[4], da[4], yb[2];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            pa[i] = img[((gi0 + i) * 4 + r) * 64 + lane];
            if constexpr (DFROMP) da[i] = alpha * __builtin_fma(-pa[i], pa[i], 1.0);
            else if constexpr (NEED_H) da[i] = img[2 * SUB + ((gi0 + i) * 4 + r) * 64 + lane];
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) yb[j] = img[SUB + ((gj0 + j) * 4 + r) * 64 + lane];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              accg[i][j] = mfma(pa[i], yb[j], accg[i][j]);
              if constexpr (NEED_H) acch[i][j] = mfma(da[i], yb[j] * yb[j], acch[i][j]);
            }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      store(lds + (cur ^ 1) * STG);
      __syncthreads();
      cur ^= 1;
    }
  }
  const size_t nsq = (size_t)ncp * ncp;
  double* slab = slabs + (size_t)split * (NEED_H ? 2 : 1) * nsq;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int bi = ti * 8 + gi0 + i, bj = tj * 8 + gj0 + j;
      if (bi < nib && bj < nib)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = bi * 16 + lk + 4 * r, col = bj * 16 + lr;
          const size_t o = (size_t)row * ncp + col;
          slab[o] = accumulate ? slab[o] + accg[i][j][r] : accg[i][j][r];
          if constexpr (NEED_H) slab[nsq + o] = accumulate ? slab[nsq + o] + acch[i][j][r] : acch[i][j][r];
        }
    }
}

// ---------------------------------------------------------------------------
// Non-orthogonal line search in ONE pass (core.rs:117-140 with M = I + αD):
// Y_α = (W + α·DW)·(X−μ) = Y + α·Z, so Y = W·(X−μ) and Z = (DW)·(X−μ) are
// computed once (two MFMA GEMMs) and Σℓ(Y_α), Σ(Y_α)² are accumulated for
// every remaining try α_j (VALU only). The host then walks the tries in the
// reference's order and stops at the first accepted α exactly as
// line_search does; only the accepted try is then evaluated in full.
// ---------------------------------------------------------------------------
constexpr int ML_NA = 12;   // tries per pass (ls_tries − 1 ≤ 12; more are chunked)
constexpr int ML_KC = 16;   // K chunk (two W images in LDS)
constexpr int ML_TS = 2, ML_TT = 16 * ML_TS;  // samples per tile (Y and Z accumulators in VGPRs)

template <int DENS>
__global__ void __launch_bounds__(FUSED_THREADS, 1)
k_multi_loss(const double* __restrict__ X, uint64_t ldx, uint64_t n_local, int nf, int nfp, int ncp,
             const double* __restrict__ WpT, const double* __restrict__ ZpT, const double* __restrict__ mu,
             double alpha, const double* __restrict__ alphas, int na, uint64_t tpw, uint64_t n_tiles,
             double* __restrict__ partials) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const int npair = ncp / 32;
  const bool active = wave < npair;
  const double inv_alpha = 1.0 / alpha;
  constexpr int WSTR = 256 + 16, XSTR = ML_TT + 16;
  extern __shared__ double smem[];
  double* ws = smem;                  // [ML_KC][WSTR]
  double* zs = ws + ML_KC * WSTR;     // [ML_KC][WSTR]
  double* xs = zs + ML_KC * WSTR;     // [ML_KC][XSTR]
  // per-try row sums live in LDS, one region per wave: rs[wave][j][i][lr][Σℓ, Σy²]
  double* rs = xs + ML_KC * XSTR + (size_t)wave * ML_NA * 2 * 16 * 2;
  for (int e = lane; e < ML_NA * 2 * 16 * 2; e += 64) rs[e] = 0.0;
  const uint64_t t_begin = (uint64_t)blockIdx.x * tpw;
  const uint64_t t_end = t_begin + tpw < n_tiles ? t_begin + tpw : n_tiles;
  for (uint64_t tt = t_begin; tt < t_end; ++tt) {
    d4 ay[2][ML_TS], az[2][ML_TS];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int t = 0; t < ML_TS; ++t) { ay[i][t] = d4{0, 0, 0, 0}; az[i][t] = d4{0, 0, 0, 0}; }
    for (int k0 = 0; k0 < nfp; k0 += ML_KC) {
      __syncthreads();
      for (int e = tid; e < ncp * ML_KC; e += FUSED_THREADS) {
        const int k = e / ncp, row = e % ncp;
        ws[k * WSTR + row] = WpT[(size_t)(k0 + k) * ncp + row];
        zs[k * WSTR + row] = ZpT[(size_t)(k0 + k) * ncp + row];
      }
      for (int e = tid; e < ML_KC * ML_TT / 2; e += FUSED_THREADS) {
        const int k = e / (ML_TT / 2), t = 2 * (e % (ML_TT / 2));
        const int kg = k0 + k;
        const uint64_t tg = tt * ML_TT + t;
        double2 v = double2{0.0, 0.0};
        if (kg < nf) {
          const double2 xv = *reinterpret_cast<const double2*>(X + (size_t)kg * ldx + tg);
          const double m = mu ? mu[kg] : 0.0;
          v.x = tg < n_local ? xv.x - m : 0.0;
          v.y = tg + 1 < n_local ? xv.y - m : 0.0;
        }
        *reinterpret_cast<double2*>(xs + k * XSTR + t) = v;
      }
      __syncthreads();
      if (active) {
#pragma unroll
        for (int kq = 0; kq < ML_KC / 4; ++kq) {
          double a[ML_TS], bw[2], bz[2];
#pragma unroll
          for (int t = 0; t < ML_TS; ++t) a[t] = xs[(kq * 4 + lk) * XSTR + t * 16 + lr];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            bw[i] = ws[(kq * 4 + lk) * WSTR + (wave * 2 + i) * 16 + lr];
            bz[i] = zs[(kq * 4 + lk) * WSTR + (wave * 2 + i) * 16 + lr];
          }
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int t = 0; t < ML_TS; ++t) {
              ay[i][t] = mfma(a[t], bw[i], ay[i][t]);
              az[i][t] = mfma(a[t], bz[i], az[i][t]);
            }
        }
      }
    }
    if (active) {
#pragma unroll 1
      for (int j = 0; j < na; ++j) {
        const double aj = alphas[j];  // uniform: scalar load
        double sl[2] = {0.0, 0.0}, sq[2] = {0.0, 0.0};
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int t = 0; t < ML_TS; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const bool valid = tt * ML_TT + t * 16 + 4 * r + lk < n_local;
              const double y = __builtin_fma(aj, az[i][t][r], ay[i][t][r]);
              sl[i] += valid ? density_loss<DENS>(y, alpha, inv_alpha) : 0.0;
              sq[i] = __builtin_fma(y, y, sq[i]);
              if (r == 3) __builtin_amdgcn_sched_barrier(0);  // 4 density chains live at a time
            }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          double l = sl[i], q = sq[i];
          l += __shfl_xor(l, 16); l += __shfl_xor(l, 32);
          q += __shfl_xor(q, 16); q += __shfl_xor(q, 32);
          if (lk == 0) {
            double* p = rs + ((j * 2 + i) * 16 + lr) * 2;
            p[0] += l;
            p[1] += q;
          }
        }
      }
    }
  }
  // partials: [na][2][ncp] (Σℓ, Σy² per try)
  double* out = partials + (size_t)blockIdx.x * ML_NA * 2 * ncp;
  if (active && lk == 0)
    for (int j = 0; j < na; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = (wave * 2 + i) * 16 + lr;
        const double* p = rs + ((j * 2 + i) * 16 + lr) * 2;
        out[(j * 2 + 0) * ncp + row] = p[0];
        out[(j * 2 + 1) * ncp + row] = p[1];
      }
}


// Multi-try loss pass with W and Z = D·W in registers (nf ≤ 256). A workgroup
// covers 64 rows (blockIdx.y = role: row blocks 4·role … 4·role+3); wave w owns
// row block w&3 and the K-half w>>2, holding the matching halves of its W and Z
// fragments (2 × NFP/8 doubles per lane), so neither matrix is re-read per tile
// (k_multi_loss re-staged both from L2 for every 32-sample tile). Per 16-sample
// block: partial Yᵀ and Zᵀ tiles from two single MFMA chains over the K-half,
// exchanged through LDS (double-buffered, one barrier per block) and summed in
// K order; then each wave of the pair evaluates every other try α_j on
// y = Y + α_j·Z with the mask-free RowAcc terms (finalized in k_reduce_rows).
constexpr int ML2_TRIES = (ML_NA + 1) / 2;  // tries per wave
template <int KS, int DENS, bool NEED_Q>
__global__ void __launch_bounds__(FUSED_THREADS, 2)
k_multi_loss2(const double* __restrict__ X, uint64_t ldx, uint64_t n_local, int nf, int ncp,
              const double* __restrict__ WpT, const double* __restrict__ ZpT, const double* __restrict__ mu,
              double alpha, const double* __restrict__ alphas, int na, uint64_t bpw, uint64_t n_blocks,
              double* __restrict__ partials, uint64_t nwgx) {
  constexpr int NFP = 4 * KS, KH = KS / 2, XS = 16 * NFP, NU = NFP / 64;  // LDS-DMA instructions per wave
  static_assert(NFP % 64 == 0, "8 waves × 8 rows per instruction");
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const int nib = ncp / 16;
  const int rb = wave & 3, kh = wave >> 2;
  uint64_t wx;
  int role;
  if (!xcd_decode((nib + 3) / 4, nwgx, wx, role)) return;
  const int ib = role * 4 + rb;
  const bool active = ib < nib;
  const int row = ib * 16 + lr;
  const double inv_alpha = 1.0 / alpha, m2a = -2.0 * alpha;
  extern __shared__ double smem[];
  EXP_TAB_DECL;
  exp_tab_load(s_exp_tab);
  double* xs0 = smem;             // [2][NFP][16]
  double* ex0 = smem + 2 * XS;    // [2][2 K-halves][4 row blocks][Y, Z][4][64]
  double wf[KH], zf[KH];
#pragma unroll
  for (int q = 0; q < KH; ++q) {
    const size_t o = (size_t)(4 * (kh * KH + q) + lk) * ncp + row;
    wf[q] = active ? WpT[o] : 0.0;
    zf[q] = active ? ZpT[o] : 0.0;
  }
  // this wave's tries: j = kh, kh + 2, … < na
  double aj[ML2_TRIES];
  RowAcc racc[ML2_TRIES];
#pragma unroll
  for (int u = 0; u < ML2_TRIES; ++u) aj[u] = (kh + 2 * u < na) ? alphas[kh + 2 * u] : 0.0;
  const int my_na = na > kh ? (na - kh + 1) / 2 : 0;
  const uint64_t b_begin = wx * bpw;
  const uint64_t b_end = b_begin + bpw < n_blocks ? b_begin + bpw : n_blocks;
  const uint64_t b_last = b_end - 1;
  // X staged by LDS-DMA as in k_tiled_yw (centred resident X, μ = null)
  (void)mu;
  const double* src[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int xr = wave * (NFP / 8) + 8 * u + (lane >> 3);
    src[u] = X + (size_t)(xr < nf ? xr : 0) * ldx + 2 * (lane & 7);
  }
  auto stage = [&](uint64_t b, double* xs) {
#pragma unroll
    for (int u = 0; u < NU; ++u)
      __builtin_amdgcn_global_load_lds((gbl_vptr)(src[u] + b * 16),
                                       (lds_vptr)(xs + (wave * (NFP / 8) + 8 * u) * 16), 16, 0, 0);
  };
  auto exch = [&](int buf, int half, int yz, int r) -> double* {
    return ex0 + ((((buf * 2 + half) * 4 + rb) * 2 + yz) * 4 + r) * 64 + lane;
  };
  if (b_begin < b_end) {
    stage(b_begin, xs0);
    __syncthreads();
    int cur = 0;
    for (uint64_t b = b_begin; b < b_end; ++b) {
      if (b + 1 < b_end) stage(b + 1, xs0 + (cur ^ 1) * XS);
      if (active) {  // partial Yᵀ, Zᵀ over this wave's K-half
        d4 ya = d4{0, 0, 0, 0}, za = d4{0, 0, 0, 0};
        const double* xrow = xs0 + cur * XS + (4 * kh * KH + lk) * 16 + lr;
#pragma unroll
        for (int q = 0; q < KH; ++q) {
          const double xa = xrow[(4 * q) * 16];
          ya = mfma(xa, wf[q], ya);
          za = mfma(xa, zf[q], za);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          *exch(cur, kh, 0, r) = ya[r];
          *exch(cur, kh, 1, r) = za[r];
        }
      }
      __syncthreads();  // exchange visible; this wave's LDS-DMA of block b + 1 landed
      if (active) {  // Y, Z summed in K order (identical in both waves of the pair), then the tries
        d4 yv, zv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          yv[r] = *exch(cur, 0, 0, r) + *exch(cur, 1, 0, r);
          zv[r] = *exch(cur, 0, 1, r) + *exch(cur, 1, 1, r);
        }
#pragma unroll
        for (int u = 0; u < ML2_TRIES; ++u) {
          if (u < my_na) {
            d4 yj;
#pragma unroll
            for (int r = 0; r < 4; ++r) yj[r] = __builtin_fma(aj[u], zv[r], yv[r]);
            loss_acc4<DENS, NEED_Q, 1>(yj, alpha, m2a, s_exp_tab, racc[u]);
            if ((b & (RENORM_BLOCKS - 1)) == RENORM_BLOCKS - 1) acc_renorm<DENS>(racc[u]);
          }
        }
      }
      cur ^= 1;
    }
  }
  // partials: [ML_NA][2][ncp] raw (Σℓ term, Σy²) per try
  double* out = partials + (size_t)wx * ML_NA * 2 * ncp;
#pragma unroll
  for (int u = 0; u < ML2_TRIES; ++u) {
    if (u < my_na) {
      double l = acc_ll<DENS>(racc[u], inv_alpha, b_begin < b_end ? 4 * (int)(b_end - b_begin) : 0), q = racc[u].q;
      l += __shfl_xor(l, 16); l += __shfl_xor(l, 32);
      q += __shfl_xor(q, 16); q += __shfl_xor(q, 32);
      if (active && lk == 0) {
        const int j = kh + 2 * u;
        out[(j * 2 + 0) * ncp + row] = l;
        out[(j * 2 + 1) * ncp + row] = q;
      }
    }
  }
}

// k_multi_loss2 on the int8 digit stage (nf ≤ 256, KSO k-steps): wave w forms the full-K Yᵀ
// (w < 4) or Zᵀ (w ≥ 4) tile of row block 4·role + (w & 3) from the digit image of X and the
// W / Z digits held in VGPRs (image row blocks 0–15: W, 16–31: Z = D·W), the two tiles meet in
// LDS, and the pair evaluates the tries on y = Y + α_j·Z exactly as k_multi_loss2 does (wave
// w takes the tries j ≡ w >> 2 mod 2). Y and Z carry fp64-GEMM accuracy (ozaki.inc); like the
// fp64 form, Y_α = Y + α·Z agrees with a per-try pass to rounding.
// F32 (tanh, no Σy²): the tries' row terms in fp32 — y_j = fl32(fl32(Y) + α_j·fl32(Z)) and
// loss_acc4_f32y as in the orthogonal screen — returning per try [Σℓ raw | Σ|y_j|] and per
// row Σ|Y|, Σ|Z| (after the ML_NA tries' slots), from which DeviceCtx::eval_loss_multi_bound
// bounds each try's distance to the exact pass at W + α_j·Z.
template <int KSO, int DENS, bool NEED_Q, bool F32 = false>
__global__ void __launch_bounds__(FUSED_THREADS, 2)
k_multi_loss2_oz(const uint8_t* __restrict__ xsl, const double* __restrict__ xsc, const uint8_t* __restrict__ wsl_g,
                 const double* __restrict__ wsc, int ncp, double alpha, const double* __restrict__ alphas, int na,
                 uint64_t bpw, uint64_t n_blocks, double* __restrict__ partials, uint64_t nwgx) {
  static_assert(!F32 || (DENS == DENS_TANH && !NEED_Q), "fp32 tries: tanh without Σy²");
  constexpr int TILE = oz_block_bytes<KSO>(), NITEM = OZ_SLICES * KSO + 1, NU = (NITEM + 7) / 8;
  constexpr int SLOT = TILE + 256, KSW = KSO < 2 ? 2 : KSO;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const int nib = ncp / 16;
  const int rb = wave & 3, yz = wave >> 2;
  uint64_t wx;
  int role;
  if (!xcd_decode((nib + 3) / 4, nwgx, wx, role)) return;
  const int ib = role * 4 + rb;
  const bool active = ib < nib;
  const int row = ib * 16 + lr;
  const double inv_alpha = 1.0 / alpha, m2a = -2.0 * alpha;
  extern __shared__ double smem[];
  EXP_TAB_DECL;
  exp_tab_load(s_exp_tab);
  uint8_t* xs0 = (uint8_t*)smem;                          // [2][SLOT]
  double* ex0 = (double*)(xs0 + 2 * SLOT);                // [2][4 row blocks][Y, Z][4][64]
  v4i wsl[OZ_SLICES][KSO];
  const int wb = yz * 16 + ib;  // image row block: W (yz = 0) or Z (1)
#pragma unroll
  for (int a = 0; a < OZ_SLICES; ++a)
#pragma unroll
    for (int k = 0; k < KSO; ++k)
      wsl[a][k] = active ? *(const v4i*)(wsl_g + (size_t)(((wb * OZ_SLICES + a) * KSW + k) * 64 + lane) * 16)
                         : v4i{0, 0, 0, 0};
  const double rsc = active ? wsc[yz * 256 + row] : 0.0;
  double aj[ML2_TRIES];
  RowAcc racc[ML2_TRIES];
  double sabs = 0.0;  // F32: Σ|Y| (yz = 0) or Σ|Z| (yz = 1) of this lane's samples
  const float c32 = (float)(m2a * fm::LOG2E);
#pragma unroll
  for (int u = 0; u < ML2_TRIES; ++u) aj[u] = (yz + 2 * u < na) ? alphas[yz + 2 * u] : 0.0;
  const int my_na = na > yz ? (na - yz + 1) / 2 : 0;
  const uint64_t b_begin = wx * bpw;
  const uint64_t b_end = b_begin + bpw < n_blocks ? b_begin + bpw : n_blocks;
  auto stage = [&](uint64_t b, uint8_t* xs) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int it = wave + 8 * u;
      if (it < NITEM - 1)
        __builtin_amdgcn_global_load_lds((gbl_vptr)(xsl + b * TILE + it * 1024 + lane * 16),
                                         (lds_vptr)(xs + it * 1024), 16, 0, 0);
      else if (it == NITEM - 1)
        __builtin_amdgcn_global_load_lds((gbl_vptr)((const uint32_t*)(xsc + b * 16) + (lane & 31)),
                                         (lds_vptr)(xs + TILE), 4, 0, 0);
    }
  };
  auto exch = [&](int buf, int w_yz, int r) -> double* {
    return ex0 + (((buf * 4 + rb) * 2 + w_yz) * 4 + r) * 64 + lane;
  };
  if (b_begin < b_end) {
    stage(b_begin, xs0);
    __syncthreads();
    int cur = 0;
    for (uint64_t b = b_begin; b < b_end; ++b) {
      if (b + 1 < b_end) stage(b + 1, xs0 + (cur ^ 1) * SLOT);
      if (active) {
        const uint8_t* tile = xs0 + cur * SLOT;
        v4i acc[OZ_SLICES];
        oz_ystage<OZ_SLICES - 1, KSO>(tile, lane, wsl, acc);
        const double* scd = (const double*)(tile + TILE);
        const double x4[4] = {scd[lk], scd[lk + 4], scd[lk + 8], scd[lk + 12]};
        const d4 v = oz_combine(acc, rsc, x4);
#pragma unroll
        for (int r = 0; r < 4; ++r) *exch(cur, yz, r) = v[r];
        if constexpr (F32)
#pragma unroll
          for (int r = 0; r < 4; ++r) sabs += fabs(v[r]);
      }
      __syncthreads();  // exchange visible; this wave's LDS-DMA of block b + 1 landed
      if (active) {
        d4 yv, zv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          yv[r] = *exch(cur, 0, r);
          zv[r] = *exch(cur, 1, r);
        }
        if constexpr (F32) {
          const f4 y32 = {(float)yv[0], (float)yv[1], (float)yv[2], (float)yv[3]};
          const f4 z32 = {(float)zv[0], (float)zv[1], (float)zv[2], (float)zv[3]};
#pragma unroll
          for (int u = 0; u < ML2_TRIES; ++u) {
            if (u < my_na) {
              const float a32 = (float)aj[u];  // α_j = 2^-k: exact
              f4 yj;
#pragma unroll
              for (int r = 0; r < 4; ++r) yj[r] = __builtin_fabsf(__builtin_fmaf(a32, z32[r], y32[r]));
              loss_acc4_f32y(yj, c32, racc[u]);
            }
          }
        } else {
#pragma unroll
          for (int u = 0; u < ML2_TRIES; ++u) {
            if (u < my_na) {
              d4 yj;
#pragma unroll
              for (int r = 0; r < 4; ++r) yj[r] = __builtin_fma(aj[u], zv[r], yv[r]);
              loss_acc4<DENS, NEED_Q, 1>(yj, alpha, m2a, s_exp_tab, racc[u]);
              if ((b & (RENORM_BLOCKS - 1)) == RENORM_BLOCKS - 1) acc_renorm<DENS>(racc[u]);
            }
          }
        }
      }
      cur ^= 1;
    }
  }
  double* out = partials + (size_t)wx * (ML_NA * 2 + (F32 ? 2 : 0)) * ncp;
#pragma unroll
  for (int u = 0; u < ML2_TRIES; ++u) {
    if (u < my_na) {
      double l, q;
      if constexpr (F32) {  // raw Σℓ = Σ|y| + (ln2/α)·Σ log2 Π((1 + 2^z)/2); Σ|y_j|
        l = __builtin_fma(racc[u].g, fm::LN2 * inv_alpha, racc[u].l);
        q = racc[u].l;
      } else {
        l = acc_ll<DENS>(racc[u], inv_alpha, b_begin < b_end ? 4 * (int)(b_end - b_begin) : 0);
        q = racc[u].q;
      }
      l += __shfl_xor(l, 16); l += __shfl_xor(l, 32);
      q += __shfl_xor(q, 16); q += __shfl_xor(q, 32);
      if (active && lk == 0) {
        const int j = yz + 2 * u;
        out[(j * 2 + 0) * ncp + row] = l;
        out[(j * 2 + 1) * ncp + row] = q;
      }
    }
  }
  if constexpr (F32) {
    sabs += __shfl_xor(sabs, 16); sabs += __shfl_xor(sabs, 32);
    if (active && lk == 0) out[(ML_NA * 2 + yz) * ncp + row] = sabs;
  }
}

// k_multi_loss2_oz with Y read back instead of formed: the tiled full pass at the same W
// (k_tiled_yw_oz MODE 0, one T chunk) left Y in HBM in fragment order, from the same digit
// products, scales and combine, so the same bits (core.rs:124 keeps Y between passes too). Each
// wave forms only the Zᵀ tile of its row block 8·role + w (image row blocks 16–31) and evaluates
// every try on y = Y + α_j·Z: half the matrix work per try of k_multi_loss2_oz, no exchange. The
// host passes k_multi_loss2_oz's sample partition (nwgx, bpw), and each lane sums its samples
// in that kernel's order, so the per-workgroup partials — and every decision — are bit for bit
// the same. NT = the tries' accumulators held (10: ls_tries = 10 fits without spilling at KSO = 4).
template <int KSO, int DENS, bool NEED_Q, int NT, bool FENCE = true>
__global__ void __launch_bounds__(FUSED_THREADS, 1)
k_multi_loss2_ozy(const uint8_t* __restrict__ xsl, const double* __restrict__ xsc, const uint8_t* __restrict__ wsl_g,
                  const double* __restrict__ wsc, int ncp, double alpha, const double* __restrict__ alphas, int na,
                  const double* __restrict__ ybuf, uint64_t bpw, uint64_t n_blocks, double* __restrict__ partials,
                  uint64_t nwgx) {
  constexpr int TILE = oz_block_bytes<KSO>(), NITEM = OZ_SLICES * KSO + 1, NU = (NITEM + 7) / 8;
  constexpr int SLOT = TILE + 256, KSW = KSO < 2 ? 2 : KSO;
  static_assert(NT <= ML_NA, "tries per pass");
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const int nib = ncp / 16;
  uint64_t wx;
  int role;
  if (!xcd_decode((nib + 7) / 8, nwgx, wx, role)) return;
  const int ib = role * 8 + wave;
  const bool active = ib < nib;
  const int row = ib * 16 + lr;
  const double inv_alpha = 1.0 / alpha, m2a = -2.0 * alpha;
  extern __shared__ double smem[];
  EXP_TAB_DECL;
  exp_tab_load(s_exp_tab);
  uint8_t* xs0 = (uint8_t*)smem;  // [2][SLOT]
  v4i wsl[OZ_SLICES][KSO];
#pragma unroll
  for (int a = 0; a < OZ_SLICES; ++a)
#pragma unroll
    for (int k = 0; k < KSO; ++k)
      wsl[a][k] = active ? *(const v4i*)(wsl_g + (size_t)((((16 + ib) * OZ_SLICES + a) * KSW + k) * 64 + lane) * 16)
                         : v4i{0, 0, 0, 0};
  const double rsc = active ? wsc[256 + row] : 0.0;
  RowAcc racc[NT];
  const uint64_t b_begin = wx * bpw;
  const uint64_t b_end = b_begin + bpw < n_blocks ? b_begin + bpw : n_blocks;
  auto stage = [&](uint64_t b, uint8_t* xs) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int it = wave + 8 * u;
      if (it < NITEM - 1)
        __builtin_amdgcn_global_load_lds((gbl_vptr)(xsl + b * TILE + it * 1024 + lane * 16),
                                         (lds_vptr)(xs + it * 1024), 16, 0, 0);
      else if (it == NITEM - 1)
        __builtin_amdgcn_global_load_lds((gbl_vptr)((const uint32_t*)(xsc + b * 16) + (lane & 31)),
                                         (lds_vptr)(xs + TILE), 4, 0, 0);
    }
  };
  auto yload = [&](uint64_t b) {
    d4 v;
    const size_t f0 = tl_frag(b >> 2, ib, (int)(b & 3), 0, nib) + lane;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = ybuf[f0 + 64 * r];
    return v;
  };
  if (b_begin < b_end) {
    stage(b_begin, xs0);
    __syncthreads();
    int cur = 0;
    for (uint64_t b = b_begin; b < b_end; ++b) {
      // Y before the DMA, so that waiting for Y leaves the DMA in flight (in-order counter)
      const d4 yv = active ? yload(b) : d4{0, 0, 0, 0};
      if (b + 1 < b_end) stage(b + 1, xs0 + (cur ^ 1) * SLOT);
      __builtin_amdgcn_sched_barrier(0);
      if (active) {
        const uint8_t* tile = xs0 + cur * SLOT;
        v4i acc[OZ_SLICES];
        oz_ystage<OZ_SLICES - 1, KSO>(tile, lane, wsl, acc);
        const double* scd = (const double*)(tile + TILE);
        const double x4[4] = {scd[lk], scd[lk + 4], scd[lk + 8], scd[lk + 12]};
        const d4 zv = oz_combine(acc, rsc, x4);
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          if (u < na) {
            const double aj = alphas[u];
            d4 yj;
#pragma unroll
            for (int r = 0; r < 4; ++r) yj[r] = __builtin_fma(aj, zv[r], yv[r]);
            // FENCE = false: the tries' density chains may interleave (each try's sums keep their
            // element order, so the same bits)
            loss_acc4<DENS, NEED_Q, 1, FENCE>(yj, alpha, m2a, s_exp_tab, racc[u]);
            if ((b & (RENORM_BLOCKS - 1)) == RENORM_BLOCKS - 1) acc_renorm<DENS>(racc[u]);
          }
        }
      }
      dma_barrier<0>();  // this wave's LDS-DMA of block b + 1 landed
      cur ^= 1;
    }
  }
  double* out = partials + (size_t)wx * ML_NA * 2 * ncp;
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    if (u < na) {
      double l = acc_ll<DENS>(racc[u], inv_alpha, b_begin < b_end ? 4 * (int)(b_end - b_begin) : 0), q = racc[u].q;
      l += __shfl_xor(l, 16); l += __shfl_xor(l, 32);
      q += __shfl_xor(q, 16); q += __shfl_xor(q, 32);
      if (active && lk == 0) {
        out[(u * 2 + 0) * ncp + row] = l;
        out[(u * 2 + 1) * ncp + row] = q;
      }
    }
  }
}

// stats[e] for the tiled path: G/H from slabs (sum over splits), rows from phase-1 partials.
// Row terms from k_tiled_yw are raw (finalize_row with dens ≥ 0); k_tiled_y's are final (dens < 0).
__global__ void k_reduce_tiled(const double* __restrict__ slabs, int nsplit, const double* __restrict__ rows,
                               int nwg1, int ncp, int nc, bool need_h, int rows_only, double* __restrict__ stats,
                               int dens, double alpha, double n) {
  const size_t nsq = (size_t)nc * nc, psq = (size_t)ncp * ncp;
  const size_t mats = rows_only ? 0 : (need_h ? 2 : 1) * nsq;
  const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t base_rows = (need_h ? 2 : 1) * nsq;
  if (e < mats) {
    const size_t m = e / nsq, f = e % nsq;
    const size_t src = m * psq + (f / nc) * ncp + f % nc;
    double s = 0.0;
    for (int k = 0; k < nsplit; ++k) s += slabs[(size_t)k * (need_h ? 2 : 1) * psq + src];
    stats[e] = s;
  } else if (e < mats + 3 * (size_t)nc) {
    const size_t f = e - mats;
    const size_t c = f / nc, row = f % nc;
    if (rows_only && c == 0) return;  // loss-only: Σψ′ not computed
    double s = 0.0;
    for (int w = 0; w < nwg1; ++w) s += rows[(size_t)w * 3 * ncp + c * ncp + row];
    stats[base_rows + f] = dens < 0 ? s : finalize_row(dens, alpha, n, (int)c, s);
  }
}

// Per-workgroup partials into the compact stats layout
// [G nc×nc | H nc×nc | Σψ′ nc | Σℓ nc | Σy² nc] (same order as k_reduce_rows).
__global__ void __launch_bounds__(256) k_reduce(const double* __restrict__ partials, int nwg, size_t pstride,
                                                int ncp, int nc, bool need_h, double* __restrict__ stats, int dens,
                                                double alpha, double n) {
  __shared__ double red[4][RED_OUT];
  const size_t nsq = (size_t)nc * nc;
  const size_t total = (need_h ? 2 : 1) * nsq + 3 * (size_t)nc;
  const size_t e = blockIdx.x * (size_t)RED_OUT + threadIdx.x % RED_OUT;
  const bool ok = e < total;
  size_t src = 0;
  if (!ok) src = 0;
  else if (e < nsq) src = (e / nc) * ncp + e % nc;
  else if (need_h && e < 2 * nsq) { const size_t f = e - nsq; src = (size_t)ncp * ncp + (f / nc) * ncp + f % nc; }
  else {
    const size_t f = e - (need_h ? 2 : 1) * nsq;
    src = (size_t)(need_h ? 2 : 1) * ncp * ncp + (f / nc) * ncp + f % nc;
  }
  const double s = reduce_partials(partials + src, nwg, pstride, ok, red);
  const size_t mats = (need_h ? 2 : 1) * nsq;
  if (ok && threadIdx.x < RED_OUT) stats[e] = e < mats ? s : finalize_row(dens, alpha, n, (int)((e - mats) / nc), s);
}

// ---------------------------------------------------------------------------
// Y = W·X̃ materialised row-major (solver.rs:182,199-214 sources / transform;
// benchmarks.rs:34 X = A·S; the Y chunks of the JADE moments). W fragments live
// in VGPRs for the whole launch (read once), X̃ blocks of 16 samples × 4·KS
// features are staged by LDS-DMA (double-buffered, one barrier per block) and
// each wave runs ONE chain of KS MFMAs per 16×16 tile with W as the A operand,
// so by the f64 C/D map lane l holds Y[16·ib + (l>>4) + 4r][16·b + (l&15)]:
// every store instruction writes 4 rows × 128 contiguous bytes. blockIdx.y
// picks 8 row blocks (128 rows); feature counts above 4·KS come in chunks of
// 4·KS (host loop; `accumulate` adds the partial product already in Y).
// Samples ≥ n_out are computed from X's zero padding and never stored.
// ---------------------------------------------------------------------------
template <int KS>
__global__ void __launch_bounds__(FUSED_THREADS, 2)
k_ystore(const double* __restrict__ X, uint64_t ldx, int nrows_x, const double* __restrict__ WpT, int ncp, int nc,
         uint64_t n_out, uint64_t bpw, uint64_t n_blocks, double* __restrict__ Y, uint64_t ldy, int accumulate,
         uint64_t nwgx) {
  constexpr int NFP = 4 * KS, XS = 16 * NFP, NU = NFP / 64;  // LDS-DMA instructions per wave per block
  static_assert(NFP % 64 == 0, "8 waves × 8 rows per instruction");
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  uint64_t wx;
  int role;
  if (!xcd_decode((ncp / 16 + 7) / 8, nwgx, wx, role)) return;
  const int ib = role * 8 + wave;
  const bool active = ib < ncp / 16;
  extern __shared__ double smem[];
  double* xs0 = smem;  // [2 buffers][2 blocks][NFP][16]
  double wf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) wf[ks] = active ? WpT[(size_t)(4 * ks + lk) * ncp + ib * 16 + lr] : 0.0;
  const double* src[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int xr = wave * (NFP / 8) + 8 * u + (lane >> 3);
    src[u] = X + (size_t)(xr < nrows_x ? xr : 0) * ldx + 2 * (lane & 7);  // rows ≥ nrows_x: zero W columns
  }
  auto stage = [&](uint64_t b, double* xs) {
#pragma unroll
    for (int u = 0; u < NU; ++u)
      __builtin_amdgcn_global_load_lds((gbl_vptr)(src[u] + b * 16),
                                       (lds_vptr)(xs + (wave * (NFP / 8) + 8 * u) * 16), 16, 0, 0);
  };
  const uint64_t b_begin = wx * bpw;
  const uint64_t b_end = b_begin + bpw < n_blocks ? b_begin + bpw : n_blocks;
  if (b_begin >= b_end) return;
  // blocks in pairs: two independent MFMA chains and one barrier per 32 samples
  auto stage2 = [&](uint64_t b0, double* xs) {
    stage(b0, xs);
    if (b0 + 1 < b_end) stage(b0 + 1, xs + XS);
  };
  stage2(b_begin, xs0);
  __syncthreads();
  int cur = 0;
  for (uint64_t b0 = b_begin; b0 < b_end; b0 += 2) {
    if (b0 + 2 < b_end) stage2(b0 + 2, xs0 + (cur ^ 1) * 2 * XS);
    __builtin_amdgcn_sched_barrier(0);  // the DMA stays ahead of this pair's stores (dma_barrier)
    if (active) {
      d4 ya = d4{0, 0, 0, 0}, yb = d4{0, 0, 0, 0};  // yb: stale LDS when the pair is cut short (not stored)
      const double* xrow = xs0 + cur * 2 * XS + lk * 16 + lr;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        ya = mfma(wf[ks], xrow[(4 * ks) * 16], ya);
        yb = mfma(wf[ks], xrow[XS + (4 * ks) * 16], yb);
      }
      const uint64_t t = b0 * 16 + lr;
      // both 16 × 16 tiles inside Y and no read-back: exactly 8 stores after the DMA
      if (!accumulate && b0 * 16 + 32 <= n_out && ib * 16 + 16 <= nc) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          double* p = Y + (size_t)(ib * 16 + lk + 4 * r) * ldy + t;
          p[0] = ya[r];
          p[16] = yb[r];
        }
        dma_barrier<8>();
        cur ^= 1;
        continue;
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint64_t th = t + 16 * h;
        if (th < n_out)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = ib * 16 + lk + 4 * r;
            if (row < nc) {
              double* p = Y + (size_t)row * ldy + th;
              const double v = h ? yb[r] : ya[r];
              *p = accumulate ? *p + v : v;
            }
          }
      }
    }
    dma_barrier<0>();  // edge tiles / inactive waves: drain everything
    cur ^= 1;
  }
}

__global__ void k_sum_slabs(const double* __restrict__ slabs, int splits, size_t n, double* __restrict__ out) {
  const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (e >= n) return;
  double s = 0.0;
  for (int k = 0; k < splits; ++k) s += slabs[(size_t)k * n + e];
  out[e] = s;
}

// Row sums Σ_t X[k][t] over this shard: partials[wg][k], T split over workgroups.
__global__ void __launch_bounds__(256) k_rowsum(const double* __restrict__ X, uint64_t ldx, uint64_t n_local,
                                                int nf, uint64_t per, double* __restrict__ partials) {
  // blockIdx.y = row k, blockIdx.x = slice [t0, t0 + per) of the (zero-padded) row;
  // 16-B loads, four independent partial sums per thread for memory-level parallelism
  __shared__ double red[256];
  const int k = blockIdx.y;
  const uint64_t t0 = blockIdx.x * per, t1 = std::min<uint64_t>(ldx, t0 + per);
  const double* row = X + (size_t)k * ldx;
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  uint64_t t = t0 + 2 * threadIdx.x;
  for (; t + 3 * 512 < t1; t += 4 * 512) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double2 v = *reinterpret_cast<const double2*>(row + t + u * 512);
      s[u] += v.x + v.y;
    }
  }
  for (; t < t1; t += 512) {
    const double2 v = *reinterpret_cast<const double2*>(row + t);
    s[0] += v.x + v.y;
  }
  red[threadIdx.x] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) partials[(size_t)blockIdx.x * nf + k] = red[0];
  (void)n_local;  // columns past n_local are zero (alloc_x zero-fills the padding)
}

// Resident-X centring: X[k][t] ← X[k][t] − μ[k] (UNDO: + μ[k]) for t < n_local,
// the padding left at zero. The subtraction is the one every pass kernel would
// otherwise do while staging X, so the centred X is bit-identical to it.
template <bool UNDO>
__global__ void __launch_bounds__(256) k_shift_rows(double* __restrict__ X, uint64_t ldx, uint64_t n_local,
                                                    const double* __restrict__ mu) {
  const int k = blockIdx.y;
  const double m = mu[k];
  double* row = X + (size_t)k * ldx;
  for (uint64_t t = 2 * ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x); t < n_local;
       t += 2 * (uint64_t)gridDim.x * blockDim.x) {
    double2 v = *reinterpret_cast<double2*>(row + t);
    v.x = UNDO ? v.x + m : v.x - m;
    if (t + 1 < n_local) v.y = UNDO ? v.y + m : v.y - m;
    *reinterpret_cast<double2*>(row + t) = v;
  }
}

// Fourth moments for JADE: out[p][q] += Σ_t z_p z_q, z_(i≤j) = y_i y_j, over a Y chunk.
__global__ void __launch_bounds__(256) k_moments4(const double* __restrict__ Y, uint64_t ldy, uint64_t cn, int nc,
                                                  const int* __restrict__ pi, const int* __restrict__ pj, int np,
                                                  double* __restrict__ out) {
  __shared__ double za[32][65];
  __shared__ double zb[32][65];
  const int tiles = (np + 31) / 32;
  const int ti = blockIdx.x / tiles, tj = blockIdx.x % tiles;
  if (tj < ti) return;  // symmetric: upper tiles only
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  double acc[2][2] = {};
  for (uint64_t t0 = 0; t0 < cn; t0 += 64) {
    for (int e = threadIdx.x; e < 32 * 64; e += 256) {
      const int r = e / 64, c = e % 64;
      const uint64_t t = t0 + c;
      const int p = ti * 32 + r, q = tj * 32 + r;
      za[r][c] = (p < np && t < cn) ? Y[(size_t)pi[p] * ldy + t] * Y[(size_t)pj[p] * ldy + t] : 0.0;
      zb[r][c] = (q < np && t < cn) ? Y[(size_t)pi[q] * ldy + t] * Y[(size_t)pj[q] * ldy + t] : 0.0;
    }
    __syncthreads();
    for (int c = 0; c < 64; ++c) {
      const double a0 = za[ty * 2][c], a1 = za[ty * 2 + 1][c];
      const double b0 = zb[tx * 2][c], b1 = zb[tx * 2 + 1][c];
      acc[0][0] = fma(a0, b0, acc[0][0]); acc[0][1] = fma(a0, b1, acc[0][1]);
      acc[1][0] = fma(a1, b0, acc[1][0]); acc[1][1] = fma(a1, b1, acc[1][1]);
    }
    __syncthreads();
  }
  for (int u = 0; u < 2; ++u)
    for (int v = 0; v < 2; ++v) {
      const int p = ti * 32 + ty * 2 + u, q = tj * 32 + tx * 2 + v;
      if (p < np && q < np) out[(size_t)p * np + q] += acc[u][v];
    }
}

// Fourth moments for JADE on MFMA (jade.rs:91-113 as a Gram of pair products).
// Every entry of the np × np pair Gram M[(i,j)][(k,l)] = Σ_t y_i y_j y_k y_l is
// one of the C(n+3, 4) distinct moments E[y_a y_b y_c y_d], a ≤ b ≤ c ≤ d, and
// that moment is the Gram entry of ROW pair (a, b) and COLUMN pair (c, d) with
// b ≤ c. So rows are ordered by their larger index (R: (a, b) ↦ b(b+1)/2 + a),
// columns by their smaller one (C: (c, d) ↦ c·n − c(c−1)/2 + d − c), and only the
// 64 × 32 (R, C) patches that hold some b ≤ c are computed — 426 of them at
// n = 64, 0.87 M Gram entries for the 0.77 M distinct moments (the symmetric
// upper triangle would be 2.2 M); k_moments4_fill then gathers the full
// lexicographic M the host expects.
// One patch per wave, any 8 patches per workgroup (a "pack"): every wave forms
// its own A/B fragments — pair products y_a·y_b of its 64 rows and 32 columns —
// in registers from the Y stage in LDS, so the waves share nothing but the
// stage. Per 64-sample stage: the nc ≤ 64 Y rows land in LDS by LDS-DMA one
// stage ahead (layout [4 sub-blocks][64 rows][16], 16-B segments XOR-swizzled
// by row so the 16 rows of a fragment hit distinct banks), then 16 k-steps of
// 8 MFMAs per wave; one barrier per stage. Samples past cn read zeros (the
// caller zero-pads the chunk to a multiple of 64).
// XCD-aware grid: block b runs on XCD b % 8 (round-robin dispatch), item
// (b % 8)·per_xcd + b / 8 ↦ (split, pack) split-major, so the ~32 workgroups an
// XCD runs at once are mostly packs of ONE split streaming the same Y range in
// lockstep — the XCD's L2 serves the re-reads. Slab s holds split s's partial
// Gram (summed in fixed order by k_moments4_reduce).
// LDS index of Y(row, t) in a [64][16] sub-block: rows are 128 B (32 banks), so rows
// r and r + 2 share banks; segment s of row r sits at slot s ^ ((r >> 1) & 7), which
// gives 16 consecutive rows at one t 16 distinct 8-B bank pairs
__device__ __forceinline__ int m4_ys(int row, int t) {
  return row * 16 + ((((t >> 1) ^ ((row >> 1) & 7))) << 1) + (t & 1);
}
constexpr int M4_STAGE = 64;                       // samples per stage
constexpr int M4_STAGE_DBL = 64 * M4_STAGE;        // doubles per stage buffer
constexpr int M4_PACK = FUSED_THREADS / 64;        // patches (waves) per workgroup
// One 64-sample stage of k_moments4_patch for one wave: 16 k-steps of 8 MFMAs, the 12
// Y operands of k-step kk + 1 read from LDS while the MFMAs of kk run. The buffer and
// sub-block offsets are compile-time, so every read is the per-lane row offset plus
// an immediate.
template <int CUR>
__device__ __forceinline__ void m4_stage(const double* smem, const int (&off)[4][12], d4 (&acc)[4][2]) {
  const double* ys = smem + CUR * M4_STAGE_DBL;
  double y[12];
#pragma unroll
  for (int r = 0; r < 12; ++r) y[r] = ys[off[0][r]];
#pragma unroll
  for (int kk = 0; kk < M4_STAGE / 4; ++kk) {
    double a[4], b[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = y[2 * i] * y[2 * i + 1];
#pragma unroll
    for (int j = 0; j < 2; ++j) b[j] = y[8 + 2 * j] * y[9 + 2 * j];
    if (kk + 1 < M4_STAGE / 4) {
      const double* sb = ys + ((kk + 1) >> 2) * 1024;
#pragma unroll
      for (int r = 0; r < 12; ++r) y[r] = sb[off[(kk + 1) & 3][r]];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);  // keep each k-step's reads with its MFMAs
  }
}
__global__ void __launch_bounds__(FUSED_THREADS, 1)
k_moments4_patch(const double* __restrict__ Y, uint64_t ldy, uint64_t n_stage, int nc, const int* __restrict__ ri,
                 const int* __restrict__ rj, const int* __restrict__ ci, const int* __restrict__ cj, int np,
                 const int* __restrict__ packs, int npack, int nsplit, uint64_t spb, uint64_t per_xcd,
                 double* __restrict__ slabs, size_t slab_stride) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const uint64_t item = (uint64_t)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  const int split = (int)(item / npack), pack = (int)(item % npack);
  if (split >= nsplit) return;  // padding item (uniform over the workgroup)
  const int pat = packs[pack * M4_PACK + wave];
  const bool active = pat >= 0;
  const int g = active ? pat >> 16 : 0, h = active ? pat & 0xffff : 0;
  extern __shared__ double smem[];  // [2][M4_STAGE_DBL]
  d4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = d4{0, 0, 0, 0};
  // this lane's pair rows: A block i ↦ R pair g·64 + 16i + lr, B block j ↦ C pair h·32 + 16j + lr
  // (pairs past np use row 0; their entries are never stored)
  int ra0[4], ra1[4], rb0[2], rb1[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = g * 64 + 16 * i + lr;
    ra0[i] = p < np ? ri[p] : 0;
    ra1[i] = p < np ? rj[p] : 0;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int q = h * 32 + 16 * j + lr;
    rb0[j] = q < np ? ci[q] : 0;
    rb1[j] = q < np ? cj[q] : 0;
  }
  const uint64_t s_begin = (uint64_t)split * spb, s_end = s_begin + spb < n_stage ? s_begin + spb : n_stage;
  // LDS-DMA: instruction u of wave w moves sub-block u, rows 8w … 8w+7 (rows ≥ nc
  // read row 0, never gathered); lane L → row 8w + L/8, slot L%8 holds segment (L%8) ^ ((row/2)%8)
  const int yrow = 8 * wave + (lane >> 3);
  const double* ysrc = Y + (size_t)(yrow < nc ? yrow : 0) * ldy + 2 * ((lane & 7) ^ ((yrow >> 1) & 7));
  auto stage = [&](uint64_t s, double* ys) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      __builtin_amdgcn_global_load_lds((gbl_vptr)(ysrc + s * M4_STAGE + 16 * u), (lds_vptr)(ys + u * 1024 + wave * 128),
                                       16, 0, 0);
  };
  // per-lane LDS offsets of the 12 operand rows (A: y_a, y_b of 4 R pairs; B: of 2 C
  // pairs) at t = 4·kq + lane/16 of a sub-block
  int off[4][12];
#pragma unroll
  for (int kq = 0; kq < 4; ++kq) {
    const int t = 4 * kq + lk;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      off[kq][2 * i] = m4_ys(ra0[i], t);
      off[kq][2 * i + 1] = m4_ys(ra1[i], t);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      off[kq][8 + 2 * j] = m4_ys(rb0[j], t);
      off[kq][9 + 2 * j] = m4_ys(rb1[j], t);
    }
  }
  if (s_begin < s_end) {  // stages alternate between the two buffers, two per trip
    stage(s_begin, smem);
    __syncthreads();
    for (uint64_t s = s_begin; s < s_end; s += 2) {
      if (s + 1 < s_end) stage(s + 1, smem + M4_STAGE_DBL);  // buffer 1 was read last in the previous trip
      if (active) m4_stage<0>(smem, off, acc);
      __syncthreads();  // stage s read by every wave, this wave's DMA of s + 1 landed
      if (s + 1 >= s_end) break;
      if (s + 2 < s_end) stage(s + 2, smem);
      if (active) m4_stage<1>(smem, off, acc);
      __syncthreads();
    }
  }
  if (!active) return;
  double* out = slabs + split * slab_stride;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = g * 64 + 16 * i + lk + 4 * r, q = h * 32 + 16 * j + lr;
        if (p < np && q < np) out[(size_t)p * np + q] = acc[i][j][r];
      }
}

// acc[p][q] (+)= Σ_s slabs[s][p][q] over the 64 × 32 (R, C) patches k_moments4_patch computed
__global__ void k_moments4_reduce(const double* __restrict__ slabs, int nsplit, size_t slab_stride, int np,
                                  const unsigned char* __restrict__ pmask, int accumulate, double* __restrict__ acc) {
  const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (e >= (size_t)np * np) return;
  const int p = (int)(e / np), q = (int)(e % np), nqc = (np + 31) / 32;
  if (!pmask[(p / 64) * nqc + q / 32]) return;
  double s = 0.0;
  for (int k = 0; k < nsplit; ++k) s += slabs[k * slab_stride + e];
  acc[e] = accumulate ? acc[e] + s : s;
}

// out[p][q] = M[(i,j)][(k,l)] in the lexicographic pair order (pi, pj) from the
// (R, C) Gram: the sorted indices a ≤ b ≤ c ≤ d name the entry (R(a,b), C(c,d)).
__global__ void k_moments4_fill(const double* __restrict__ acc, const int* __restrict__ pi, const int* __restrict__ pj,
                                int n, int np, double* __restrict__ out) {
  const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (e >= (size_t)np * np) return;
  const int p = (int)(e / np), q = (int)(e % np);
  int v[4] = {pi[p], pj[p], pi[q], pj[q]};
#pragma unroll
  for (int i = 0; i < 3; ++i)  // sort 4
#pragma unroll
    for (int j = 0; j < 3 - i; ++j)
      if (v[j] > v[j + 1]) { const int t = v[j]; v[j] = v[j + 1]; v[j + 1] = t; }
  const int r = v[1] * (v[1] + 1) / 2 + v[0];
  const int c = v[2] * n - v[2] * (v[2] - 1) / 2 + (v[3] - v[2]);
  out[e] = acc[(size_t)r * np + c];
}

// ---------------------------------------------------------------------------
// Synthetic mixture (benches/benchmarks.rs:8-35), generated in HBM.
// S[i][t] from LCG state number i·T + t + 1 (jump-ahead per column, then the
// fixed affine map of T steps per row), Laplace by inverse CDF; u == 0 is
// replaced by 2^-32.
// ---------------------------------------------------------------------------
struct Affine { uint64_t a, c; };
__host__ __device__ inline Affine lcg_jump(uint64_t n) {
  uint64_t a = 6364136223846793005ull, c = 1ull, ra = 1ull, rc = 0ull;
  while (n) {
    if (n & 1ull) { ra = ra * a; rc = rc * a + c; }
    c = c * a + c;
    a = a * a;
    n >>= 1;
  }
  return {ra, rc};
}

__device__ __forceinline__ double laplace_of(uint64_t st) {
  double u = (double)(st >> 33) / 2147483648.0;
  if (u == 0.0) u = 0x1p-32;
  return u < 0.5 ? log(2.0 * u) : -log(2.0 * (1.0 - u));
}

#include "jade_sweeps.inc"
#include "expm.inc"  // try 1's map expm(α·D) on the device, the host's bits (after the granules)

// Cumulant matrices for the sweeps from the lexicographic fourth moments M (np × np, pair
// index m ↔ (i, j), i ≤ j, the order of jade_warm_start's pidx and pos): A[pos(k,l)][m] =
// (q(k,l) + q(l,k)) / 2 with q = M[m][pos]/t − δ_ij δ_kl − δ_ik δ_jl − δ_il δ_jk — the host
// build's expressions in its order (jade.rs:101-126), so the same bits.
__global__ void __launch_bounds__(256) k_jade_cumulants(const double* __restrict__ M, const int* __restrict__ pi,
                                                       const int* __restrict__ pj, int np, double t,
                                                       double* __restrict__ A) {
  const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (size_t)np * np) return;
  const int ps = (int)(e / np), m = (int)(e % np);
  const int i = pi[m], j = pj[m], k = pi[ps], l = pj[ps];
  const double x = M[(size_t)m * np + ps] / t;
  const double d1 = (i == j && k == l) ? 1.0 : 0.0;
  const double d2 = (i == k && j == l) ? 1.0 : 0.0, d3 = (i == l && j == k) ? 1.0 : 0.0;
  const double qkl = x - d1 - d2 - d3;  // q(k, l)
  const double qlk = x - d1 - d3 - d2;  // q(l, k): δ_ik δ_jl and δ_il δ_jk trade places
  A[e] = (qkl + qlk) / 2.0;
}

// ---------------------------------------------------------------------------
// Exhaustive accuracy of the fp32 transcendental instructions the line-search
// screen uses (v_exp_f32 = 2^x, v_log_f32 = log2 x), over every fp32 input of the
// ranges the screen feeds them: the screen's rigorous bound (DeviceCtx::
// eval_loss_screen) is built from compile-time constants that these measurements
// must not exceed (tests/test_gpu_screen32.py). fp64 libm is the reference.
//   out[blk][0]: max |2^z_hw − 2^z| / 2^z over z ∈ [−126, 0]
//   out[blk][1]: max |2^z_hw − 2^z| (absolute) over z ∈ [−150, −126)
//   out[blk][2]: max |log2_hw p − log2 p| (absolute) over p ∈ [2^-4, 1]
//   out[blk][3]: 1 unless 2^0 ≠ 1 or log2 1 ≠ 0 (then 0)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_check_f32_transc(double* __restrict__ out) {
  __shared__ double red[4][256];
  double m0 = 0.0, m1 = 0.0, m2 = 0.0, ok = 1.0;
  const uint32_t nthr = gridDim.x * blockDim.x, id = blockIdx.x * blockDim.x + threadIdx.x;
  // z: bit patterns 0x80000000 (−0) … 0xC3160000 (−150)
  for (uint32_t b = 0x80000000u + id; b <= 0xC3160000u; b += nthr) {
    const float z = __uint_as_float(b);
    const double hw = (double)__builtin_amdgcn_exp2f(z), ref = exp2((double)z);
    if (z >= -126.0f) m0 = fmax(m0, fabs(hw - ref) / ref);
    else m1 = fmax(m1, fabs(hw - ref));
  }
  // p: bit patterns of 2^-4 … 1
  for (uint32_t b = 0x3d800000u + id; b <= 0x3f800000u; b += nthr) {
    const float p = __uint_as_float(b);
    m2 = fmax(m2, fabs((double)__builtin_amdgcn_logf(p) - log2((double)p)));
  }
  if (id == 0 && (__builtin_amdgcn_exp2f(0.0f) != 1.0f || __builtin_amdgcn_logf(1.0f) != 0.0f)) ok = 0.0;
  red[0][threadIdx.x] = m0; red[1][threadIdx.x] = m1; red[2][threadIdx.x] = m2; red[3][threadIdx.x] = ok;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int c = 0; c < 4; ++c)
        red[c][threadIdx.x] = c == 3 ? fmin(red[c][threadIdx.x], red[c][threadIdx.x + s])
                                     : fmax(red[c][threadIdx.x], red[c][threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x < 4) out[blockIdx.x * 4 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void k_gen_sources(double* __restrict__ S, uint64_t lds, int nf, uint64_t t_begin, uint64_t cn,
                              uint64_t seed, uint64_t jump_a, uint64_t jump_c) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t >= cn) return;
  const Affine j = lcg_jump(t_begin + t + 1);
  uint64_t st = j.a * seed + j.c;
  for (int i = 0; i < nf; ++i) {
    S[(size_t)i * lds + t] = laplace_of(st);
    st = jump_a * st + jump_c;
  }
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device), raised when a
// larger size is asked for; thread-safe (the rank contexts of an in-process group launch
// from their own host threads)
static void lds_attr(const void* f, int bytes) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> set;
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  int& have = set[{f, dev}];
  if (bytes > have) {
    HIP_OK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    have = bytes;
  }
}

// The last DeviceCtx teardown: [0] wall ms, [1] ms in its hipFree calls, [2] the largest
// single hipFree of the context's life, [3] ms of the closing hipDeviceSynchronize
static std::mutex g_teardown_mu;
static double g_teardown[4] = {0, 0, 0, 0};

// Live device contexts per device in this process (the JADE sweeps launch plainly only when
// their context is alone on its device; jade_sweeps_impl)
static std::mutex g_ctx_mu;
static std::map<int, int> g_ctx_count;
static int ctxs_on_device(int dev) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  auto it = g_ctx_count.find(dev);
  return it == g_ctx_count.end() ? 0 : it->second;
}
static void ctx_count_add(int dev, int d) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  g_ctx_count[dev] += d;
}

// ---------------------------------------------------------------------------
// Device context: one GPU, one X shard, optional collective (RCCL, or an
// in-process rank group; collective.hpp).
// ---------------------------------------------------------------------------
struct DeviceCtx : Evaluator {
  // Timed HBM allocation calls (a 6 s stall in the first setup after a
  // large context was freed): [0] hipMalloc, [1] hipFree, [2] hipMemGetInfo — total ms, count,
  // largest single call. pc_ctx_alloc_stats; the destructor's own record: pc_last_teardown.
  struct AllocStats { double ms[3] = {0, 0, 0}, mx[3] = {0, 0, 0}; uint64_t n[3] = {0, 0, 0}; };
  AllocStats as_;
  template <class F>
  hipError_t timed_call(int k, F&& f) {
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = f();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    as_.ms[k] += ms;
    as_.mx[k] = std::max(as_.mx[k], ms);
    ++as_.n[k];
    return e;
  }
  hipError_t t_malloc(void** p, size_t n) { return timed_call(0, [&] { return hipMalloc(p, n); }); }
  hipError_t t_free(void* p) { return timed_call(1, [&] { return hipFree(p); }); }
  hipError_t t_meminfo(size_t* f, size_t* t) { return timed_call(2, [&] { return hipMemGetInfo(f, t); }); }
  int device = 0, rank = 0, world = 1;
  hipStream_t stream = nullptr;
  std::unique_ptr<Collective> coll_;
  double* X = nullptr;
  uint64_t nf = 0, n_local_ = 0, ldx = 0, n_total = 0, t0 = 0;
  int n_cu = 256;
  // scratch
  double* d_w = nullptr; size_t cap_w = 0;
  double* d_mu = nullptr; size_t cap_mu = 0;
  double* d_part = nullptr; size_t cap_part = 0;
  double* d_stats = nullptr; size_t cap_stats = 0;
  double* d_chunk = nullptr; size_t cap_chunk = 0;
  double* d_ybuf = nullptr; size_t cap_ybuf = 0;
  bool ybuf_failed = false;
  // state of the last split (loss-only) evaluation whose Y is kept in d_ybuf
  size_t kept_nc = 0; int kept_nb = 0;
  hipEvent_t ev[4];
  double last_kernel_ms = 0, last_call_ms = 0;
  double last_pass_kernel_ms() const override { return last_kernel_ms; }
  double sum_kernel_ms = 0, sum_call_ms = 0;
  uint64_t n_kernel = 0;
  // Pinned host staging for the per-pass uploads (W image, W digit image): the copy is
  // issued asynchronously and an event after it guards the slot — the next writer of the
  // slot waits on that event, so no stream synchronisation follows the upload.
  struct PinSlot { void* p = nullptr; size_t cap = 0; hipEvent_t ev = nullptr; bool pending = false; unsigned flags = 0; };
  PinSlot pin_w_, pin_wsl_, pin_out_, pin_in_;
  // Without a collective the last kernel of a pass (the fixed-order reduction) stores the
  // statistics straight into coherent pinned host memory: no D2H copy on the call's GPU
  // timeline. With one, the statistics stay in HBM for the all-reduce.
  PinSlot pin_direct_{nullptr, 0, nullptr, false, hipHostMallocCoherent};
  double* direct_acquire(size_t n) {
    if (coll_) return nullptr;
    return (double*)pin_acquire(pin_direct_, std::max<size_t>(n, 1) * sizeof(double));
  }
  // D2H of n doubles through the pinned out slot (a DMA copy; a pageable destination takes a
  // staging blit and a blocking copy): enqueue now, copy_out() after the stream has synced
  const double* d2h_enqueue(const double* dsrc, size_t n) {
    double* h = (double*)pin_acquire(pin_out_, std::max<size_t>(n, 1) * sizeof(double));
    HIP_OK(hipMemcpyAsync(h, dsrc, n * sizeof(double), hipMemcpyDeviceToHost, stream));
    pin_release(pin_out_);
    return h;
  }
  static void copy_out(double* dst, const double* staged, size_t n) { std::memcpy(dst, staged, n * sizeof(double)); }
  void* pin_acquire(PinSlot& sl, size_t bytes) {
    if (sl.pending) {
      HIP_OK(hipEventSynchronize(sl.ev));
      sl.pending = false;
    }
    if (sl.cap < bytes) {
      if (sl.p) HIP_OK(hipHostFree(sl.p));
      sl.p = nullptr;
      sl.cap = 0;
      HIP_OK(hipHostMalloc(&sl.p, bytes, sl.flags));
      sl.cap = bytes;
    }
    if (!sl.ev) HIP_OK(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
    return sl.p;
  }
  void pin_release(PinSlot& sl) {  // after the copies from the slot are enqueued
    HIP_OK(hipEventRecord(sl.ev, stream));
    sl.pending = true;
  }

  DeviceCtx(int dev, int rk, int ws, const char* uid, std::shared_ptr<LocalGroup> grp)
      : device(dev), rank(rk), world(ws) {
    HIP_OK(hipSetDevice(device));
    HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    for (auto& e : ev) HIP_OK(hipEventCreate(&e));
    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, device));
    n_cu = prop.multiProcessorCount;
    // world > 1 without an RCCL id or a group: a detached shard (no communicator; every
    // statistic is this shard's partial sum and the caller adds them up)
    // (an id at world 1: a one-rank RCCL communicator — the RCCL path on one GPU)
    if (grp) coll_ = make_local_collective(std::move(grp), rank);
    else if (uid) coll_ = make_rccl_collective(rank, world, uid);
    if (const char* e = std::getenv("PICARD_TEST_PIN_DIGITS")) pin_test_ = std::atoi(e) != 0;
    ctx_count_add(device, 1);
  }
  ~DeviceCtx() override {
    const auto td0 = std::chrono::steady_clock::now();
    const AllocStats before = as_;
    ctx_count_add(device, -1);
    (void)hipSetDevice(device);
    coll_.reset();
    for (double* p : {X, d_w, d_mu, d_part, d_stats, d_chunk, d_ybuf, d_tbuf, d_ybuf2, d_slab, d_trow, d_shift_sum, d_shift_part, d_wys, d_src, d_jade})
      if (p) (void)t_free(p);
    for (void* p : {(void*)d_xsl, (void*)d_xsc, (void*)d_wsc, (void*)d_xsf, (void*)d_xm})  // d_wsl lies inside d_wsc's allocation
      if (p) (void)t_free(p);
    for (auto& e : ev) (void)hipEventDestroy(e);
    for (auto& pr : ar_ev_)
      for (auto& e : pr)
        if (e) (void)hipEventDestroy(e);
    for (PinSlot* sl : {&pin_w_, &pin_wsl_, &pin_out_, &pin_in_, &pin_direct_, &pin_xm_, &pin_xmo_}) {
      if (sl->pending) (void)hipEventSynchronize(sl->ev);
      if (sl->p) (void)hipHostFree(sl->p);
      if (sl->ev) (void)hipEventDestroy(sl->ev);
    }
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    // the release as a whole: hipDeviceSynchronize charges any deferred work of the frees to
    // this teardown instead of to the next context's first allocation —
    // only when no other context of this process lives on the device, so closing one rank of an
    // in-process group (or an error path) never waits for another context's work
    const auto ts = std::chrono::steady_clock::now();
    if (ctxs_on_device(device) == 0) (void)hipDeviceSynchronize();
    const double sync_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts).count();
    std::lock_guard<std::mutex> lk(g_teardown_mu);
    g_teardown[0] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - td0).count();
    g_teardown[1] = as_.ms[1] - before.ms[1];
    g_teardown[2] = as_.mx[1];
    g_teardown[3] = sync_ms;
  }

  uint64_t n_features() const override { return nf; }
  uint64_t n_samples() const override { return n_total; }
  uint64_t n_local() const override { return n_local_; }
  bool partial_sums() const override { return world > 1 && !coll_; }
  void abort_group(const std::string& why) noexcept override {
    if (coll_) coll_->abort(why);
  }
  // wait for this context's stream; with a collective, a failing peer ends the wait
  void sync() {
    if (coll_) {
      coll_->wait(stream);
      harvest_allreduce_timing();
    } else if (sync_poll_) {
      // poll the stream (yielding the core to any runnable thread between probes): a blocking
      // hipStreamSynchronize wakes ≈ 12 µs after the work ends, a cost every pass pays once —
      // C2-shaped fits are launch-bound (profiles/r06_y/ab_sync_poll.log: N = 64, T = 1e6
      // 0.80 → 0.75 ms per step). Past 0.5 s (setup kernels, JADE) the blocking wait takes over.
      const double t0 = now_ms_d();
      hipError_t e;
      for (uint32_t k = 0; (e = hipStreamQuery(stream)) == hipErrorNotReady; ++k) {
        if ((k & 1023u) == 1023u && now_ms_d() - t0 > 500.0) {
          e = hipStreamSynchronize(stream);
          break;
        }
        sched_yield();
      }
      HIP_OK(e);
    } else {
      HIP_OK(hipStreamSynchronize(stream));
    }
  }
  static double now_ms_d() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  // PICARD_SYNC_POLL=0: every wait on the context's stream is a blocking hipStreamSynchronize
  const bool sync_poll_ = [] {
    const char* e = std::getenv("PICARD_SYNC_POLL");
    return !(e && std::atoi(e) == 0);
  }();
  // Time inside the all-reduces (bench.py's per-rank report): RCCL — device time between HIP
  // events around each ncclAllReduce on the stream (the kernel waits there for the slowest
  // rank); in-process group — host time of the exchange. Events come from a ring, read back
  // at the next sync.
  static constexpr int AR_RING = 16;
  hipEvent_t ar_ev_[AR_RING][2] = {};
  int ar_pending_ = 0;
  double ar_ms_ = 0.0;
  uint64_t ar_timed_ = 0;
  void harvest_allreduce_timing() {
    for (int i = 0; i < ar_pending_; ++i) {
      float ms = 0.0f;
      if (hipEventElapsedTime(&ms, ar_ev_[i][0], ar_ev_[i][1]) == hipSuccess) {
        ar_ms_ += ms;
        ++ar_timed_;
      } else {
        (void)hipGetLastError();
      }
    }
    ar_pending_ = 0;
  }

  double* ensure(double*& p, size_t& cap, size_t n) {
    if (n > cap) {
      if (p) HIP_OK(t_free(p));
      p = nullptr;
      cap = 0;
      if (t_malloc((void**)&p, n * sizeof(double)) != hipSuccess) {
        (void)hipGetLastError();
        // the int8 slice image is a cache: its HBM goes to the pass buffers — unless the
        // ranks agreed on it (the screen branch issues its own collectives): then the
        // allocation fails instead and the group aborts rather than diverging
        if (!xsl_pinned()) release_xsl();
        HIP_OK(t_malloc((void**)&p, n * sizeof(double)));
      }
      cap = n;
    }
    return p;
  }

  void alloc_x(uint64_t nf_, uint64_t n_local, uint64_t n_tot, uint64_t t0_) {
    HIP_OK(hipSetDevice(device));
    if (X) HIP_OK(t_free(X));
    nf = nf_; n_local_ = n_local; n_total = n_tot; t0 = t0_;
    xshift_.clear();
    raw_sums_.clear();
    release_xsl();  // a new X: its slice image is rebuilt on demand
    xsl_failed_ = false;
    wsl_nc_ = 0;    // … and W is sliced again (n_features may change)
    ldx = (n_local + 127) / 128 * 128;  // a fused-pass tile (≤ 128 samples) never crosses a row end
    if (ldx == 0) ldx = 128;
    HIP_OK(t_malloc((void**)&X, nf * ldx * sizeof(double) + 256));
    HIP_OK(hipMemsetAsync(X, 0, nf * ldx * sizeof(double) + 256, stream));
  }

  void load(const double* xh, uint64_t nf_, uint64_t n_local, uint64_t n_tot, uint64_t t0_) {
    alloc_x(nf_, n_local, n_tot, t0_);
    if (n_local)
      HIP_OK(hipMemcpy2DAsync(X, ldx * sizeof(double), xh, n_local * sizeof(double), n_local * sizeof(double),
                              nf, hipMemcpyHostToDevice, stream));
    sync();
  }

  void download(double* out) {
    HIP_OK(hipSetDevice(device));
    unshift_x();  // the caller's data (up to rounding if it was centred in place)
    if (n_local_)
      HIP_OK(hipMemcpy2DAsync(out, n_local_ * sizeof(double), X, ldx * sizeof(double), n_local_ * sizeof(double),
                              nf, hipMemcpyDeviceToHost, stream));
    sync();
  }

  static uint64_t shard_t0(uint64_t n_tot, int world, int rank) {
    const uint64_t base = n_tot / world, rem = n_tot % world;
    return rank * base + std::min<uint64_t>(rank, rem);
  }
  static uint64_t shard_n(uint64_t n_tot, int world, int rank) {
    const uint64_t base = n_tot / world, rem = n_tot % world;
    return base + (rank < (int)rem ? 1 : 0);
  }

  void generate(uint64_t nf_, uint64_t n_tot, uint64_t seed, double* a_out) {
    const uint64_t tt0 = shard_t0(n_tot, world, rank), nl = shard_n(n_tot, world, rank);
    alloc_x(nf_, nl, n_tot, tt0);
    // mixing matrix: states N·T + 1 … N·T + N² (benchmarks.rs:26-32)
    std::vector<double> A(nf * nf);
    const Affine j = lcg_jump(nf * n_tot);
    uint64_t st = j.a * seed + j.c;
    for (size_t e = 0; e < nf * nf; ++e) {
      st = st * 6364136223846793005ull + 1ull;
      A[e] = (double)(st >> 33) / 2147483648.0 - 0.5;
    }
    if (a_out) std::memcpy(a_out, A.data(), A.size() * sizeof(double));
    ystore_upload(A.data(), nf, nf);
    const Affine jt = lcg_jump(n_tot);  // row i → i+1 at fixed t
    const uint64_t CH = 1ull << 22;
    m4_full_ = nullptr;  // d_chunk is reused
    double* S = ensure(d_chunk, cap_chunk, nf * CH);
    for (uint64_t c0 = 0; c0 < nl; c0 += CH) {
      const uint64_t cn = std::min<uint64_t>(CH, nl - c0);
      k_gen_sources<<<(cn + 255) / 256, 256, 0, stream>>>(S, CH, (int)nf, tt0 + c0, cn, seed, jt.a, jt.c);
      HIP_OK(hipGetLastError());
      // X[:, c0:c0+cn] = A·S (benchmarks.rs:34) on MFMA; the padding past n_local stays zero
      ystore_run(S, CH, nf, nf, cn, X + c0, ldx);
    }
    sync();
  }

  void allreduce(double* d, size_t n, const char* tag) {
    if (!coll_) return;
    if (std::strcmp(coll_->kind(), "rccl") != 0) {
      const auto t0 = std::chrono::steady_clock::now();
      coll_->allreduce(d, n, stream, tag);
      ar_ms_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      ++ar_timed_;
      return;
    }
    if (ar_pending_ == AR_RING) {  // ring full before a sync: wait for the oldest pairs
      HIP_OK(hipEventSynchronize(ar_ev_[AR_RING - 1][1]));
      harvest_allreduce_timing();
    }
    hipEvent_t* e = ar_ev_[ar_pending_];
    for (int k = 0; k < 2; ++k)
      if (!e[k]) HIP_OK(hipEventCreate(&e[k]));
    HIP_OK(hipEventRecord(e[0], stream));
    coll_->allreduce(d, n, stream, tag);
    HIP_OK(hipEventRecord(e[1], stream));
    ++ar_pending_;
  }

  // ---- Y = W·Xs stored row-major on MFMA (k_ystore) ------------------------
  // w: host nc × nrows row-major; Xs: device, nrows × (≥ 16·⌈n_out/16⌉) with
  // leading dimension lds and 16-B aligned rows; Y: device nc × n_out, ld ldy.
  double* d_wys = nullptr; size_t cap_wys = 0;
  static int ystore_ks(uint64_t nrows) { return nrows <= 64 ? 16 : nrows <= 128 ? 32 : 64; }
  template <int KS>
  void ystore_ks_launch(const double* Xs, uint64_t lds, uint64_t nrows, const double* dwt, int ncp, size_t nc,
                        uint64_t n_out, double* Y, uint64_t ldy) {
    lds_attr((const void*)k_ystore<KS>, 4 * 16 * 4 * KS * (int)sizeof(double));
    const uint64_t n_blocks = (n_out + 15) / 16;
    const int nroles = (ncp / 16 + 7) / 8;
    // two workgroups per CU in ONE round (a 2·n_cu + 1-th would run alone afterwards)
    const uint64_t want = std::max<uint64_t>(1, std::min<uint64_t>(n_blocks, std::max(1, 2 * n_cu / nroles)));
    const uint64_t bpw = ((n_blocks + want - 1) / want + 1) & ~uint64_t(1);  // whole block pairs
    const unsigned nwg = (unsigned)((n_blocks + bpw - 1) / bpw);
    constexpr int CHK = 4 * KS;
    for (uint64_t k0 = 0; k0 < nrows; k0 += CHK)
      k_ystore<KS><<<xcd_grid(nwg, nroles), FUSED_THREADS, (size_t)4 * 16 * CHK * sizeof(double), stream>>>(
          Xs + k0 * lds, lds, (int)std::min<uint64_t>(CHK, nrows - k0), dwt + k0 * ncp, ncp, (int)nc, n_out, bpw,
          n_blocks, Y, ldy, k0 > 0 ? 1 : 0, (uint64_t)nwg);
    HIP_OK(hipGetLastError());
  }
  // Wᵀ (zero-padded to whole chunks and row blocks) into d_wys, once per map
  void ystore_upload(const double* w, size_t nc, uint64_t nrows) {
    const uint64_t chk = 4 * (uint64_t)ystore_ks(nrows), nfp = (nrows + chk - 1) / chk * chk;
    const size_t ncp = (nc + 15) / 16 * 16;
    std::vector<double> wt((size_t)nfp * ncp, 0.0);
    for (size_t i = 0; i < nc; ++i)
      for (size_t k = 0; k < nrows; ++k) wt[k * ncp + i] = w[i * nrows + k];
    ensure(d_wys, cap_wys, wt.size());
    HIP_OK(hipMemcpyAsync(d_wys, wt.data(), wt.size() * sizeof(double), hipMemcpyHostToDevice, stream));
    sync();  // the host image must outlive the copy; the kernels stay async
  }
  // Y[:, :n_out] = W·Xs with the map of the last ystore_upload (same nc, nrows)
  void ystore_run(const double* Xs, uint64_t lds, uint64_t nrows, size_t nc, uint64_t n_out, double* Y, uint64_t ldy) {
    if (n_out == 0 || nc == 0) return;
    const int ncp = (int)((nc + 15) / 16 * 16);
    switch (ystore_ks(nrows)) {
      case 16: ystore_ks_launch<16>(Xs, lds, nrows, d_wys, ncp, nc, n_out, Y, ldy); break;
      case 32: ystore_ks_launch<32>(Xs, lds, nrows, d_wys, ncp, nc, n_out, Y, ldy); break;
      default: ystore_ks_launch<64>(Xs, lds, nrows, d_wys, ncp, nc, n_out, Y, ldy); break;
    }
  }

  // this shard's row sums of the resident X into st (device), no all-reduce;
  // partials in *part_buf (grown as needed)
  void local_rowsum(double* st, double*& part_buf, size_t& part_cap) {
    // ≥ 8 workgroups per CU in total, slices a multiple of 512 samples (16-B loads)
    const uint64_t slices = std::max<uint64_t>(1, std::min<uint64_t>((ldx + 511) / 512,
                                                                     (uint64_t)(8 * n_cu + nf - 1) / nf));
    const uint64_t per = ((ldx + slices - 1) / slices + 511) / 512 * 512;
    const int nwg = (int)((ldx + per - 1) / per);
    double* part = ensure(part_buf, part_cap, (size_t)nwg * nf);
    k_rowsum<<<dim3(nwg, (unsigned)nf), 256, 0, stream>>>(X, ldx, n_local_, (int)nf, per, part);
    HIP_OK(hipGetLastError());
    k_sum_slabs<<<(nf + 255) / 256, 256, 0, stream>>>(part, nwg, nf, st);
    HIP_OK(hipGetLastError());
  }

  void rowsum(double* out) override {
    HIP_OK(hipSetDevice(device));
    double* st = ensure(d_stats, cap_stats, nf);
    if (xshift_.empty()) local_rowsum(st, d_part, cap_part);
    else  // centred in place: the sums of the caller's data, kept from before the shift
      HIP_OK(hipMemcpyAsync(st, raw_sums_.data(), nf * sizeof(double), hipMemcpyHostToDevice, stream));
    allreduce(st, nf, "rowsum");
    HIP_OK(hipMemcpyAsync(out, st, nf * sizeof(double), hipMemcpyDeviceToHost, stream));
    sync();
  }

  // Resident-X centring. Every pass computes Y = W·(X − μ); instead of
  // subtracting μ while staging X in every pass, the first call with a given μ
  // subtracts it from the resident X in place (k_shift_rows: the same fp64
  // subtraction, so the passes read bit-identical X − μ) and the kernels then
  // run with μ = null. A call with another μ (or none) first restores X by
  // adding the old μ back, which is exact only up to rounding — the solver
  // always passes one μ per fit, so its passes never hit that path.
  std::vector<double> xshift_;  // μ currently subtracted from the resident X (empty: none)
  std::vector<double> raw_sums_;  // this shard's row sums of X before the shift
  double* d_shift_sum = nullptr; size_t cap_shift_sum = 0;
  double* d_shift_part = nullptr; size_t cap_shift_part = 0;
  void shift_rows(const double* mu_host, bool undo) {
    if (!n_local_) return;
    drop_xsl();  // the slice image follows the resident X
    double* dmu = ensure(d_mu, cap_mu, nf);
    HIP_OK(hipMemcpyAsync(dmu, mu_host, nf * sizeof(double), hipMemcpyHostToDevice, stream));
    const unsigned gx = (unsigned)std::min<uint64_t>((n_local_ / 2 + 255) / 256 + 1, std::max(1, 4 * n_cu));
    if (undo) k_shift_rows<true><<<dim3(gx, (unsigned)nf), 256, 0, stream>>>(X, ldx, n_local_, dmu);
    else k_shift_rows<false><<<dim3(gx, (unsigned)nf), 256, 0, stream>>>(X, ldx, n_local_, dmu);
    HIP_OK(hipGetLastError());
    sync();  // the host μ buffer may go away after return
  }
  void unshift_x() {
    if (xshift_.empty()) return;
    shift_rows(xshift_.data(), true);
    xshift_.clear();
    raw_sums_.clear();
  }
  // the μ the kernels must still subtract: always null (see above)
  const double* resident_mu(const double* mu) {
    if (mu && !xshift_.empty() && std::memcmp(mu, xshift_.data(), nf * sizeof(double)) == 0) return nullptr;
    unshift_x();
    if (mu) {
      raw_sums_.assign(nf, 0.0);
      // own buffers: callers may hold d_stats / d_part pointers across this call
      double* st = ensure(d_shift_sum, cap_shift_sum, nf);
      local_rowsum(st, d_shift_part, cap_shift_part);
      HIP_OK(hipMemcpyAsync(raw_sums_.data(), st, nf * sizeof(double), hipMemcpyDeviceToHost, stream));
      shift_rows(mu, false);
      xshift_.assign(mu, mu + nf);
    }
    return nullptr;
  }

  void gram(const double* mu, double* out) override {
    std::vector<double> eye(nf * nf, 0.0);
    for (size_t i = 0; i < nf; ++i) eye[i * nf + i] = 1.0;
    std::vector<double> st(EvalStats::size(nf, false));
    run_eval(eye.data(), nf, mu, DENS_LINEAR, 1.0, false, st.data());
    std::memcpy(out, st.data(), nf * nf * sizeof(double));
  }

  void eval(const double* w, size_t nc, const double* mu, pc_density d, bool need_h, EvalStats* out) override {
    out->nc = nc;
    out->has_h = need_h;
    out->buf.assign(EvalStats::size(nc, need_h), 0.0);
    run_eval(w, nc, mu, d.kind, d.alpha, need_h, out->buf.data());
  }

  // Block → workgroup partition shared by the fused, loss-only and completion
  // kernels: identical partitions give identical summation orders, so the split
  // evaluation is bit-identical to the fused pass. 2 workgroups per CU: the
  // split kernels fit two (≤128 VGPRs), the fused one runs them in two rounds.
  int partition(uint64_t n_blocks, uint64_t* bpw) const {
    const uint64_t nb = std::max<uint64_t>(n_blocks, 1);
    const uint64_t want = std::min<uint64_t>((uint64_t)2 * n_cu, nb);
    *bpw = (nb + want - 1) / want;
    return (int)((nb + *bpw - 1) / *bpw);
  }

  static int pick_nb(size_t nc) { return nc <= 16 ? 1 : nc <= 32 ? 2 : nc <= 64 ? 4 : nc <= 128 ? 8 : 0; }

  // the padded fp64 W staged in pin_w_ by run_eval, not yet copied to d_w
  const double* wp_pending_ = nullptr;
  size_t wp_n_ = 0;
  void flush_wp() {
    if (!wp_pending_) return;
    HIP_OK(hipMemcpyAsync(d_w, wp_pending_, wp_n_ * sizeof(double), hipMemcpyHostToDevice, stream));
    wp_pending_ = nullptr;
  }

  template <int NB, bool H, int D, bool Q>
  void launch_fused(int nfp, const double* dmu, double alpha, double* st, size_t nc) {
    using S = FusedShape<NB>;
    const uint64_t n_blocks = (n_local_ + S::TB - 1) / S::TB;
    uint64_t bpw;
    const int nwg = partition(n_blocks, &bpw);
    const size_t pstride = fused_partial_stride(S::NCP, H);
    double* part = ensure(d_part, cap_part, (size_t)nwg * pstride);
    const size_t lds = (size_t)(2 * S::TS * nfp * 16 + 2 * (H ? 3 : 2) * S::FRAGS) * sizeof(double);
    (void)nfp;
    // NB = 8 without H: the warp-specialised 16-wave kernel (same sums as k_eval_fused<8>),
    // on the int8-digit Y stage when the digit image is there (not for the Gram)
    const bool ws = NB == 8 && !H;
    // (after the partial buffer: an allocation that released the digit image falls back to
    // the fp64 Y stage, which issues the same collectives)
    const bool oz_ok = D != DENS_LINEAR && dmu == nullptr && oz_fused_ready_ && xsl_valid_;
    const bool oz = ws && oz_ok;
    // NB = 4 without H, nf ≤ 64: k_eval_fused<4> on the int8-digit Y stage
    constexpr bool OZ4 = NB == 4 && !H && D != DENS_LINEAR;
    const bool oz4 = OZ4 && oz_ok && oz_kso() == 1;
    // … and its warp-specialised form on the centred resident X (PICARD_NO_WS4=1: the 8-wave kernel)
    const bool ws4 = NB == 4 && !H && dmu == nullptr && nf <= 64 && !no_ws4_;
    // the digit-stage forms of the warp-specialised kernels never read the fp64 W: its copy is
    // left out of the call's timeline
    if (!((ws && oz) || (!ws && ws4 && oz4))) flush_wp();
    // … and with G = ψ·Yᵀ on the i8 matrix cores too (fused_g8.inc): bounded ψ (tanh, exp), the
    // row scales of the W image built for this image's exponent range (upload_wsl)
    constexpr bool G8D = D == DENS_TANH || D == DENS_EXP;
    const bool g8 = G8D && oz && g_stage_ == 0 && g8_scales_ok_ && g8_emax_ == xsc_emax_ && nf <= 128;
    if (g8) {
      if constexpr (G8D) {
        double psc = 0x1p46;  // tanh: |ψ| ≤ 1
        if (D == DENS_EXP) {  // |ψ| = |y|·e^{−αy²/2} ≤ 1/√(α·e) < 2^Fψ
          const double bound = 1.0 / std::sqrt(alpha * 2.718281828459045) * (1.0 + 1e-12);
          psc = std::ldexp(1.0, 46 - (std::ilogb(bound) + 1));
        }
        auto kg8x = k_eval_fused_g8x<D, Q>;
        lds_attr((const void*)kg8x, G8X_LDS);
        HIP_OK(hipEventRecord(ev[1], stream));
        kg8x<<<nwg, G8X_THREADS, G8X_LDS, stream>>>(bpw, n_blocks, part, d_xsl, d_xsc, d_wsl, d_wsc, alpha, psc);
        HIP_OK(hipGetLastError());
        ++n_int8_passes_;
        ++n_g8_passes_;
        HIP_OK(hipEventRecord(ev[2], stream));
        const size_t total = EvalStats::size(nc, H);
        k_reduce<<<(total + RED_OUT - 1) / RED_OUT, 256, 0, stream>>>(part, nwg, pstride, S::NCP, (int)nc, H, st, D,
                                                                      alpha, (double)n_local_);
        HIP_OK(hipGetLastError());
        return;
      }
    }
    auto kws = oz ? k_eval_fused_ws<D, Q, true> : k_eval_fused_ws<D, Q, false>;
    auto kfu = oz4 ? k_eval_fused<NB, H, D, Q, OZ4> : k_eval_fused<NB, H, D, Q, false>;
    auto kw4 = oz4 ? k_eval_fused_ws4<D, Q, OZ4> : k_eval_fused_ws4<D, Q, false>;
    lds_attr(ws ? (const void*)kws : ws4 ? (const void*)kw4 : (const void*)kfu, 160 * 1024 - EXP_TAB_BYTES);
    HIP_OK(hipEventRecord(ev[1], stream));
    if (ws)
      kws<<<nwg, WS_THREADS, lds, stream>>>(X, ldx, n_local_, (int)nf, d_w, dmu, alpha, bpw, n_blocks, part, d_xsl, d_xsc,
                                           d_wsl, d_wsc);
    else if (ws4)
      kw4<<<nwg, WS_THREADS, lds, stream>>>(X, ldx, (int)nf, d_w, alpha, bpw, n_blocks, part, d_xsl, d_xsc, d_wsl, d_wsc);
    else
      kfu<<<nwg, FUSED_THREADS, lds, stream>>>(X, ldx, n_local_, (int)nf, d_w, dmu, alpha, bpw, n_blocks, part, d_xsl,
                                               d_xsc, d_wsl, d_wsc);
    HIP_OK(hipGetLastError());
    if (oz || oz4) ++n_int8_passes_;
    HIP_OK(hipEventRecord(ev[2], stream));
    const size_t total = EvalStats::size(nc, H);
    k_reduce<<<(total + RED_OUT - 1) / RED_OUT, 256, 0, stream>>>(part, nwg, pstride, S::NCP, (int)nc, H, st, D, alpha,
                                                      (double)n_local_);
    HIP_OK(hipGetLastError());
  }

  template <int NB, bool H, bool Q>
  void dispatch_dens(int dens, int nfp, const double* dmu, double alpha, double* st, size_t nc) {
    switch (dens) {
      case DENS_TANH: launch_fused<NB, H, DENS_TANH, Q>(nfp, dmu, alpha, st, nc); break;
      case DENS_EXP: launch_fused<NB, H, DENS_EXP, Q>(nfp, dmu, alpha, st, nc); break;
      case DENS_CUBE: launch_fused<NB, H, DENS_CUBE, Q>(nfp, dmu, alpha, st, nc); break;
      default: launch_fused<NB, H, DENS_LINEAR, false>(nfp, dmu, alpha, st, nc); break;  // Gram
    }
  }
  // Σy² (Q) is accumulated with H (non-orthogonal) or when the caller asks for it
  template <int NB>
  void dispatch_h(bool h, bool q, int dens, int nfp, const double* dmu, double alpha, double* st, size_t nc) {
    if constexpr (NB == 8) {  // H at nc > 64 goes to the tiled path (register budget)
      if (h) throw computation_error("fused pass with H needs nc <= 64");
    } else if (h) {
      dispatch_dens<NB, true, true>(dens, nfp, dmu, alpha, st, nc);
      return;
    }
    if (q) dispatch_dens<NB, false, true>(dens, nfp, dmu, alpha, st, nc);
    else dispatch_dens<NB, false, false>(dens, nfp, dmu, alpha, st, nc);
  }

  void run_eval(const double* w, size_t nc, const double* mu, int dens, double alpha, bool need_h, double* stats_host) {
    HIP_OK(hipSetDevice(device));
    const size_t total = EvalStats::size(nc, need_h);
    double* st = ensure(d_stats, cap_stats, total);
    double* direct = direct_acquire(total);
    if (direct) st = direct;
    HIP_OK(hipEventRecord(ev[0], stream));
    const int nb = pick_nb(nc);
    const int nfp = 16 * std::max(nb, 1);  // fused pass: K padded to 16·NB (host builds Wp accordingly)
    const bool fused = nb > 0 && nf <= (uint64_t)nfp && !(need_h && nb == 8) &&
                       !((dens == DENS_TANH || dens == DENS_EXP) && !(alpha > 0.0));
    const double* dmu = resident_mu(mu);  // null: X is centred in place
    const bool tiled = !fused && tiled_ok(nc, dens, alpha);
    if (tiled) {
      HIP_OK(hipEventRecord(ev[1], stream));
      tiled_eval(w, nc, dmu, dens, alpha, need_h, st, 0);
      HIP_OK(hipEventRecord(ev[2], stream));
    } else if (fused) {
      const int ncp = 16 * nb;
      const size_t nwp = (size_t)ncp * nfp;
      ensure(d_w, cap_w, nwp);
      double* wp = (double*)pin_acquire(pin_w_, nwp * sizeof(double));
      std::fill(wp, wp + nwp, 0.0);
      for (size_t i = 0; i < nc; ++i)
        for (size_t k = 0; k < nf; ++k) wp[i * nfp + k] = w[i * nf + k];
      wp_pending_ = wp;  // copied by launch_fused when the kernel it picks reads it
      wp_n_ = nwp;
      oz_fused_ready_ = false;
      if (dmu == nullptr && !need_h && dens != DENS_LINEAR && oz_any(nc) && ensure_xsl()) {
        upload_wsl(w, nc);
        oz_fused_ready_ = true;
      }
      try {
        switch (nb) {
          case 1: dispatch_h<1>(need_h, want_y2, dens, nfp, dmu, alpha, st, nc); break;
          case 2: dispatch_h<2>(need_h, want_y2, dens, nfp, dmu, alpha, st, nc); break;
          case 4: dispatch_h<4>(need_h, want_y2, dens, nfp, dmu, alpha, st, nc); break;
          default: dispatch_h<8>(need_h, want_y2, dens, nfp, dmu, alpha, st, nc); break;
        }
      } catch (...) {
        wp_pending_ = nullptr;
        throw;
      }
      wp_pending_ = nullptr;
      pin_release(pin_w_);  // (after the copy, if one was enqueued)
    } else {
      throw computation_error("no evaluation path for density id " + std::to_string(dens));
    }
    const double* staged = direct;
    if (direct) {
      pin_release(pin_direct_);
    } else {
      allreduce(st, total, need_h ? "eval+H" : "eval");
      staged = d2h_enqueue(st, total);
    }
    HIP_OK(hipEventRecord(ev[3], stream));
    sync();
    copy_out(stats_host, staged, total);
    float a = 0, b = 0;
    const bool timed = fused || tiled;  // "fused" kind = every full pass (fused or tiled)
    if (timed) { HIP_OK(hipEventElapsedTime(&a, ev[1], ev[2])); }
    HIP_OK(hipEventElapsedTime(&b, ev[0], ev[3]));
    last_kernel_ms = timed ? a : b;
    last_call_ms = b;
    if (timed) { sum_kernel_ms += a; ++n_kernel; }
    sum_call_ms += b;
  }

  // ---- non-ortho multi-try loss pass ---------------------------------------
  // ll_out / y2_out: [na][nc] (Σℓ, Σy² of Y + α_j·Z), summed over ranks
  template <int KS, int D>
  void multi2_launch(int ncp, const double* dw, const double* dz, const double* dmu, double alpha,
                     const double* dal, int na, int nwg, uint64_t bpw, uint64_t n_blocks, double* part) {
    const int nroles = (ncp / 16 + 3) / 4;
    const size_t lds = (size_t)(2 * 16 * 4 * KS + 2 * 2 * 4 * 2 * 4 * 64) * sizeof(double);
    auto k = want_y2 ? k_multi_loss2<KS, D, true> : k_multi_loss2<KS, D, false>;
    lds_attr((const void*)k, 160 * 1024 - EXP_TAB_BYTES);
    k<<<xcd_grid(nwg, nroles), FUSED_THREADS, lds, stream>>>(X, ldx, n_local_, (int)nf, ncp, dw, dz, dmu, alpha, dal, na,
                                                             bpw, n_blocks, part, (uint64_t)nwg);
  }
  template <int KSO, int D>
  void multi2_oz_launch(int ncp, double alpha, const double* dal, int na, int nwg, uint64_t bpw, uint64_t n_blocks,
                        double* part, bool f32 = false) {
    const int nroles = (ncp / 16 + 3) / 4;
    const size_t lds = (size_t)2 * (oz_block_bytes<KSO>() + 256) + (size_t)2 * 4 * 2 * 4 * 64 * sizeof(double);
    auto k = f32 && D == DENS_TANH ? k_multi_loss2_oz<KSO, DENS_TANH, false, true>
             : want_y2            ? k_multi_loss2_oz<KSO, D, true>
                                  : k_multi_loss2_oz<KSO, D, false>;
    lds_attr((const void*)k, (int)lds);
    k<<<xcd_grid(nwg, nroles), FUSED_THREADS, lds, stream>>>(d_xsl, d_xsc, d_wsl, d_wsc, ncp, alpha, dal, na, bpw,
                                                             n_blocks, part, (uint64_t)nwg);
  }
  template <int D>
  void multi2_oz_dispatch(int ncp, double alpha, const double* dal, int na, int nwg, uint64_t bpw, uint64_t n_blocks,
                          double* part, bool f32 = false) {
    switch (oz_kso()) {
      case 1: multi2_oz_launch<1, D>(ncp, alpha, dal, na, nwg, bpw, n_blocks, part, f32); break;
      case 2: multi2_oz_launch<2, D>(ncp, alpha, dal, na, nwg, bpw, n_blocks, part, f32); break;
      default: multi2_oz_launch<4, D>(ncp, alpha, dal, na, nwg, bpw, n_blocks, part, f32); break;
    }
  }
  // k_multi_loss2_ozy on k_multi_loss2_oz's partition (nwg, bpw): the same partials
  template <int KSO, int D>
  void multi2_ozy_launch(int ncp, double alpha, const double* dal, int na, int nwg, uint64_t bpw, uint64_t n_blocks,
                         double* part) {
    const int nroles = (ncp / 16 + 7) / 8;
    const size_t lds = (size_t)2 * (oz_block_bytes<KSO>() + 256);
    auto k = na <= 10 ? (want_y2 ? k_multi_loss2_ozy<KSO, D, true, 10> : k_multi_loss2_ozy<KSO, D, false, 10>)
                      : (want_y2 ? k_multi_loss2_ozy<KSO, D, true, ML_NA> : k_multi_loss2_ozy<KSO, D, false, ML_NA>);
    // unfenced try chains by default (1.4 % faster at C4, profiles/r06_g); PICARD_MULTI_FENCE=1 fences
    if (!multi_fence_ && na <= 10)
      k = want_y2 ? k_multi_loss2_ozy<KSO, D, true, 10, false> : k_multi_loss2_ozy<KSO, D, false, 10, false>;
    lds_attr((const void*)k, (int)lds);
    k<<<xcd_grid(nwg, nroles), FUSED_THREADS, lds, stream>>>(d_xsl, d_xsc, d_wsl, d_wsc, ncp, alpha, dal, na, ybuf_read_,
                                                             bpw, n_blocks, part, (uint64_t)nwg);
  }
  template <int D>
  void multi2_ozy_dispatch(int ncp, double alpha, const double* dal, int na, int nwg, uint64_t bpw, uint64_t n_blocks,
                           double* part) {
    switch (oz_kso()) {
      case 1: multi2_ozy_launch<1, D>(ncp, alpha, dal, na, nwg, bpw, n_blocks, part); break;
      case 2: multi2_ozy_launch<2, D>(ncp, alpha, dal, na, nwg, bpw, n_blocks, part); break;
      default: multi2_ozy_launch<4, D>(ncp, alpha, dal, na, nwg, bpw, n_blocks, part); break;
    }
  }
  template <int D>
  void multi2_dispatch(int ks, int ncp, const double* dw, const double* dz, const double* dmu, double alpha,
                       const double* dal, int na, int nwg, uint64_t bpw, uint64_t n_blocks, double* part) {
    switch (ks) {
      case 16: multi2_launch<16, D>(ncp, dw, dz, dmu, alpha, dal, na, nwg, bpw, n_blocks, part); break;
      case 32: multi2_launch<32, D>(ncp, dw, dz, dmu, alpha, dal, na, nwg, bpw, n_blocks, part); break;
      default: multi2_launch<64, D>(ncp, dw, dz, dmu, alpha, dal, na, nwg, bpw, n_blocks, part); break;
    }
  }

  void multi_loss(const double* w, const double* z, size_t nc, const double* mu, pc_density d, const double* alphas,
                  int na, double* ll_out, double* y2_out) {
    HIP_OK(hipSetDevice(device));
    const int ncp = (int)((nc + 31) / 32 * 32);
    const int ks = yw_ks(nf);  // nf ≤ 256: register-resident k_multi_loss2
    const int nfp = ks ? 4 * ks : (int)((nf + ML_KC - 1) / ML_KC * ML_KC);
    const size_t nwt = (size_t)2 * nfp * ncp + ML_NA;
    double* dw = ensure(d_w, cap_w, nwt);
    HIP_OK(hipEventRecord(ev[0], stream));
    // [Wᵀ | Zᵀ | α] for the fp64 kernels; the int8 kernels take W and Z from their digit images
    // and only need the α's
    auto upload_wt = [&](bool full) {
      std::vector<double> wt(full ? nwt : (size_t)ML_NA, 0.0);
      double* al = wt.data() + (full ? (size_t)2 * nfp * ncp : 0);
      if (full)
        for (size_t i = 0; i < nc; ++i)
          for (size_t k = 0; k < nf; ++k) {
            wt[k * ncp + i] = w[i * nf + k];
            wt[(size_t)nfp * ncp + k * ncp + i] = z[i * nf + k];
          }
      for (int j = 0; j < na; ++j) al[j] = alphas[j];
      HIP_OK(hipMemcpyAsync(full ? dw : dw + (size_t)2 * nfp * ncp, wt.data(), wt.size() * sizeof(double),
                            hipMemcpyHostToDevice, stream));
    };
    const double* dmu = resident_mu(mu);  // null: X is centred in place
    const size_t pst = (size_t)ML_NA * 2 * ncp;
    const double* dal = dw + (size_t)2 * nfp * ncp;
    if (!ks) upload_wt(true);
    if (ks) {
      const uint64_t n_blocks = std::max<uint64_t>((n_local_ + 15) / 16, 1);
      const int nroles = (ncp / 16 + 3) / 4;
      const int nwg = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)2 * n_cu / nroles, n_blocks));
      const uint64_t bpw = (n_blocks + nwg - 1) / nwg;
      double* part = ensure(d_part, cap_part, (size_t)nwg * pst);
      double* st0 = ensure(d_stats, cap_stats, (size_t)2 * na * nc);
      (void)st0;
      // Y and Z on the int8 digit stage (after the pass buffers: an allocation may release the image)
      bool oz = y_stage_ != 1 && dmu == nullptr && ensure_xsl();
      if (oz) upload_wsl2(w, z, nc);
      oz = oz && xsl_valid_;
      // Y of this W already in HBM (the full tiled pass before this search): read, not formed
      // (tanh at 256 features holds its tries' accumulators without spilling only without Σy² and
      // with ≤ 10 tries: otherwise k_multi_loss2_oz)
      const bool ozy_fits = !(oz_kso() == 4 && d.kind == DENS_TANH && (want_y2 || na > 10));
      const int yslot = !(oz && multi_ybuf_ && ozy_fits) ? -1 : ytile_match(0, w, nc) ? 0 : ytile_match(1, w, nc) ? 1 : -1;
      const bool ytile = yslot >= 0;
      ybuf_read_ = yslot == 1 ? d_ybuf2 : d_tbuf;
      upload_wt(!oz);
      HIP_OK(hipEventRecord(ev[1], stream));
      if (ytile) {
        switch (d.kind) {
          case DENS_TANH: multi2_ozy_dispatch<DENS_TANH>(ncp, d.alpha, dal, na, nwg, bpw, n_blocks, part); break;
          case DENS_EXP: multi2_ozy_dispatch<DENS_EXP>(ncp, d.alpha, dal, na, nwg, bpw, n_blocks, part); break;
          default: multi2_ozy_dispatch<DENS_CUBE>(ncp, d.alpha, dal, na, nwg, bpw, n_blocks, part); break;
        }
        ++n_int8_passes_;
        ++n_multi_ybuf_;
      } else if (oz) {
        switch (d.kind) {
          case DENS_TANH: multi2_oz_dispatch<DENS_TANH>(ncp, d.alpha, dal, na, nwg, bpw, n_blocks, part); break;
          case DENS_EXP: multi2_oz_dispatch<DENS_EXP>(ncp, d.alpha, dal, na, nwg, bpw, n_blocks, part); break;
          default: multi2_oz_dispatch<DENS_CUBE>(ncp, d.alpha, dal, na, nwg, bpw, n_blocks, part); break;
        }
        ++n_int8_passes_;
      } else
      switch (d.kind) {
        case DENS_TANH: multi2_dispatch<DENS_TANH>(ks, ncp, dw, dw + (size_t)nfp * ncp, dmu, d.alpha, dal, na, nwg, bpw, n_blocks, part); break;
        case DENS_EXP: multi2_dispatch<DENS_EXP>(ks, ncp, dw, dw + (size_t)nfp * ncp, dmu, d.alpha, dal, na, nwg, bpw, n_blocks, part); break;
        default: multi2_dispatch<DENS_CUBE>(ks, ncp, dw, dw + (size_t)nfp * ncp, dmu, d.alpha, dal, na, nwg, bpw, n_blocks, part); break;
      }
      HIP_OK(hipGetLastError());
      HIP_OK(hipEventRecord(ev[2], stream));
      double* st = ensure(d_stats, cap_stats, (size_t)2 * na * nc);
      k_reduce_rows<<<(2 * na * (int)nc + RED_OUT - 1) / RED_OUT, 256, 0, stream>>>(part, nwg, pst, 0, ncp, (int)nc, 2 * na, st,
                                                                          d.kind, d.alpha, (double)n_local_, -1);
      HIP_OK(hipGetLastError());
      multi_finish(st, nc, na, ll_out, y2_out);
      return;
    }
    const uint64_t n_tiles = (n_local_ + ML_TT - 1) / ML_TT;
    const int nwg = (int)std::min<uint64_t>((uint64_t)n_cu, std::max<uint64_t>(n_tiles, 1));
    const uint64_t tpw = (std::max<uint64_t>(n_tiles, 1) + nwg - 1) / nwg;
    double* part = ensure(d_part, cap_part, (size_t)nwg * pst);
    HIP_OK(hipMemsetAsync(part, 0, (size_t)nwg * pst * sizeof(double), stream));
    const size_t lds = (size_t)(2 * ML_KC * (256 + 16) + ML_KC * (ML_TT + 16) + 8 * ML_NA * 2 * 16 * 2) * sizeof(double);
    HIP_OK(hipEventRecord(ev[1], stream));
    switch (d.kind) {
      case DENS_TANH: k_multi_loss<DENS_TANH><<<nwg, FUSED_THREADS, lds, stream>>>(X, ldx, n_local_, (int)nf, nfp, ncp, dw, dw + (size_t)nfp * ncp, dmu, d.alpha, dal, na, tpw, n_tiles, part); break;
      case DENS_EXP: k_multi_loss<DENS_EXP><<<nwg, FUSED_THREADS, lds, stream>>>(X, ldx, n_local_, (int)nf, nfp, ncp, dw, dw + (size_t)nfp * ncp, dmu, d.alpha, dal, na, tpw, n_tiles, part); break;
      default: k_multi_loss<DENS_CUBE><<<nwg, FUSED_THREADS, lds, stream>>>(X, ldx, n_local_, (int)nf, nfp, ncp, dw, dw + (size_t)nfp * ncp, dmu, d.alpha, dal, na, tpw, n_tiles, part); break;
    }
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ev[2], stream));
    double* st = ensure(d_stats, cap_stats, (size_t)2 * na * nc);
    // st[(j·2 + c)·nc + row] = Σ_w part[w][(j·2 + c)·ncp + row]
    k_reduce_rows<<<(2 * na * (int)nc + RED_OUT - 1) / RED_OUT, 256, 0, stream>>>(part, nwg, pst, 0, ncp, (int)nc, 2 * na, st,
                                                                        -1, 0.0, 0.0, 0);
    HIP_OK(hipGetLastError());
    multi_finish(st, nc, na, ll_out, y2_out);
  }
  void multi_finish(double* st, size_t nc, int na, double* ll_out, double* y2_out) {
    allreduce(st, (size_t)2 * na * nc, "loss_multi");
    std::vector<double> h((size_t)2 * na * nc);
    const double* staged = d2h_enqueue(st, h.size());
    run_overlap();  // the caller's host work while the pass runs
    finish_timing(true, 3);
    copy_out(h.data(), staged, h.size());
    for (int j = 0; j < na; ++j) {
      std::memcpy(ll_out + (size_t)j * nc, h.data() + (size_t)(j * 2 + 0) * nc, nc * sizeof(double));
      std::memcpy(y2_out + (size_t)j * nc, h.data() + (size_t)(j * 2 + 1) * nc, nc * sizeof(double));
    }
  }
  // Non-ortho tries with fp32 row terms and a rigorous bound (Evaluator::eval_loss_multi_bound):
  // tanh without Σy², the int8 stage at nf ≤ 256. Per try j and row i, against the exact pass
  // at W + α_j·Z (whose y differs from Y + α_j·Z by fp64 rounding, inside the 1e-10 slack):
  //   |ỹ − y| ≤ 2^-24·(|Y| + α_j|Z|) (the fp32 conversions) + 2^-24·|ỹ| (the fp32 fma)
  //             + 3·2^-125 (subnormal results of the three roundings),
  //   Σ|ỹ| in fp32 per 4 samples: ≤ 2^-23·Σ|ỹ| (1.0001 covers the higher orders), ℓ Lipschitz 1,
  //   the log term: screen_f32_block_bound per 4 samples (the orthogonal screen's constants),
  // so bnd = 2^-24·1.0001·(ΣY + α_jΣZ) + 2^-22·1.0001·Σ|ỹ| + (ldx/4)·block + 3·2^-125·ldx
  //          + 1e-10·Σℓ. A rank whose scales leave the fp32 range (or that has no digit image)
  // runs the exact kernel into the same layout with zero bound terms: every rank issues the
  // same all-reduce, and each rank's share of the bound covers its own arithmetic.
  // On C4 the pass takes 31.7 ms instead of 41.2, but near convergence the tries differ by less
  // than the fp32 bound (≈ 1e-4 in loss units): used always, 28 of 128 searches paid a full pass
  // for a try the exact pass then rejected (whole fit 15.6 s against 15.0; profiles/r03_d/
  // c4_multi_bound.txt). Used only until the first such search (Solver::multi_bound_on_), the
  // fit took 15.30 s against 15.12 s exact (profiles/r04_b/c4_policy.txt): no gain either, so it
  // stays opt-in (PICARD_MULTI_F32=1).
  bool multi_f32_ = std::getenv("PICARD_MULTI_F32") && std::atoi(std::getenv("PICARD_MULTI_F32")) == 1;
  bool eval_loss_multi_bound(const double* w, const double* z, size_t nc, const double* mu, pc_density d,
                             const double* alphas, int na, double* ll_out, double* bnd_out) override {
    if (!multi_f32_ || !multi_loss_ok(nc, d) || d.kind != DENS_TANH || want_y2 || na > ML_NA || yw_ks(nf) == 0)
      return false;
    HIP_OK(hipSetDevice(device));
    const int ncp = (int)((nc + 31) / 32 * 32);
    std::vector<double> al(ML_NA, 0.0);
    for (int j = 0; j < na; ++j) al[j] = alphas[j];
    double* dal = ensure(d_w, cap_w, (size_t)ML_NA);
    HIP_OK(hipEventRecord(ev[0], stream));
    HIP_OK(hipMemcpyAsync(dal, al.data(), ML_NA * sizeof(double), hipMemcpyHostToDevice, stream));
    const double* dmu = resident_mu(mu);
    const size_t pst = (size_t)(ML_NA * 2 + 2) * ncp;
    const uint64_t n_blocks = std::max<uint64_t>((n_local_ + 15) / 16, 1);
    const int nroles = (ncp / 16 + 3) / 4;
    const int nwg = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)2 * n_cu / nroles, n_blocks));
    const uint64_t bpw = (n_blocks + nwg - 1) / nwg;
    double* part = ensure(d_part, cap_part, (size_t)nwg * pst);
    const size_t nst = (size_t)2 * na * nc + 3 * nc;  // [tries: Σℓ, Σ|ỹ|] [ΣY] [ΣZ] [constant bound]
    double* st = ensure(d_stats, cap_stats, nst);
    bool oz = y_stage_ != 1 && dmu == nullptr && ensure_xsl();
    if (oz) upload_wsl2(w, z, nc);
    oz = oz && xsl_valid_;
    // fp32 range: every |Y|, |Z| scale 2^(f_i + e_t − 20) in [2^-100, 2^98]
    bool f32 = oz && xsc_range_ok_;
    for (int m = 0; f32 && m < 2; ++m) {
      const double* a = m == 0 ? w : z;
      for (size_t i = 0; f32 && i < nc; ++i) {
        double mx = 0.0;
        for (size_t k = 0; k < nf; ++k) mx = std::max(mx, std::fabs(a[i * nf + k]));
        if (!(mx > 0.0)) continue;
        int e = 0;
        (void)std::frexp(mx, &e);
        if (e - 20 + xsc_emin_ < -100 || e - 20 + xsc_emax_ > 98) f32 = false;
      }
    }
    if (oz) {
      HIP_OK(hipEventRecord(ev[1], stream));
      multi2_oz_dispatch<DENS_TANH>(ncp, d.alpha, dal, na, nwg, bpw, n_blocks, part, f32);
      ++n_int8_passes_;
    } else {  // no digit image: the fp64 multi-try pass (exact sums, zero bound terms), same layout
      const int ks = yw_ks(nf), nfp = 4 * ks;
      std::vector<double> wt((size_t)2 * nfp * ncp + ML_NA, 0.0);
      for (size_t i = 0; i < nc; ++i)
        for (size_t k = 0; k < nf; ++k) {
          wt[k * ncp + i] = w[i * nf + k];
          wt[(size_t)nfp * ncp + k * ncp + i] = z[i * nf + k];
        }
      for (int j = 0; j < na; ++j) wt[(size_t)2 * nfp * ncp + j] = alphas[j];
      double* dw = ensure(d_w, cap_w, wt.size());
      HIP_OK(hipMemcpyAsync(dw, wt.data(), wt.size() * sizeof(double), hipMemcpyHostToDevice, stream));
      HIP_OK(hipEventRecord(ev[1], stream));
      multi2_dispatch<DENS_TANH>(ks, ncp, dw, dw + (size_t)nfp * ncp, dmu, d.alpha, dw + (size_t)2 * nfp * ncp, na,
                                 nwg, bpw, n_blocks, part);
      HIP_OK(hipStreamSynchronize(stream));  // wt is pageable and local
    }
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ev[2], stream));
    const size_t pstu = f32 ? pst : (size_t)ML_NA * 2 * ncp;
    k_reduce_rows<<<(2 * na * (int)nc + RED_OUT - 1) / RED_OUT, 256, 0, stream>>>(part, nwg, pstu, 0, ncp, (int)nc, 2 * na, st,
                                                                        DENS_TANH, d.alpha, (double)n_local_, -1);
    HIP_OK(hipGetLastError());
    if (f32) {
      k_reduce_rows<<<(2 * (int)nc + RED_OUT - 1) / RED_OUT, 256, 0, stream>>>(part, nwg, pst, (size_t)ML_NA * 2 * ncp,
                                                                         ncp, (int)nc, 2, st + (size_t)2 * na * nc,
                                                                         -1, 0.0, 0.0, 0);
      HIP_OK(hipGetLastError());
    } else {
      HIP_OK(hipMemsetAsync(st + (size_t)2 * na * nc, 0, 2 * nc * sizeof(double), stream));
    }
    double* cb = (double*)pin_acquire(pin_in_, nc * sizeof(double));
    const double cst = f32 ? (double)(ldx / 4) * screen_f32_block_bound(d.alpha) + 3.0 * 0x1p-125 * (double)ldx : 0.0;
    for (size_t i = 0; i < nc; ++i) cb[i] = cst;
    HIP_OK(hipMemcpyAsync(st + (size_t)2 * na * nc + 2 * nc, cb, nc * sizeof(double), hipMemcpyHostToDevice, stream));
    pin_release(pin_in_);
    allreduce(st, nst, "loss_multi_bound");
    std::vector<double> h(nst);
    const double* staged = d2h_enqueue(st, nst);
    finish_timing(true, 3);
    copy_out(h.data(), staged, nst);
    const double* sy = h.data() + (size_t)2 * na * nc;
    const double* sz = sy + nc;
    const double* sc = sz + nc;
    for (int j = 0; j < na; ++j)
      for (size_t i = 0; i < nc; ++i) {
        const double l = h[((size_t)j * 2 + 0) * nc + i], ya = h[((size_t)j * 2 + 1) * nc + i];
        ll_out[(size_t)j * nc + i] = l;
        bnd_out[(size_t)j * nc + i] = 0x1p-24 * 1.0001 * (sy[i] + std::fabs(alphas[j]) * sz[i]) +
                                      0x1p-22 * 1.0001 * std::fabs(ya) + sc[i] + 1e-10 * std::fabs(l);
      }
    return true;
  }
  bool multi_loss_ok(size_t nc, pc_density d) const {
    return nc <= 256 && (d.kind == DENS_TANH || d.kind == DENS_EXP || d.kind == DENS_CUBE) &&
           (d.kind == DENS_CUBE || d.alpha > 0.0) && std::getenv("PICARD_NO_MULTI") == nullptr;
  }
  bool eval_loss_multi(const double* w, const double* z, size_t nc, const double* mu, pc_density d,
                       const double* alphas, int na, double* ll_out, double* y2_out) override {
    if (!multi_loss_ok(nc, d)) return false;
    for (int j0 = 0; j0 < na; j0 += ML_NA) {
      const int nj = std::min(ML_NA, na - j0);
      multi_loss(w, z, nc, mu, d, alphas + j0, nj, ll_out + (size_t)j0 * nc, y2_out + (size_t)j0 * nc);
    }
    return true;
  }

  // ---- tiled two-phase path ----------------------------------------------
  double* d_tbuf = nullptr; size_t cap_tbuf = 0;   // y, ψ, ψ′ fragments of one T chunk
  // Y of the whole shard left in HBM by a full tiled pass on the int8 stage (one T chunk): valid
  // for W = YTile::w (nc rows) and the digit image of generation YTile::gen; the multi-try pass
  // at that W reads it instead of forming Y again (k_multi_loss2_ozy).
  // PICARD_MULTI_YBUF=0 (A/B knob) forms Y in every multi-try pass.
  // Two slots: slot 0 is the y region of d_tbuf, slot 1 a second buffer (d_ybuf2, allocated when
  // HBM has room) — a full pass at a new W writes the slot the last one did not, so the W of a
  // search keeps its Y through a rejected try-1 full pass at another W.
  struct YTile {
    bool valid = false;
    size_t nc = 0;
    uint64_t gen = 0;
    std::vector<double> w;
  };
  YTile ytile_[2];
  int ytile_last_ = 0;          // the slot the last full tiled pass wrote
  double* ytarget_ = nullptr;   // where the current tiled pass writes its y fragments
  double* d_ybuf2 = nullptr;
  size_t cap_ybuf2 = 0;
  bool ybuf2_failed_ = false;
  bool ytile_match(int s, const double* w, size_t nc) const {
    const YTile& y = ytile_[s];
    return y.valid && y.nc == nc && y.gen == xsl_gen_ && y.w.size() == nc * nf &&
           std::memcmp(y.w.data(), w, nc * nf * sizeof(double)) == 0;
  }
  // the second y buffer: only with ≥ 16 GB left beside it, and never at the digit image's expense
  bool ensure_ybuf2(size_t n) {
    if (n <= cap_ybuf2) return true;
    if (ybuf2_failed_) return false;
    size_t fr = 0, tot = 0;
    HIP_OK(t_meminfo(&fr, &tot));
    if (d_ybuf2) {
      HIP_OK(t_free(d_ybuf2));
      fr += cap_ybuf2 * sizeof(double);
      d_ybuf2 = nullptr;
      cap_ybuf2 = 0;
      ytile_[1].valid = false;
    }
    if (n * sizeof(double) + (size_t(16) << 30) > fr || t_malloc((void**)&d_ybuf2, n * sizeof(double)) != hipSuccess) {
      (void)hipGetLastError();
      d_ybuf2 = nullptr;
      ybuf2_failed_ = true;
      return false;
    }
    cap_ybuf2 = n;
    return true;
  }
  uint64_t n_multi_ybuf_ = 0;
  const double* ybuf_read_ = nullptr;  // the slot the current multi-try pass reads
  const bool multi_ybuf_ = !(std::getenv("PICARD_MULTI_YBUF") && std::atoi(std::getenv("PICARD_MULTI_YBUF")) == 0);
  const bool multi_fence_ = std::getenv("PICARD_MULTI_FENCE") && std::atoi(std::getenv("PICARD_MULTI_FENCE")) == 1;
  const int gram_sbb_ = std::getenv("PICARD_GRAM_SBB") && std::atoi(std::getenv("PICARD_GRAM_SBB")) == 1 ? 1 : 2;
  double* d_slab = nullptr; size_t cap_slab = 0;
  double* d_trow = nullptr; size_t cap_trow = 0;
  double tiled_budget_ = 0;  // bytes the fragment buffers may take (set on first use)
  static bool tiled_ok(size_t nc, int dens, double alpha) {
    (void)nc;
    (void)alpha;
    return dens <= DENS_LINEAR;  // any shape; tanh/exp at α ≤ 0 through the libm forms
  }
  // the density id the tiled kernels run: the libm forms for tanh/exp unless α > 0
  static int tiled_dens(int dens, double alpha) {
    if (dens == DENS_TANH && !(alpha > 0.0)) return DENS_TANH_S;
    if (dens == DENS_EXP && !(alpha > 0.0)) return DENS_EXP_S;
    return dens;
  }
  // K steps per MFMA chain of phase 1 (one chunk of ≤ 256 features)
  static int yw_ks(uint64_t nf) { return nf <= 64 ? 16 : nf <= 128 ? 32 : 64; }
  template <int KS, int D>
  void yw_launch_ks(int mode, int ncp, double alpha, uint64_t ntl, int nwg1, bool acc, const double* X0,
                    uint64_t nrows, const double* wpt, double* yb, double* pb, double* db, const double* yin) {
    const uint64_t n_blocks = ntl * 4;  // whole 64-sample tiles: phase 2 reads every sub-block
    const uint64_t bpw = (n_blocks + nwg1 - 1) / nwg1;
    const int nroles = (ncp / 16 + 7) / 8;
    const size_t lds = (size_t)2 * 16 * 4 * KS * sizeof(double);
    // partial y of earlier feature chunks (yin) only exists above 4·KS = 256 features
    constexpr bool YC = KS == 64;
    auto k = yin && YC ? (mode == 0 ? k_tiled_yw<KS, D, 0, YC> : mode == 1 ? k_tiled_yw<KS, D, 1, YC> : k_tiled_yw<KS, D, 2, YC>)
                       : (mode == 0 ? k_tiled_yw<KS, D, 0, false> : mode == 1 ? k_tiled_yw<KS, D, 1, false>
                                                                             : k_tiled_yw<KS, D, 2, false>);
    if (yin && !YC) throw computation_error("tiled pass: feature chunks need KS = 64");
    lds_attr((const void*)k, 160 * 1024 - EXP_TAB_BYTES);
    k<<<xcd_grid(nwg1, nroles), FUSED_THREADS, lds, stream>>>(X0, ldx, 0, (int)nrows, ncp, wpt, nullptr, alpha, bpw,
                                                              n_blocks, d_trow, acc ? 1 : 0, yb, pb, db, yin,
                                                              (uint64_t)nwg1);
  }
  template <int D>
  void yw_launch(int ks, int mode, int ncp, double alpha, uint64_t ntl, int nwg1, bool acc, const double* X0,
                 uint64_t nrows, const double* wpt, double* yb, double* pb, double* db, const double* yin) {
    switch (ks) {
      case 16: yw_launch_ks<16, D>(mode, ncp, alpha, ntl, nwg1, acc, X0, nrows, wpt, yb, pb, db, yin); break;
      case 32: yw_launch_ks<32, D>(mode, ncp, alpha, ntl, nwg1, acc, X0, nrows, wpt, yb, pb, db, yin); break;
      default: yw_launch_ks<64, D>(mode, ncp, alpha, ntl, nwg1, acc, X0, nrows, wpt, yb, pb, db, yin); break;
    }
  }
  // one T chunk: phase 1 over the feature chunks (partial y through the y
  // buffer), then phase 2 (mode 0)
  // phase 1 on the int8 digit stage: one launch over the T chunk starting at tile t0
  template <int KSO, int D>
  void yw_oz_launch(int mode, int ncp, double alpha, uint64_t ntl, int nwg1, bool acc, uint64_t t0, double* yb,
                    double* pb, double* db) {
    const uint64_t n_blocks = ntl * 4;
    const uint64_t bpw = (n_blocks + nwg1 - 1) / nwg1;
    const int nroles = (ncp / 16 + 7) / 8;
    const size_t lds = (size_t)2 * (oz_block_bytes<KSO>() + 256);
    auto k = mode == 0 ? k_tiled_yw_oz<KSO, D, 0> : k_tiled_yw_oz<KSO, D, 1>;
    lds_attr((const void*)k, (int)lds);
    k<<<xcd_grid(nwg1, nroles), FUSED_THREADS, lds, stream>>>(d_xsl + t0 * 4 * oz_block_bytes<KSO>(), d_xsc + t0 * TL_TT,
                                                              d_wsl, d_wsc, ncp, alpha, bpw, n_blocks, d_trow,
                                                              acc ? 1 : 0, yb, pb, db, (uint64_t)nwg1);
  }
  template <int D>
  void tiled_launch(int mode, int ks, int ncp, double alpha, uint64_t ntl, bool need_h, int nsplit, int nwg1, bool acc,
                    const double* X0, bool oz, uint64_t t0) {
    const size_t chunk = (size_t)ncp * ntl * TL_TT;
    constexpr bool dfromp = D == DENS_TANH;  // ψ′ = α(1 − ψ²) formed in phase 2
    double* yb = ytarget_ ? ytarget_ : d_tbuf;
    double* pb = d_tbuf + chunk;
    double* db = need_h && !dfromp ? d_tbuf + 2 * chunk : nullptr;
    const uint64_t kc = 4 * (uint64_t)ks;  // features per chunk
    if constexpr (D != DENS_LINEAR) {
      if (oz) {  // all features in one launch (nf ≤ 256)
        if (oz_kso() == 4) yw_oz_launch<4, D>(mode, ncp, alpha, ntl, nwg1, acc, t0, yb, pb, db);
        else if (oz_kso() == 2) yw_oz_launch<2, D>(mode, ncp, alpha, ntl, nwg1, acc, t0, yb, pb, db);
        else yw_oz_launch<1, D>(mode, ncp, alpha, ntl, nwg1, acc, t0, yb, pb, db);
        HIP_OK(hipGetLastError());
        ++n_int8_passes_;
      }
    }
    for (uint64_t k0 = 0; k0 < nf && !oz; k0 += kc) {
      const bool last = k0 + kc >= nf;
      yw_launch<D>(ks, last ? mode : 2, ncp, alpha, ntl, nwg1, acc, X0 + k0 * ldx, std::min<uint64_t>(kc, nf - k0),
                   d_w + k0 * ncp, yb, pb, db, k0 > 0 ? yb : nullptr);
      HIP_OK(hipGetLastError());
    }
    if (mode == 0) {
      const int nto = (ncp / 16 + 7) / 8;
      const uint64_t tps = (ntl + nsplit - 1) / nsplit;
      const size_t lds2 = (size_t)2 * (db ? 3 : 2) * 8 * 256 * sizeof(double);
      // two sub-blocks per barrier (PICARD_GRAM_SBB=1: one) where both buffers fit the LDS
      const int sbb = gram_sbb_ == 1 || (size_t)2 * lds2 > 160 * 1024 ? 1 : 2;
      auto k2 = sbb == 1 ? (!need_h ? k_tiled_gram2<false, false, 1>
                            : dfromp ? k_tiled_gram2<true, true, 1> : k_tiled_gram2<true, false, 1>)
                         : (!need_h ? k_tiled_gram2<false, false, 2>
                            : dfromp ? k_tiled_gram2<true, true, 2> : k_tiled_gram2<true, false, 2>);
      lds_attr((const void*)k2, 160 * 1024);
      k2<<<xcd_grid(nsplit, nto * nto), FUSED_THREADS, lds2 * sbb, stream>>>(yb, pb, db, ncp, ntl, tps, d_slab,
                                                                             acc ? 1 : 0, alpha, (uint64_t)nsplit);
      HIP_OK(hipGetLastError());
    }
  }
  // mode 0: all stats; mode 1: Σℓ, Σy² only (loss-only try; the completion recomputes)
  void tiled_eval(const double* w, size_t nc, const double* dmu, int dens, double alpha, bool need_h, double* st,
                  int mode) {
    if (dmu) throw computation_error("tiled pass expects the centred resident X");
    const int ncp = (int)((nc + 31) / 32 * 32);
    const int ks = yw_ks(nf);
    const uint64_t kc = 4 * (uint64_t)ks, nfp = (nf + kc - 1) / kc * kc;
    ensure(d_w, cap_w, (size_t)nfp * ncp);  // Wᵀ for the fp64 phase 1 (uploaded below)
    const uint64_t n_tiles = (n_local_ + TL_TT - 1) / TL_TT;
    // T chunks bound the fragment buffers (3 arrays of ncp × chunk) by what HBM
    // has free next to X (at least 24 GB): C4 (256 × 1e7, 61 GB) is one chunk
    if (tiled_budget_ == 0) {
      size_t fr = 0, tot = 0;
      HIP_OK(t_meminfo(&fr, &tot));
      const double have = (double)fr + (double)cap_tbuf * sizeof(double) - 16e9;
      tiled_budget_ = std::max(24e9, std::min(have, 0.6 * (double)tot));
      // PICARD_TILED_CHUNK_MB (measurement knob): T chunks whose y/ψ fragments fit that many MiB
      // (e.g. the 256 MiB Infinity Cache, so phase 2 reads them from MALL instead of HBM)
      if (const char* e = std::getenv("PICARD_TILED_CHUNK_MB"))
        if (std::atof(e) > 0) tiled_budget_ = std::atof(e) * 1048576.0;
    }
    const double narr = need_h && tiled_dens(dens, alpha) != DENS_TANH ? 3.0 : 2.0;  // y, ψ (, ψ′)
    const uint64_t max_tiles =
        std::max<uint64_t>(1, (uint64_t)(tiled_budget_ / (narr * ncp * TL_TT * sizeof(double))));
    const uint64_t ct = std::min<uint64_t>(std::max<uint64_t>(n_tiles, 1), max_tiles);
    const int nroles = (ncp / 16 + 7) / 8;
    const int nwg1 = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)n_cu * 2 / nroles, ct * 4));
    const int nto = (ncp / 16 + 7) / 8;
    const int nsplit = (int)std::max<uint64_t>(1, std::min<uint64_t>(ct, (uint64_t)(2 * n_cu / (nto * nto))));
    // y buffer: always in mode 0; in mode 1 only to carry partial y across feature chunks
    // reallocation is detected by the capacity, not the address: the allocator may hand the
    // freed buffer's address straight back, and the kept Y in it is gone either way
    const size_t tcap0 = cap_tbuf;
    if (mode == 0) ensure(d_tbuf, cap_tbuf, (size_t)narr * ncp * ct * TL_TT);
    else if (nf > kc) ensure(d_tbuf, cap_tbuf, (size_t)ncp * ct * TL_TT);
    if (cap_tbuf != tcap0) ytile_[0].valid = false;  // reallocated
    if (mode == 0) ensure(d_slab, cap_slab, (size_t)nsplit * (need_h ? 2 : 1) * ncp * ncp);
    ensure(d_trow, cap_trow, (size_t)nwg1 * 3 * ncp);
    const int td = tiled_dens(dens, alpha);
    // phase 1 on the int8 digit stage (nf ≤ 256; not the whitening Gram), after every buffer
    // of the pass is allocated (an allocation may release an unpinned image)
    bool oz = y_stage_ != 1 && nf <= 256 && td != DENS_LINEAR && ensure_xsl();
    if (oz) upload_wsl(w, nc);
    oz = oz && xsl_valid_;
    // the slot of this pass's y fragments (mode 1 writes y only as feature-chunk partials: slot 0)
    const bool single = ct >= std::max<uint64_t>(n_tiles, 1);
    int slot = 0;
    if (mode == 0 && oz && single && multi_ybuf_) {
      if (ytile_match(0, w, nc)) slot = 0;
      else if (ytile_match(1, w, nc)) slot = 1;
      else slot = ytile_last_ ^ 1;
      if (slot == 1 && !ensure_ybuf2((size_t)ncp * ct * TL_TT)) slot = 0;
    }
    if (mode == 0 || nf > kc) ytile_[slot].valid = false;  // this pass writes those y fragments
    ytarget_ = slot == 1 ? d_ybuf2 : d_tbuf;
    if (!oz) {  // Wᵀ, zero-padded to whole feature chunks (the int8 phase 1 reads W's digit image)
      std::vector<double> wt((size_t)nfp * ncp, 0.0);
      for (size_t i = 0; i < nc; ++i)
        for (size_t k = 0; k < nf; ++k) wt[k * ncp + i] = w[i * nf + k];
      HIP_OK(hipMemcpyAsync(d_w, wt.data(), wt.size() * sizeof(double), hipMemcpyHostToDevice, stream));
    }
    for (uint64_t t0 = 0; t0 < std::max<uint64_t>(n_tiles, 1); t0 += ct) {
      const uint64_t ntl = std::min<uint64_t>(ct, std::max<uint64_t>(n_tiles, 1) - t0);
      const bool acc = t0 > 0;
      const double* X0 = X + t0 * TL_TT;
      switch (td) {
        case DENS_TANH: tiled_launch<DENS_TANH>(mode, ks, ncp, alpha, ntl, need_h, nsplit, nwg1, acc, X0, oz, t0); break;
        case DENS_EXP: tiled_launch<DENS_EXP>(mode, ks, ncp, alpha, ntl, need_h, nsplit, nwg1, acc, X0, oz, t0); break;
        case DENS_CUBE: tiled_launch<DENS_CUBE>(mode, ks, ncp, alpha, ntl, need_h, nsplit, nwg1, acc, X0, oz, t0); break;
        case DENS_TANH_S: tiled_launch<DENS_TANH_S>(mode, ks, ncp, alpha, ntl, need_h, nsplit, nwg1, acc, X0, oz, t0); break;
        case DENS_EXP_S: tiled_launch<DENS_EXP_S>(mode, ks, ncp, alpha, ntl, need_h, nsplit, nwg1, acc, X0, oz, t0); break;
        default: tiled_launch<DENS_LINEAR>(mode, ks, ncp, alpha, ntl, need_h, nsplit, nwg1, acc, X0, false, t0); break;
      }
    }
    ytarget_ = nullptr;
    if (mode == 0 && oz && single) {  // one chunk: all of Y stays
      YTile& y = ytile_[slot];
      y.valid = true;
      y.nc = nc;
      y.gen = xsl_gen_;
      y.w.assign(w, w + nc * nf);
      ytile_last_ = slot;
    }
    const size_t total = (size_t)(mode == 0 ? (need_h ? 2 : 1) * nc * nc : 0) + 3 * nc;
    k_reduce_tiled<<<(total + 255) / 256, 256, 0, stream>>>(d_slab, nsplit, d_trow, nwg1, ncp, (int)nc, need_h,
                                                            mode == 1 ? 1 : 0, st, td, alpha, (double)n_local_);
    HIP_OK(hipGetLastError());
  }

  // ---- split line-search evaluation -------------------------------------
  bool fused_ok(size_t nc, int dens, double alpha, bool need_h) const {
    const int nb = pick_nb(nc);
    return nb > 0 && nf <= (uint64_t)(16 * nb) && !(need_h && nb == 8) &&
           !((dens == DENS_TANH || dens == DENS_EXP) && !(alpha > 0.0)) && dens != DENS_LINEAR;
  }
  // d_ybuf sized for Y of this shard in fragment order; false if HBM is short
  bool ensure_ybuf(int nb) {
    const int tb = 16 * (8 / nb);
    const uint64_t nblk = (n_local_ + tb - 1) / tb;
    const size_t need = (size_t)nblk * 16 * nb * tb;
    if (need <= cap_ybuf) return true;
    if (ybuf_failed) return false;
    size_t fr = 0, tot = 0;
    HIP_OK(t_meminfo(&fr, &tot));
    if (d_ybuf) { HIP_OK(t_free(d_ybuf)); fr += cap_ybuf * sizeof(double); d_ybuf = nullptr; cap_ybuf = 0; }
    if (need * sizeof(double) + (size_t(2) << 30) > fr || t_malloc((void**)&d_ybuf, need * sizeof(double)) != hipSuccess) {
      (void)hipGetLastError();
      d_ybuf = nullptr;
      ybuf_failed = true;
      return false;
    }
    cap_ybuf = need;
    return true;
  }

  // ---- int8-slice Y stage (ozaki.inc) ---------------------------------------
  // The slice image of the centred resident X is built once per resident μ
  // (k_slice_x) and dropped whenever X changes (alloc_x, shift_rows). y_stage_
  // = PC_YSTAGE_F64 keeps every pass on the fp64 MFMA Y stage.
  uint8_t* d_xsl = nullptr;
  double* d_xsc = nullptr;
  size_t cap_xsl = 0;
  bool xsl_valid_ = false, xsl_failed_ = false;
  uint64_t xsl_gen_ = 0;  // digit images built so far (k_slice_x launches)
  uint8_t* d_wsl = nullptr;
  double* d_wsc = nullptr;
  int y_stage_ = 0;
  uint64_t n_int8_passes_ = 0;
  // G = ψ·Yᵀ on int8 digits (fused_g8.inc, fused_g8x.inc): g_stage_ 0 = where the shape allows
  // (default), 1 = the fp64 G stage (PICARD_G8=0 or pc_ctx_set_g_stage(1)); the y-row scales in
  // d_wsc[256 …] are valid for the W image and the digit image whose largest sample exponent is
  // g8_emax_
  int g_stage_ = (std::getenv("PICARD_G8") && std::atoi(std::getenv("PICARD_G8")) == 0) ? 1 : 0;
  bool g8_scales_ok_ = false;

  int g8_emax_ = INT_MIN;
  uint64_t n_g8_passes_ = 0;
  bool d_wsl_ready_ = false, oz_fused_ready_ = false;
  void drop_xsl() { xsl_valid_ = false; }
  // free the slice image for good (until the next load / generate): the fp64 Y stage
  // serves every pass from then on
  void release_xsl() {
    if (d_xsl) { HIP_OK(hipStreamSynchronize(stream)); (void)t_free(d_xsl); (void)t_free(d_xsc); }
    d_xsl = nullptr; d_xsc = nullptr; cap_xsl = 0;
    if (d_xsf) { (void)t_free(d_xsf); d_xsf = nullptr; }
    cap_xsf_ = 0;
    xsf_e0_ = INT_MIN;
    xsl_valid_ = false;
    xsl_failed_ = true;
  }
  // fp32 sample scales 2^(e_t − E0) of the digit image for k_screen_oz2 (screen.hip), built
  // on first use per image (E0 = the image's largest exponent); xsf_e0_ = INT_MIN: not built
  float* d_xsf = nullptr;
  size_t cap_xsf_ = 0;
  int xsf_e0_ = INT_MIN;
  // false when the second screen cannot run here (the caller uses k_screen_oz)
  bool ensure_xsf() {
    if (!xsc_range_ok_ || xsc_emax_ - xsc_emin_ > 100) return false;  // u = y'·2^(e_t − E0) stays normal
    if (xsf_e0_ == xsc_emax_ && d_xsf) return true;
    if (cap_xsf_ < ldx) {
      if (d_xsf) (void)t_free(d_xsf);
      d_xsf = nullptr;
      cap_xsf_ = 0;
      if (t_malloc((void**)&d_xsf, ldx * sizeof(float)) != hipSuccess) {
        (void)hipGetLastError();
        d_xsf = nullptr;
        return false;
      }
      cap_xsf_ = ldx;
    }
    HIP_OK(screen2_build_xsf(d_xsc, ldx, xsc_emax_, d_xsf, stream));
    xsf_e0_ = xsc_emax_;
    return true;
  }
  // the shapes the i8 loss kernel covers: 64 < nc ≤ 128, nf ≤ 128, centred X
  bool oz_shape(size_t nc) const { return y_stage_ != 1 && pick_nb(nc) == 8 && nf <= 128 && nf > 0; }
  // … and the NB = 4 forms: 32 < nc ≤ 64 with nf ≤ 64 (a 1-k-step image)
  bool oz4_shape(size_t nc) const { return y_stage_ != 1 && pick_nb(nc) == 4 && nf <= 64 && nf > 0; }
  bool oz_any(size_t nc) const { return oz_shape(nc) || oz4_shape(nc); }
  // k-steps of 64 features of the resident X's digit image (nf ≤ 256)
  int oz_kso() const { return nf <= 64 ? 1 : nf <= 128 ? 2 : 4; }
  size_t oz_bb() const { return (size_t)oz_kso() * OZ_SLICES * 1024; }
  int wsl_ksw() const { return oz_kso() == 4 ? 4 : 2; }  // k-step stride of the W digit image
  bool ensure_xsl() {
    if (xsl_valid_) return true;
    if (xsl_failed_ || nf > 256) return false;
    // the scratch of the Σ 2^e_t sum first: an allocation here may release the image
    const int nwg_e = (int)std::max<uint64_t>(1, std::min<uint64_t>((ldx + 4095) / 4096, 1024));
    ensure(d_shift_part, cap_shift_part, std::max<size_t>((size_t)nwg_e + 1, 4 * (size_t)std::min(nwg_e, 256)));
    if (xsl_failed_) return false;
    const uint64_t n_blocks = ldx / 16;
    const size_t need = (size_t)n_blocks * oz_bb();
    if (need > cap_xsl) {
      size_t fr = 0, tot = 0;
      HIP_OK(t_meminfo(&fr, &tot));
      if (d_xsl) { HIP_OK(t_free(d_xsl)); HIP_OK(t_free(d_xsc)); fr += cap_xsl + ldx * sizeof(double); }
      d_xsl = nullptr; d_xsc = nullptr; cap_xsl = 0;
      // keep ≥ 4 GB free next to X for the pass buffers; otherwise stay on fp64
      if (need + ldx * sizeof(double) + (size_t(4) << 30) > fr || t_malloc((void**)&d_xsl, need) != hipSuccess ||
          t_malloc((void**)&d_xsc, ldx * sizeof(double)) != hipSuccess) {
        (void)hipGetLastError();
        if (d_xsl) (void)t_free(d_xsl);
        d_xsl = nullptr; d_xsc = nullptr;
        xsl_failed_ = true;
        return false;
      }
      cap_xsl = need;
    }
    xsf_e0_ = INT_MIN;  // the fp32 scales follow the image
    const unsigned grid = (unsigned)std::min<uint64_t>(n_blocks, (uint64_t)n_cu * 16);
    if (oz_kso() == 1) k_slice_x<1><<<grid, 64, 0, stream>>>(X, ldx, (int)nf, n_blocks, d_xsl, d_xsc);
    else if (oz_kso() == 2) k_slice_x<2><<<grid, 128, 0, stream>>>(X, ldx, (int)nf, n_blocks, d_xsl, d_xsc);
    else k_slice_x<4><<<grid, 256, 0, stream>>>(X, ldx, (int)nf, n_blocks, d_xsl, d_xsc);
    HIP_OK(hipGetLastError());
    ++xsl_gen_;
    {  // Σ_t 2^e_t of this shard (padding included: it only loosens the screen's bound)
      const int nwg = nwg_e;
      const uint64_t per = ((ldx + nwg - 1) / nwg + 511) / 512 * 512;
      double* part = d_shift_part;
      k_rowsum<<<dim3((unsigned)((ldx + per - 1) / per), 1), 256, 0, stream>>>(d_xsc, ldx, ldx, 1, per, part);
      HIP_OK(hipGetLastError());
      k_sum_slabs<<<1, 256, 0, stream>>>(part, (int)((ldx + per - 1) / per), 1, part + nwg);
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemcpyAsync(&xsc_sum_, part + nwg, sizeof(double), hipMemcpyDeviceToHost, stream));
      sync();
      // min / max of 2^e_t (part is free again: NaN scales make the range unusable)
      const int nr = (int)std::min<uint64_t>(nwg, 256);
      k_xsc_range<<<nr, 256, 0, stream>>>(d_xsc, ldx, part);
      HIP_OK(hipGetLastError());
      std::vector<double> mm(4 * (size_t)nr);
      HIP_OK(hipMemcpyAsync(mm.data(), part, mm.size() * sizeof(double), hipMemcpyDeviceToHost, stream));
      sync();
      double lo = INFINITY, hi = 0.0, sq = 0.0;
      bool nan = false;
      for (int b = 0; b < nr; ++b) {
        lo = std::min(lo, mm[4 * b]);
        hi = std::max(hi, mm[4 * b + 1]);
        nan |= mm[4 * b + 2] != 0.0;
        sq += mm[4 * b + 3];
      }
      // Σ_t 4^e_t (padding included), an upper bound: each fp64 sum of positive terms errs by
      // far less than 1e-9 relative (≤ 4096 sequential terms per thread, then trees)
      xsc_s4_ = sq * (1.0 + 1e-9);
      xg_valid_ = false;  // the digit Grams follow the image
      xsc_range_ok_ = !nan && lo > 0.0 && std::isfinite(hi);
      if (xsc_range_ok_) {
        (void)std::frexp(lo, &xsc_emin_);
        (void)std::frexp(hi, &xsc_emax_);
        xsc_emin_ -= 1;  // 2^e = 0.5·2^(e+1): frexp gives e + 1
        xsc_emax_ -= 1;
      }
    }
    xsl_valid_ = true;
    return true;
  }
  double xsc_sum_ = 0.0;
  // The line-search screen's statistical bound (screen_rank_bound): per digit plane b an upper
  // bound λ_b on the largest eigenvalue of this shard's digit Gram D_b = Σ_t d_b,t·d_b,tᵀ
  // (Gershgorin on the exact integer matrix), and S4 = Σ_t 4^e_t. Valid with the image.
  double xsc_s4_ = 0.0;
  double xg_lam_[OZ_SLICES] = {};
  bool xg_valid_ = false, xg_failed_ = false;
  uint64_t n_digit_gram_ = 0;
  bool ensure_digit_gram() {
    if (xg_valid_) return true;
    if (xg_failed_ || !xsl_valid_ || !d_xsl || oz_kso() > 2 || !xsc_range_ok_) return false;
    const int kso = oz_kso(), fpl = 4 * kso, np = fpl * (fpl + 1) / 2;
    const uint64_t n_blocks = ldx / 16, n_chunks = (n_blocks + 3) / 4;
    const uint64_t want = std::max<uint64_t>(1, (uint64_t)n_cu);
    const uint32_t per = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(DG_MAX_CHUNKS, (n_chunks + want - 1) / want));
    const int nwg = (int)std::max<uint64_t>(1, (n_chunks + per - 1) / per);
    const size_t n_out = (size_t)OZ_SLICES * np * 256;
    int* part = nullptr;
    double* red = nullptr;
    if (t_malloc((void**)&part, (size_t)nwg * n_out * sizeof(int)) != hipSuccess ||
        t_malloc((void**)&red, n_out * sizeof(double)) != hipSuccess) {
      (void)hipGetLastError();
      if (part) (void)t_free(part);
      xg_failed_ = true;  // the screen keeps its worst-case bound
      return false;
    }
    if (kso == 2) k_digit_gram<2><<<nwg, 512, 0, stream>>>(d_xsl, n_blocks, per, part);
    else k_digit_gram<1><<<nwg, 512, 0, stream>>>(d_xsl, n_blocks, per, part);
    HIP_OK(hipGetLastError());
    k_sum_islabs<<<(unsigned)((n_out + 255) / 256), 256, 0, stream>>>(part, nwg, n_out, red);
    HIP_OK(hipGetLastError());
    std::vector<double> g(n_out);
    HIP_OK(hipMemcpyAsync(g.data(), red, n_out * sizeof(double), hipMemcpyDeviceToHost, stream));
    sync();
    HIP_OK(t_free(part));
    HIP_OK(t_free(red));
    ++n_digit_gram_;
    // Gershgorin: λmax(D_b) ≤ max_f Σ_g |D_b[f][g]|. Tile pair (t1, t2), lane l, reg r holds
    // D_b[fpl·i + t1][fpl·j + t2] with i = 4·(l >> 4) + r, j = l & 15 (and its mirror if t1 ≠ t2)
    // (An eigenbasis bound — Ostrowski on the approximate eigenvectors — is ≈ 1.2× tighter on the
    // noise planes and ≈ 1.8× on plane 0, ≈ 18 % off the C3 D ≤ 2 bound; its host eigh costs
    // 2–15 ms per plane once per image, which a C2 fit of 25 ms cannot afford: not used.)
    std::vector<double> rs(fpl * 16);
    for (int b = 0; b < OZ_SLICES; ++b) {
      std::fill(rs.begin(), rs.end(), 0.0);
      int p = 0;
      for (int t1 = 0; t1 < fpl; ++t1)
        for (int t2 = t1; t2 < fpl; ++t2, ++p)
          for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 4; ++r) {
              const double v = std::fabs(g[((size_t)(b * np + p) * 64 + l) * 4 + r]);
              const int i = 4 * (l >> 4) + r, j = l & 15;
              rs[fpl * i + t1] += v;
              if (t1 != t2) rs[fpl * j + t2] += v;
            }
      double mx = 0.0;
      for (double v : rs) mx = std::max(mx, v);
      xg_lam_[b] = mx * (1.0 + 1e-12);  // integer sums < 2^53: exact but for the last few adds
    }
    xg_valid_ = true;
    return true;
  }
  // The digit G stage scales every y of a row by one power of two set by the image's LARGEST
  // sample exponent emax, so a typical sample keeps 2^(emax − e_typ) fewer bits of y (its X
  // digits carry their own 2^e_t; y's fixed point does not). Its G error grows by that factor
  // (measured, tests/test_gpu_g8.py: ≈ 1e-13 relative at T ≈ 5e3 for Δe = 0.8, 1.1e-12 for
  // Δe ≈ 3.8; falling as 1/√T), so the stage runs only while Δe = emax − log2(mean of 2^e_t over
  // the valid samples) ≤ G8_SPREAD_MAX + ⌊½·log2(T / 5000)⌋ (one more bit per 4× samples: at most
  // ≈ 4e-13 at any T) — samples 16× the typical one at T ≈ 5e3 put G back on fp64 MFMA (same
  // all-reduce: no agreement needed). The bench mixture: Δe ≈ 0.9 at T = 2e5 (C3 shards: ≤ 7.5).
  static constexpr double G8_SPREAD_MAX = 2.5;
  bool g8_spread_ok(int emax) const {
    if (n_local_ == 0) return true;
    // padding samples carry the scale 1 exactly (k_slice_x): remove them from the sum
    const double valid = xsc_sum_ - (double)(ldx - n_local_);
    if (!(valid > 0.0)) return false;
    const double extra = std::floor(std::fmax(0.0, 0.5 * std::log2((double)n_local_ / 5000.0)));
    return (double)emax - std::log2(valid / (double)n_local_) <= G8_SPREAD_MAX + extra;
  }
  // exponent range of the digit image's sample scales 2^e_t (the fp32 screen's range check)
  int xsc_emin_ = 0, xsc_emax_ = 0;
  bool xsc_range_ok_ = false;
  // W (nc × nf, host) → slice image [wave][a][kstep][lane][16 B] + row scales 2^(f_i − 12).
  // The same W as the last call (a completion at the W of the loss-only try) is not
  // sliced again. Digits: oz_digits' arithmetic with a 1.5·2^52 shifter for rint
  // (exact round-half-even for |v| < 2^51, no libm call on the host).
  std::vector<double> wsl_w_;
  size_t wsl_nc_ = 0;
  static constexpr size_t WSL_IMG_MAX = (size_t)32 * OZ_SLICES * 4 * 64 * 16;  // 32 row blocks × 4 k-steps
  // one allocation [512 row scales | slice image], the layout of the pinned slot, so that one
  // copy uploads both (a call's GPU timeline pays a dependency gap per copy)
  static constexpr size_t WSC_BYTES = 512 * sizeof(double);
  void alloc_wsl() {
    if (!d_wsc) {
      HIP_OK(t_malloc((void**)&d_wsc, WSC_BYTES + WSL_IMG_MAX));
      d_wsl = (uint8_t*)d_wsc + WSC_BYTES;
    }
  }
  // the multi-try pass: W in row blocks 0–15 (scales 0–255), Z = D·W in 16–31 (256–511)
  void upload_wsl2(const double* w, const double* z, size_t nc) {
    alloc_wsl();
    if (nc > 256) throw computation_error("int8 W image: nc > 256");
    const int ksw = wsl_ksw();
    const size_t half = (size_t)16 * OZ_SLICES * ksw * 64 * 16;
    double* sc = (double*)pin_acquire(pin_wsl_, WSC_BYTES + WSL_IMG_MAX);
    uint8_t* img = (uint8_t*)sc + WSC_BYTES;
    std::memset(img, 0, 2 * half);
    for (int i = 0; i < 512; ++i) sc[i] = 0x1p-12;
    oz_split_rows(w, nc, nf, img, sc, ksw);
    oz_split_rows(z, nc, nf, img + half, sc + 256, ksw);
    wsl_nc_ = 0;  // the image no longer holds a single W
    HIP_OK(hipMemcpyAsync(d_wsc, sc, WSC_BYTES + 2 * half, hipMemcpyHostToDevice, stream));
    pin_release(pin_wsl_);
  }
  void upload_wsl(const double* w, size_t nc) {
    const int emax = xsc_range_ok_ ? xsc_emax_ : INT_MIN;
    if (wsl_nc_ == nc && wsl_w_.size() == nc * nf && std::memcmp(wsl_w_.data(), w, nc * nf * sizeof(double)) == 0 &&
        (nc > 128 || g8_emax_ == emax))
      return;
    // up to 16 row blocks (256 rows); k-step stride wsl_ksw() (2: the NB = 8 / 4 kernels,
    // 4: the tiled pass at nf ≤ 256); the multi-try pass puts Z in row blocks 16–31
    constexpr size_t IMG_MAX = WSL_IMG_MAX;
    const int ksw = wsl_ksw();
    const size_t img_bytes = (size_t)((nc + 15) / 16) * OZ_SLICES * ksw * 64 * 16;
    alloc_wsl();
    if (nc > 256) throw computation_error("int8 W image: nc > 256");
    double* sc = (double*)pin_acquire(pin_wsl_, WSC_BYTES + IMG_MAX);
    uint8_t* img = (uint8_t*)sc + WSC_BYTES;
    std::memset(img, 0, img_bytes);
    for (int i = 0; i < 256; ++i) sc[i] = 0x1p-12;
    wsl_dn2_.assign(nc * OZ_SLICES, 0.0);
    oz_split_rows(w, nc, nf, img, sc, ksw, wsl_dn2_.data());  // host_linalg.cpp: rows split over the host threads
    // fused_g8.inc: ysc_j = 2^(46 − F_j) with |y_jt| < 2^F_j for every sample:
    // |y_jt| ≤ Σ_k|W_jk|·max_k|X_kt| < 2^(ilogb(Σ|W_j|) + 1)·2^emax (Σ|W_j| taken 1e-12 high for its
    // own rounding; the digit forms of W and X and the fp64 combine stay within 2^-50 of it, and
    // the 6-digit range reaches 0.996·2^47); zero rows (padding) get 1
    g8_scales_ok_ = false;
    g8_emax_ = INT_MIN;
    if (nc <= 128 && emax != INT_MIN && g8_spread_ok(emax)) {
      bool ok = true;
      for (size_t j = 0; j < 128; ++j) {
        double s1 = 0.0;
        if (j < nc)
          for (size_t k = 0; k < nf; ++k) s1 += std::fabs(w[j * nf + k]);
        if (!std::isfinite(s1)) { ok = false; break; }
        if (s1 == 0.0) { sc[256 + j] = 1.0; continue; }
        const int fj = std::ilogb(s1 * (1.0 + 1e-12)) + 1 + emax;
        if (fj < -900 || fj > 900) { ok = false; break; }
        sc[256 + j] = std::ldexp(1.0, 46 - fj);
      }
      g8_scales_ok_ = ok;
      g8_emax_ = ok ? emax : INT_MIN;
    }
    wsl_w_.assign(w, w + nc * nf);
    wsl_nc_ = nc;
    HIP_OK(hipMemcpyAsync(d_wsc, sc, WSC_BYTES + img_bytes, hipMemcpyHostToDevice, stream));
    pin_release(pin_wsl_);  // the pinned images stay untouched until these copies are done
  }
  // Σ_k w_a,ik² per row and digit level of the W in the image (upload_wsl) and of the paired
  // screen's two W's (upload_wsl_pair): the screen's statistical bound
  std::vector<double> wsl_dn2_, pair_dn2_[2];
  // two tries' W for the paired screen: w1 in row blocks 0 … NB − 1, w2 in NB … 2·NB − 1 (row
  // scales 0 … and 16·NB …), the layout k_screen_oz2<NB, ·, 2> reads
  void upload_wsl_pair(const double* w1, const double* w2, size_t nc, int nb) {
    alloc_wsl();
    if (nc > (size_t)16 * nb) throw computation_error("paired W image: nc > 16·NB");
    const int ksw = wsl_ksw();
    const size_t half = (size_t)nb * OZ_SLICES * ksw * 64 * 16;
    double* sc = (double*)pin_acquire(pin_wsl_, WSC_BYTES + WSL_IMG_MAX);
    uint8_t* img = (uint8_t*)sc + WSC_BYTES;
    std::memset(img, 0, 2 * half);
    for (int i = 0; i < 512; ++i) sc[i] = 0x1p-12;
    pair_dn2_[0].assign(nc * OZ_SLICES, 0.0);
    pair_dn2_[1].assign(nc * OZ_SLICES, 0.0);
    oz_split_rows(w1, nc, nf, img, sc, ksw, pair_dn2_[0].data());
    oz_split_rows(w2, nc, nf, img + half, sc + 16 * nb, ksw, pair_dn2_[1].data());
    wsl_nc_ = 0;  // the image no longer holds a single W
    HIP_OK(hipMemcpyAsync(d_wsc, sc, WSC_BYTES + 2 * half, hipMemcpyHostToDevice, stream));
    pin_release(pin_wsl_);
  }
  // NB = 8 (64 < nc ≤ 128) or NB = 4 (32 < nc ≤ 64, nf ≤ 64; partition in 32-sample blocks,
  // that of k_eval_fused<4> / k_eval_loss<4>)
  template <int D, bool Q, int DMAX = OZ_SLICES - 1, bool F32L = false, int NB = 8>
  void launch_loss_oz(double alpha, bool store, double* st_rows) {
    constexpr int NCP = 16 * NB, KSO = NB == 8 ? 2 : 1;
    const uint64_t n_blocks = NB == 8 ? (n_local_ + 15) / 16 : (n_local_ + 31) / 32;
    uint64_t bpw;
    const int nwg = partition(n_blocks, &bpw);
    double* part = ensure(d_part, cap_part, (size_t)nwg * 2 * NCP);
    // never launch on a released image (callers allocate their buffers before relying on it)
    if (!xsl_valid_ || !d_xsl) throw computation_error("int8 digit image released while a pass was set up");
    if (oz_kso() != KSO) throw computation_error("int8 digit image of another layout");
    const size_t lds = (size_t)2 * 2 * (oz_block_bytes<KSO>() + 256) + (size_t)2 * 2 * 8 * 4 * 64 * sizeof(double);
    auto kern = F32L ? (oz_pair_ ? k_eval_loss_oz<D, false, Q, DMAX, F32L, NB>
                                 : k_eval_loss_oz<D, false, Q, DMAX, F32L, NB, false>)
                     : store ? k_eval_loss_oz<D, true, Q, DMAX, false, NB> : k_eval_loss_oz<D, false, Q, DMAX, false, NB>;
    lds_attr((const void*)kern, (int)lds);
    HIP_OK(hipEventRecord(ev[1], stream));
    kern<<<nwg, OZW_THREADS, lds, stream>>>(d_xsl, d_xsc, d_wsl, d_wsc, alpha, bpw, n_blocks, part,
                                              store ? d_ybuf : nullptr);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ev[2], stream));
    k_reduce_rows<<<(2 * (int)kept_nc_pending + RED_OUT - 1) / RED_OUT, 256, 0, stream>>>(
        part, nwg, 2 * NCP, 0, NCP, (int)kept_nc_pending, 2, st_rows, D, alpha, (double)n_local_, 1);
    HIP_OK(hipGetLastError());
    ++n_int8_passes_;
    if (DMAX < OZ_SLICES - 1) ++n_screen_passes_;
  }
  uint64_t n_screen_passes_ = 0;
  bool oz_pair_ = std::getenv("PICARD_OZ_NOPAIR") == nullptr;  // A/B knob: paired M-wave blocks
  bool no_ws4_ =std::getenv("PICARD_NO_WS4") != nullptr;
  // the tanh screen evaluates ℓ in fp32 (PICARD_SCREEN_F64=1: the fp64 row terms of the
  // exact pass, a tighter bound at a higher cost)
  bool screen_f32_ = std::getenv("PICARD_SCREEN_F64") == nullptr;
  // Sources on the int8 digit stage (k_ystore_oz) when this context already holds the digit
  // image of the current centring: W digits uploaded, blocks b_first … of the image, Y
  // row-major (ld ldy), samples [0, n_out) of that range. The image is never built for a
  // transform alone (building it is a pass of its own).
  bool ystore_oz_ok(size_t nc) const { return xsl_valid_ && oz_shape(nc); }
  void ystore_oz_run(uint64_t b_first, uint64_t n_out, size_t nc, double* Y, uint64_t ldy) {
    const uint64_t n_blocks = (n_out + 15) / 16;
    uint64_t bpw;
    const int nwg = partition(n_blocks, &bpw);
    const size_t lds = (size_t)2 * 2 * (OZ_BLOCK_BYTES + 256) + (size_t)2 * 2 * 8 * 4 * 64 * sizeof(double);
    lds_attr((const void*)k_ystore_oz, (int)lds);
    k_ystore_oz<<<nwg, OZW_THREADS, lds, stream>>>(d_xsl, d_xsc, d_wsl, d_wsc, b_first, bpw, n_blocks, n_out, (int)nc,
                                                   Y, ldy);
    HIP_OK(hipGetLastError());
    ++n_int8_passes_;
  }
  // Rank agreement on a per-rank capability that selects between branches with different
  // collectives: the first call all-reduces the local flag (all ranks must have it);
  // later calls reuse the answer, and a rank that loses the capability afterwards
  // raises instead of diverging. state: 0 not asked, 1 all have it, -1 some do not.
  int screen_agreed_ = 0, ybuf_agreed_ = 0;
  uint64_t n_agree_ = 0;
  bool pin_test_ = false;  // PICARD_TEST_PIN_DIGITS=1: pin the image without a group (tests)
  // (either agreement pins it: a paired screen may be the first screen of a fit)
  bool xsl_pinned() const { return (coll_ && (screen_agreed_ == 1 || screen_pair_agreed_ == 1)) || pin_test_; }
  bool agree_once(int& state, bool local, const char* what) {
    if (state == 0) {
      ++n_agree_;
      double* f = ensure(d_shift_sum, cap_shift_sum, std::max<size_t>(nf, 1));  // scratch (not d_stats)
      const double one = local ? 1.0 : 0.0;
      HIP_OK(hipMemcpyAsync(f, &one, sizeof(double), hipMemcpyHostToDevice, stream));
      allreduce(f, 1, "agree");
      double all = 0.0;
      HIP_OK(hipMemcpyAsync(&all, f, sizeof(double), hipMemcpyDeviceToHost, stream));
      sync();
      state = all == (double)world ? 1 : -1;
    }
    if (state < 0) return false;
    if (!local) {
      // the other ranks take the agreed branch: end the group instead of diverging
      const std::string m = std::string("the ranks agreed on ") + what + " but rank " + std::to_string(rank) + " lost it";
      abort_group(m);
      throw computation_error(m);
    }
    return true;
  }

  // The orthogonal line-search screen (Evaluator::eval_loss_screen): the loss-only
  // pass on diagonals D ≤ DMAX of the int8 digit stage (DMAX = 3: 10 digit products
  // instead of 28). The exact stage's y differs from it by 2^(f_i+e_t−12)·Σ_{D>DMAX} 256^−D·P_D,
  // |P_D| ≤ nf·Σ_{a+b=D} |d_a|max·|d_b|max (|d_0| ≤ 65, |d_a| ≤ 128), so with ℓ
  // Lipschitz in y (tanh: |ℓ′| = |tanh αy| ≤ 1; exp: |ℓ′| ≤ 1/√(αe)) each row's Σℓ
  // moves by at most Lip·2^(f_i−12)·B·Σ_t 2^e_t; 1e-10 of Σ_t|ℓ| covers the rounding
  // of both passes (their sums run in the same order). Ortho densities tanh / exp.
  // diagonals the first screen keeps: D ≤ 2 (6 digit products, 3 planes) by default, with the
  // statistical tail bound (screen_rank_bound); a try it leaves undecided above the current loss
  // goes to D ≤ 3 (10 products, 4 planes), then D ≤ 4 (15, 5) — eval_loss_screen_fine's levels.
  // PICARD_SCREEN_DMAX=3 / 4 starts the chain there. A rank without the digit Grams (or the
  // fp32 screen form) runs D ≤ 3 where D ≤ 2 is asked (same collectives; its bound is its own).
  int screen_dmax_ = [] {
    const char* e = std::getenv("PICARD_SCREEN_DMAX");
    const int v = e ? std::atoi(e) : 2;
    return v == 3 || v == 4 ? v : 2;
  }();
  // fp32 ℓ in the tanh screen (loss_acc4_f32): hardware error constants, each at least the
  // exhaustive measurement of pc_device_check_fp32_transcendentals on MI355X (the -m gpu
  // test fails if a device exceeds them): v_exp_f32 relative on [−126, 0], absolute below;
  // v_log_f32 absolute on [2^-4, 1] (the product of 4 factors in [1/2, 1]). Measured:
  // 1.42·2^-24 and 8.0·2^-24 on [2^-6, 1] (tests/test_gpu_screen32.py)
  static constexpr double SCREEN_EXP2_REL = 0x1p-23, SCREEN_EXP2_TINY = 0x1p-124, SCREEN_LOG2_ABS = 0x1p-21;
  // Bound (Σℓ units) on |Σ of one lane-block's 4 fp32 ℓ log terms − the exact ones|:
  //   z = fl32(|y|)·c32 is within 3.0000002·2^-24·|z*| of z* = −2α|y|·log2 e, so
  //   |2^z − 2^z*| ≤ 2^z*·|z*|·3.0003·2^-24·ln2 ≤ 1.1038·2^-24 (max_z |z|2^z = 1/(e·ln2));
  //   v_exp_f32 adds ≤ E_rel·2^z/(1 + 2^z) ≤ E_rel/2 (in (1+e) relative terms), or E_tiny;
  //   fl32((1+e)/2) and the 3 products round by 2^-24 each; v_log_f32 adds E_log;
  //   d log2 = d(1+e)/((1+e)·ln2), and the log2 sum enters Σℓ times ln2/α.
  static double screen_f32_block_bound(double alpha) {
    const double u = 0x1p-24;
    const double per_elem = 1.1038 * u + 0.50005 * SCREEN_EXP2_REL + u + SCREEN_EXP2_TINY;
    return 1.001 * (4.0 * per_elem + 3.0 * u + fm::LN2 * SCREEN_LOG2_ABS) / alpha;
  }
  bool eval_loss_screen(const double* w, size_t nc, const double* mu, pc_density d, double* ll_out,
                        double* bound_out) override {
    return screen_at(screen_dmax_, w, nc, mu, d, ll_out, bound_out);
  }
  // the finer screens: level 1, 2, … keep D ≤ screen_dmax_ + level, up to D ≤ 4
  bool eval_loss_screen_fine(int level, const double* w, size_t nc, const double* mu, pc_density d, double* ll_out,
                             double* bound_out) override {
    return level >= 1 && screen_dmax_ + level <= 4 && screen_at(screen_dmax_ + level, w, nc, mu, d, ll_out, bound_out);
  }
  // W row exponents (the kernels' f_i: 2^f_i > max_k |W_ik|; 0 for a zero row), and whether
  // the fp32 screen's scales 2^(f_i+e_t−20) all stay normal fp32 with room (see screen_at)
  void screen_row_exps(const double* w, size_t nc, std::vector<int>& fexp, bool& f32_ok) const {
    fexp.assign(nc, 0);
    for (size_t i = 0; i < nc; ++i) {
      double mx = 0.0;
      for (size_t k = 0; k < nf; ++k) {
        const double f = std::fabs(w[i * nf + k]);
        mx = f > mx ? f : mx;  // = fmax: a NaN weight is skipped, as fmax skips it
      }
      if (mx > 0.0) {
        (void)std::frexp(mx, &fexp[i]);
        if (fexp[i] - 20 + xsc_emin_ < -100 || fexp[i] - 20 + xsc_emax_ > 99) f32_ok = false;
      }
    }
  }
  // This rank's part of the bound per row: the truncation tail and the fp32 terms. The exact
  // stage's y differs from the screen's by Σ_{dmax < a+b ≤ 6} W_a,i·X_b,t (W_a,i = 2^(f_i−6−8a)·w_a,i,
  // X_b,t = 2^(e_t−6−8b)·d_b,t: the digit levels), and ℓ is Lipschitz in y, so each row's Σℓ moves
  // by at most Lip·Σ_(a,b) Σ_t |W_a,i·X_b,t|. Two rigorous bounds of that sum; the smaller is taken:
  //  * worst case: every digit at its largest, 2^(f_i−12)·Σ_D 256^−D·max|P_D|·Σ_t 2^e_t;
  //  * statistical (dn2 and the digit Grams present): Cauchy–Schwarz over t with the weights
  //    2^e_t, Σ_t 2^e_t·|w_a,i·d_b,t| ≤ √(Σ_t 4^e_t)·√(w_a,i·D_b·w_a,iᵀ) ≤ √(S4·λ_b·‖w_a,i‖²)
  //    (D_b the exact digit Gram, λ_b ≥ its largest eigenvalue) — ≈ 30× smaller on the bench
  //    mixtures, which lets a D ≤ 2 screen decide what the worst case needed D ≤ 3 for.
  // f32l: the fp32 combine's absolute term (fl(R23), D ≥ 3 only: |P_2| < 2^24 is exact in fp32)
  // and the fp32 ℓ terms per 4-sample block.
  void screen_rank_bound(int dmax, const std::vector<int>& fexp, const double* dn2, size_t nc, pc_density d,
                         bool f32l, double* bnd) const {
    auto pm = [](int dd) {  // Σ_{a+b=dd} |d_a|max·|d_b|max per feature
      double v = 0.0;
      for (int a = 0; a < OZ_SLICES; ++a) {
        const int b = dd - a;
        if (b >= 0 && b < OZ_SLICES) v += (a == 0 ? 65.0 : 128.0) * (b == 0 ? 65.0 : 128.0);
      }
      return v;
    };
    double bsum = 0.0, bf32 = 0.0;
    for (int dd = dmax + 1; dd <= OZ_SLICES - 1; ++dd) bsum += std::ldexp(pm(dd), -8 * dd);  // exact stage: D ≤ 6
    if (f32l && dmax >= 3) bf32 = std::ldexp(256.0 * pm(2) + pm(3) + pm(4) / 256.0, -46) * (1.0 + 1e-6);
    const double lip = d.kind == DENS_TANH ? 1.0 : 1.0 / std::sqrt(d.alpha * std::exp(1.0));
    const double worst = (double)nf * bsum * xsc_sum_ * lip, f32abs = (double)nf * bf32 * xsc_sum_ * lip;
    const bool stat = dn2 != nullptr && xg_valid_;
    for (size_t i = 0; i < nc; ++i) {
      double tail = worst;
      if (stat) {
        double st = 0.0;
        for (int a = 0; a < OZ_SLICES; ++a)
          for (int b = 0; b < OZ_SLICES; ++b) {
            const int dd = a + b;
            if (dd > dmax && dd <= OZ_SLICES - 1)
              st += std::ldexp(std::sqrt(dn2[i * OZ_SLICES + a] * xg_lam_[b] * xsc_s4_), -8 * dd);
          }
        tail = std::min(tail, st * lip * (1.0 + 1e-9));  // (1e-9: the rounding of these few ops)
      }
      bnd[i] = std::ldexp(tail + f32abs, fexp[i] - 12) * (1.0 + 1e-12);
      if (f32l) bnd[i] += (double)(ldx / 4) * screen_f32_block_bound(d.alpha);
    }
  }
  // PICARD_SCREEN_PAIRS=0: no paired screens (the solver screens tries one by one)
  const bool screen_pairs_ = !(std::getenv("PICARD_SCREEN_PAIRS") && std::atoi(std::getenv("PICARD_SCREEN_PAIRS")) == 0);
  int screen_pair_agreed_ = 0;
  // the sample-exponent window every rank's image must lie in for the paired screen: the fp32
  // range test then depends on W alone (rank-identical), so every rank takes the same branch
  static constexpr int PAIR_EMIN = -40, PAIR_EMAX = 40;
  // Two tries in one pass (k_screen_oz2<NB, ·, 2>): the tanh fp32 D ≤ 3 screen only. A paired
  // and a single screen issue different all-reduces, so with a communicator the ranks agree once
  // that each holds the digit image and its fp32 scales with sample exponents inside
  // [PAIR_EMIN, PAIR_EMAX]; the per-call test (both W's row exponents against that window) is on
  // rank-identical data. Each try's rows are those of screen_at for that W alone: the same
  // kernel arithmetic per W, the same bound terms.
  bool eval_loss_screen2(const double* w1, const double* w2, size_t nc, const double* mu, pc_density d, double* ll1,
                         double* bnd1, double* ll2, double* bnd2) override {
    if (!screen_pairs_ || screen_dmax_ > 3 || !screen_nows_ || !screen_v2_ || !screen_f32_) return false;
    if (y_stage_ != 0 || !oz_any(nc) || !(d.alpha > 0.0) || d.kind != DENS_TANH) return false;
    std::vector<int> f1, f2;
    bool w_ok = true;
    screen_row_exps(w1, nc, f1, w_ok);
    screen_row_exps(w2, nc, f2, w_ok);
    for (size_t i = 0; i < nc && w_ok; ++i)
      w_ok = f1[i] - 20 + PAIR_EMIN >= -100 && f1[i] - 20 + PAIR_EMAX <= 99 && f2[i] - 20 + PAIR_EMIN >= -100 &&
             f2[i] - 20 + PAIR_EMAX <= 99;
    if (!w_ok) return false;  // rank-identical
    const bool nb4 = oz4_shape(nc);
    const int nb = nb4 ? 4 : 8;
    HIP_OK(hipSetDevice(device));
    const double* dmu = resident_mu(mu);
    double* st_rows = ensure(d_stats, cap_stats, 6 * nc);  // per try [Σℓ | Σ|ỹ| | bound]
    {
      uint64_t bpw0;
      const int nwg0 = partition(nb4 ? (n_local_ + 31) / 32 : (n_local_ + 15) / 16, &bpw0);
      ensure(d_part, cap_part, (size_t)std::max(nwg0, 2 * n_cu) * 2 * 2 * (nb4 ? 64 : 128));
    }
    bool ok = dmu == nullptr && ensure_xsl() && ensure_xsf() && xsc_range_ok_ && xsc_emin_ >= PAIR_EMIN &&
              xsc_emax_ <= PAIR_EMAX;
    if (coll_) ok = agree_once(screen_pair_agreed_, ok, "the paired line-search screen");
    if (!ok) return false;
    // D ≤ 2 where this rank has the digit Grams (else D ≤ 3: the same collectives)
    const int dmax = screen_dmax_ == 2 && ensure_digit_gram() ? 2 : 3;
    upload_wsl_pair(w1, w2, nc, nb);
    d_wsl_ready_ = false;  // the image holds two W's: no completion may reuse it
    kept_nc_pending = nc;
    HIP_OK(hipEventRecord(ev[0], stream));
    double* direct = direct_acquire(6 * nc);
    if (direct) st_rows = direct;
    const bool launched =
        nb4 ? launch_screen_oz2<4>(d.alpha, st_rows, 2, dmax) : launch_screen_oz2<8>(d.alpha, st_rows, 2, dmax);
    if (!launched) throw computation_error("paired screen: launch geometry out of range after the agreement");
    double* bnd = direct ? direct : (double*)pin_acquire(pin_in_, 6 * nc * sizeof(double));
    screen_rank_bound(dmax, f1, pair_dn2_[0].data(), nc, d, true, bnd + 2 * nc);
    screen_rank_bound(dmax, f2, pair_dn2_[1].data(), nc, d, true, bnd + 5 * nc);
    n_screen_products += 2 * (uint64_t)((dmax + 1) * (dmax + 2) / 2);
    std::vector<double> tmp(6 * nc);
    const double* staged = direct;
    if (direct) {
      pin_release(pin_direct_);  // the kernel writes rows 0–1 of each try, the host row 2
    } else {
      HIP_OK(hipMemcpyAsync(st_rows + 2 * nc, bnd + 2 * nc, nc * sizeof(double), hipMemcpyHostToDevice, stream));
      HIP_OK(hipMemcpyAsync(st_rows + 5 * nc, bnd + 5 * nc, nc * sizeof(double), hipMemcpyHostToDevice, stream));
      pin_release(pin_in_);
      allreduce(st_rows, 6 * nc, "screen pair");
      staged = d2h_enqueue(st_rows, 6 * nc);
    }
    finish_timing(true, 4);
    ++n_screen_tries;  // the pass covered two tries
    copy_out(tmp.data(), staged, 6 * nc);
    const double kappa1 = 0x1p-22 * 1.0001;
    for (int t = 0; t < 2; ++t) {
      const double* r = tmp.data() + (size_t)t * 3 * nc;
      double* llo = t ? ll2 : ll1;
      double* bo = t ? bnd2 : bnd1;
      for (size_t i = 0; i < nc; ++i) {
        llo[i] = r[i];
        bo[i] = r[2 * nc + i] + kappa1 * std::fabs(r[nc + i]) + 1e-10 * std::fabs(r[i]);
      }
    }
    return true;
  }
  bool screen_at(int dmax, const double* w, size_t nc, const double* mu, pc_density d, double* ll_out,
                 double* bound_out) {
    if (y_stage_ != 0 || !oz_any(nc) || !(d.alpha > 0.0) || (d.kind != DENS_TANH && d.kind != DENS_EXP))
      return false;
    const bool nb4 = oz4_shape(nc);
    HIP_OK(hipSetDevice(device));
    const double* dmu = resident_mu(mu);
    double* st_rows = ensure(d_stats, cap_stats, 3 * nc);  // [Σℓ | Σ|ỹ| (fp32 screen) | bound]
    double* direct = nullptr;
    {  // the pass buffers before the image is relied on (an allocation may release it)
      uint64_t bpw0;
      const int nwg0 = partition(nb4 ? (n_local_ + 31) / 32 : (n_local_ + 15) / 16, &bpw0);
      ensure(d_part, cap_part, (size_t)nwg0 * 2 * (nb4 ? 64 : 128));
    }
    bool ok = dmu == nullptr && ensure_xsl();
    // With a communicator every rank must take the same branch (a screen and a full pass
    // issue different all-reduces): the ranks agree once on availability (the digit image
    // is a per-rank allocation).
    if (coll_) ok = agree_once(screen_agreed_, ok, "the int8 digit image (line-search screen)");
    if (!ok) return false;
    upload_wsl(w, nc);
    d_wsl_ready_ = true;
    kept_nc_pending = nc;
    // W row exponents (the kernels' f_i: 2^f_i > max_k |W_ik|; 0 for a zero row)
    std::vector<int> fexp(nc, 0);
    std::vector<char> zero_row(nc, 1);
    for (size_t i = 0; i < nc; ++i) {
      double mx = 0.0;
      for (size_t k = 0; k < nf; ++k) {
        const double f = std::fabs(w[i * nf + k]);
        mx = f > mx ? f : mx;  // = fmax: a NaN weight is skipped, as fmax skips it
      }
      if (mx > 0.0) { (void)std::frexp(mx, &fexp[i]); zero_row[i] = 0; }
    }
    // fp32 screen (tanh): every scale 2^(f_i+e_t−20) a normal fp32 power of two with room for
    // |Q01| < 2^28 above it and 2^-24 below it (else this rank runs the fp64-ℓ screen: both
    // issue the same all-reduce and each rank's part of the bound covers its own arithmetic)
    bool f32l = d.kind == DENS_TANH && screen_f32_ && xsc_range_ok_;
    for (size_t i = 0; f32l && i < nc; ++i)
      if (!zero_row[i] && (fexp[i] - 20 + xsc_emin_ < -100 || fexp[i] - 20 + xsc_emax_ > 99)) f32l = false;
    // D ≤ 2 only with this rank's digit Grams (its worst-case tail is ≈ 190× D ≤ 3's)
    if (dmax == 2 && !ensure_digit_gram()) dmax = 3;
    HIP_OK(hipEventRecord(ev[0], stream));
    direct = direct_acquire(3 * nc);  // (after the image checks: no early return holds the slot)
    if (direct) st_rows = direct;
    dmax = nb4 ? screen_launch<4>(d, dmax, f32l, st_rows) : screen_launch<8>(d, dmax, f32l, st_rows);
    n_screen_products += (uint64_t)((dmax + 1) * (dmax + 2) / 2);
    // this rank's bound: summed over ranks with the statistics (its own row of the all-reduce)
    // (fp32 ℓ: 4 lane-blocks of 4 samples per 16-sample block of each row, padding included)
    double* bnd = direct ? direct + 2 * nc : (double*)pin_acquire(pin_in_, nc * sizeof(double));  // H2D by DMA
    screen_rank_bound(dmax, fexp, wsl_dn2_.size() == nc * OZ_SLICES ? wsl_dn2_.data() : nullptr, nc, d, f32l, bnd);
    std::vector<double> tmp(3 * nc);
    const double* staged = direct;
    if (direct) {
      pin_release(pin_direct_);  // the kernel writes rows 0–1, the host row 2 (disjoint)
    } else {
      HIP_OK(hipMemcpyAsync(st_rows + 2 * nc, bnd, nc * sizeof(double), hipMemcpyHostToDevice, stream));
      pin_release(pin_in_);
      allreduce(st_rows, 3 * nc, "screen");
      staged = d2h_enqueue(st_rows, 3 * nc);
    }
    finish_timing(true, 4);
    copy_out(tmp.data(), staged, 3 * nc);
    // the rounding slack: Σ_t |ℓ| ≤ |Σℓ| for tanh (ℓ ≥ 0), ≤ n/α for exp (|ℓ| ≤ 1/α);
    // fp32 screen: κ1·Σ|ỹ| covers |ỹ| against the DMAX-digit y and the fp32 sum of |ỹ|
    // (slot 1 is Σ|ỹ| on the ranks that ran it, 0 on the others: the kernels' Σy² is not kept)
    const double n_all = (double)n_total, kappa1 = 0x1p-22 * 1.0001;
    for (size_t i = 0; i < nc; ++i) {
      ll_out[i] = tmp[i];
      const double abs_l = d.kind == DENS_TANH ? std::fabs(tmp[i]) : n_all / d.alpha;
      bound_out[i] = tmp[2 * nc + i] + kappa1 * std::fabs(tmp[nc + i]) + 1e-10 * abs_l;
    }
    return true;
  }

  // the non-specialised fp32 screen (k_screen_oz; PICARD_SCREEN_WS=1: the warp-specialised
  // k_eval_loss_oz<…, F32L> instead)
  bool screen_nows_ = std::getenv("PICARD_SCREEN_WS") == nullptr;
  template <int DMAX, int NB>
  void launch_screen_oz(double alpha, double* st_rows) {
    constexpr int NCP = 16 * NB, KSO = NB == 8 ? 2 : 1, U = 16 / NB, SLOT = (DMAX + 1) * KSO * 1024;
    const uint64_t n_blocks = (n_local_ + 15) / 16;
    uint64_t bpw;
    const int nwg = partition((n_blocks + U - 1) / U, &bpw);
    bpw *= U;  // 16-sample blocks per workgroup, whole steps
    double* part = ensure(d_part, cap_part, (size_t)nwg * 2 * NCP);
    if (!xsl_valid_ || !d_xsl) throw computation_error("int8 digit image released while a pass was set up");
    if (oz_kso() != KSO) throw computation_error("int8 digit image of another layout");
    const size_t lds = (size_t)3 * U * SLOT + (size_t)3 * U * 256 + (size_t)U * NCP * 2 * sizeof(double);
    lds_attr((const void*)k_screen_oz<DMAX, NB>, (int)lds);
    HIP_OK(hipEventRecord(ev[1], stream));
    k_screen_oz<DMAX, NB><<<nwg, OZW_THREADS, lds, stream>>>(d_xsl, d_xsc, d_wsl, d_wsc, alpha, bpw, n_blocks, part);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ev[2], stream));
    k_reduce_rows<<<(2 * (int)kept_nc_pending + RED_OUT - 1) / RED_OUT, 256, 0, stream>>>(
        part, nwg, 2 * NCP, 0, NCP, (int)kept_nc_pending, 2, st_rows, DENS_TANH, alpha, (double)n_local_, 1);
    HIP_OK(hipGetLastError());
    ++n_int8_passes_;
    ++n_screen_passes_;
  }
  // k_screen_oz2 (screen.hip): the same statistics and bound as k_screen_oz on the interleaved
  // schedule; PICARD_SCREEN_V2=0 keeps k_screen_oz. false: not available here.
  bool screen_v2_ = !(std::getenv("PICARD_SCREEN_V2") && std::atoi(std::getenv("PICARD_SCREEN_V2")) == 0);
  bool screen32_ = std::getenv("PICARD_SCREEN32") && std::atoi(std::getenv("PICARD_SCREEN32")) == 1;
  template <int NB>
  bool launch_screen_oz2(double alpha, double* st_rows, int nw = 1, int dmax = 3) {
    constexpr int NCP = 16 * NB;
    // k_screen_oz32 (PICARD_SCREEN32=1): one try at NB = 8, two blocks per step, one workgroup per CU
    const bool f32form = screen32_ && NB == 8 && nw == 1 && dmax == 3;
    const int U = f32form ? 2 : screen2_blocks_per_step(NB);
    const uint64_t n_blocks = (n_local_ + 15) / 16;
    const uint64_t want =
        std::min<uint64_t>((uint64_t)(f32form ? 1 : 2) * n_cu, std::max<uint64_t>((n_blocks + U - 1) / U, 1));
    const uint64_t steps_per_wg = ((n_blocks + U - 1) / U + want - 1) / want;
    const uint64_t bpw = steps_per_wg * U;
    const int nwg = (int)std::max<uint64_t>(1, (n_blocks + bpw - 1) / bpw);
    // 32-bit buffer offsets within a workgroup's range (and the kernel's 32-bit block counts)
    if ((bpw + 2 * (uint64_t)U) * screen2_tile_bytes(NB) >= (1ull << 31) || n_blocks >= (1ull << 32)) return false;
    if (!ensure_xsf()) return false;
    double* part = ensure(d_part, cap_part, (size_t)nwg * nw * 2 * NCP);
    if (!xsl_valid_ || !d_xsl) throw computation_error("int8 digit image released while a pass was set up");
    if (oz_kso() != (NB == 8 ? 2 : 1)) throw computation_error("int8 digit image of another layout");
    Screen2Args a;
    a.xsl = d_xsl; a.xsf = d_xsf; a.wsl = d_wsl; a.wsc = d_wsc;
    a.c32 = (float)(-2.0 * alpha * fm::LOG2E);
    a.e0 = xsf_e0_;
    a.ln2_alpha = fm::LN2 / alpha;
    a.bpw = (uint32_t)bpw; a.n_blocks = (uint32_t)n_blocks; a.nwg = nwg; a.partials = part;
    a.nw = nw;
    a.form32 = f32form;
    a.dmax = dmax;
    HIP_OK(hipEventRecord(ev[1], stream));
    HIP_OK(screen2_launch(NB, a, stream));
    HIP_OK(hipEventRecord(ev[2], stream));
    // try w's rows into st_rows + w·3·nc ([Σℓ | Σ|ỹ|], the bound row is the host's)
    for (int w = 0; w < nw; ++w) {
      k_reduce_rows<<<(2 * (int)kept_nc_pending + RED_OUT - 1) / RED_OUT, 256, 0, stream>>>(
          part, nwg, (size_t)nw * 2 * NCP, (size_t)w * 2 * NCP, NCP, (int)kept_nc_pending, 2,
          st_rows + (size_t)w * 3 * kept_nc_pending, DENS_TANH, alpha, (double)n_local_, 1);
      HIP_OK(hipGetLastError());
    }
    ++n_int8_passes_;
    ++n_screen_passes_;
    return true;
  }
  // returns the diagonals the launched screen keeps (D ≤ 2 is k_screen_oz2's only: elsewhere 3)
  template <int NB>
  int screen_launch(pc_density d, int dmax, bool f32l, double* st_rows) {
    if (f32l && dmax <= 3 && screen_nows_ && screen_v2_ && launch_screen_oz2<NB>(d.alpha, st_rows, 1, dmax))
      return dmax;
    if (dmax < 3) dmax = 3;
    screen_launch_other<NB>(d, dmax, f32l, st_rows);
    return dmax;
  }
  template <int NB>
  void screen_launch_other(pc_density d, int dmax, bool f32l, double* st_rows) {
    if (f32l && dmax == 3 && screen_nows_) launch_screen_oz<3, NB>(d.alpha, st_rows);
    else if (f32l && dmax == 3) launch_loss_oz<DENS_TANH, false, 3, true, NB>(d.alpha, false, st_rows);
    else if (f32l) launch_loss_oz<DENS_TANH, false, 4, true, NB>(d.alpha, false, st_rows);
    else if (d.kind == DENS_TANH && dmax == 3) launch_loss_oz<DENS_TANH, false, 3, false, NB>(d.alpha, false, st_rows);
    else if (d.kind == DENS_TANH) launch_loss_oz<DENS_TANH, false, 4, false, NB>(d.alpha, false, st_rows);
    else if (dmax == 3) launch_loss_oz<DENS_EXP, false, 3, false, NB>(d.alpha, false, st_rows);
    else launch_loss_oz<DENS_EXP, false, 4, false, NB>(d.alpha, false, st_rows);
  }

  template <int NB, int D, bool Q>
  void launch_loss(const double* dmu, double alpha, bool store, double* st_rows) {
    using S = FusedShape<NB>;
    const uint64_t n_blocks = (n_local_ + S::TB - 1) / S::TB;
    if constexpr (NB == 8 || NB == 4) {
      if (dmu == nullptr && (NB == 8 ? oz_shape(kept_nc_pending) : oz4_shape(kept_nc_pending)) && d_wsl_ready_) {
        uint64_t bpw0;
        const int nwg0 = partition(n_blocks, &bpw0);
        ensure(d_part, cap_part, (size_t)nwg0 * 2 * S::NCP);  // may release an unpinned image …
        if (xsl_valid_) {  // … then the fp64 stage below runs (same collectives)
          launch_loss_oz<D, Q, OZ_SLICES - 1, false, NB>(alpha, store, st_rows);
          return;
        }
      }
    }
    uint64_t bpw;
    const int nwg = partition(n_blocks, &bpw);
    double* part = ensure(d_part, cap_part, (size_t)nwg * 2 * S::NCP);
    const size_t lds = (size_t)2 * S::TS * 16 * NB * 16 * sizeof(double);
    // NB = 8 on the centred resident X: LDS-DMA staging, two blocks per barrier
    if (NB == 8 && dmu == nullptr) {
      const size_t lds2 = (size_t)2 * 2 * 128 * 16 * sizeof(double);
      HIP_OK(hipEventRecord(ev[1], stream));
      if (store)
        k_eval_loss2<D, true, Q><<<nwg, FUSED_THREADS, lds2, stream>>>(X, ldx, (int)nf, d_w, alpha, bpw, n_blocks, part,
                                                                      d_ybuf);
      else
        k_eval_loss2<D, false, Q><<<nwg, FUSED_THREADS, lds2, stream>>>(X, ldx, (int)nf, d_w, alpha, bpw, n_blocks, part,
                                                                       nullptr);
    } else if (store) {
      HIP_OK(hipEventRecord(ev[1], stream));
      k_eval_loss<NB, D, true, Q><<<nwg, FUSED_THREADS, lds, stream>>>(X, ldx, n_local_, (int)nf, d_w, dmu, alpha, bpw,
                                                                    n_blocks, part, d_ybuf);
    } else {
      HIP_OK(hipEventRecord(ev[1], stream));
      k_eval_loss<NB, D, false, Q><<<nwg, FUSED_THREADS, lds, stream>>>(X, ldx, n_local_, (int)nf, d_w, dmu, alpha,
                                                                     bpw, n_blocks, part, nullptr);
    }
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ev[2], stream));
    k_reduce_rows<<<(2 * (int)kept_nc_pending + RED_OUT - 1) / RED_OUT, 256, 0, stream>>>(
        part, nwg, 2 * S::NCP, 0, S::NCP, (int)kept_nc_pending, 2, st_rows, D, alpha,
                                         (double)n_local_, 1);
    HIP_OK(hipGetLastError());
  }
  size_t kept_nc_pending = 0;

  template <int NB, bool H, int D>
  void launch_fromy(double alpha, double* st) {
    using S = FusedShape<NB>;
    const uint64_t n_blocks = (n_local_ + S::TB - 1) / S::TB;
    uint64_t bpw;
    const int nwg = partition(n_blocks, &bpw);
    const size_t pstride = fused_partial_stride(S::NCP, H);
    double* part = ensure(d_part, cap_part, (size_t)nwg * pstride);
    const size_t lds = (size_t)2 * (H ? 3 : 2) * S::FRAGS * sizeof(double);
    HIP_OK(hipEventRecord(ev[1], stream));
    k_eval_fromy<NB, H, D><<<nwg, FUSED_THREADS, lds, stream>>>(d_ybuf, n_local_, alpha, bpw, n_blocks, part);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ev[2], stream));
    const size_t nc = kept_nc;
    const size_t e1 = (H ? 2 : 1) * nc * nc + nc;  // [G | H | Σψ′]
    k_reduce<<<(e1 + RED_OUT - 1) / RED_OUT, 256, 0, stream>>>(part, nwg, pstride, S::NCP, (int)nc, H, st, D, alpha,
                                                   (double)n_local_);
    HIP_OK(hipGetLastError());
  }

  double sum_loss_ms = 0, sum_fromy_ms = 0, sum_multi_ms = 0, sum_screen_ms = 0;
  uint64_t n_screen = 0;
  uint64_t n_multi = 0;
  uint64_t n_loss = 0, n_fromy = 0;
  void finish_timing(bool kernel_timed, int kind = 0) {
    HIP_OK(hipEventRecord(ev[3], stream));
    sync();
    float a = 0, b = 0;
    if (kernel_timed) HIP_OK(hipEventElapsedTime(&a, ev[1], ev[2]));
    HIP_OK(hipEventElapsedTime(&b, ev[0], ev[3]));
    last_kernel_ms = kernel_timed ? a : b;
    last_call_ms = b;
    sum_call_ms += b;
    if (kernel_timed) { sum_split_ms += a; ++n_split; }
    if (kind == 1) { sum_loss_ms += a; ++n_loss; }
    if (kind == 2) { sum_fromy_ms += a; ++n_fromy; }
    if (kind == 3) { sum_multi_ms += a; ++n_multi; }
    if (kind == 4) { sum_screen_ms += a; ++n_screen; ++n_screen_tries; }
  }
  uint64_t n_screen_tries = 0;  // tries the screen passes covered (a paired pass: 2)
  uint64_t n_screen_products = 0;  // Σ over those tries of the digit products each kept ((D+1)(D+2)/2)
  double sum_split_ms = 0;
  uint64_t n_split = 0;

  bool eval_loss(const double* w, size_t nc, const double* mu, pc_density d, bool need_h, EvalStats* out,
                 bool keep = true) override {
    if (!fused_ok(nc, d.kind, d.alpha, need_h)) {
      if (!tiled_ok(nc, d.kind, d.alpha)) {
        eval(w, nc, mu, d, need_h, out);
        return false;
      }
      // tiled shapes: loss-only phase 1 now, full recompute (phase 1 + 2) on completion
      HIP_OK(hipSetDevice(device));
      out->nc = nc;
      out->has_h = need_h;
      out->buf.assign(EvalStats::size(nc, need_h), 0.0);
      const size_t total = EvalStats::size(nc, need_h);
      double* st = ensure(d_stats, cap_stats, total);
      HIP_OK(hipEventRecord(ev[0], stream));
      const double* dmu = resident_mu(mu);  // null: X is centred in place
      HIP_OK(hipEventRecord(ev[1], stream));
      tiled_eval(w, nc, dmu, d.kind, d.alpha, need_h, st, 1);
      HIP_OK(hipEventRecord(ev[2], stream));
      allreduce(st + total - 2 * nc, 2 * nc, "loss");
      const double* staged = d2h_enqueue(st + total - 2 * nc, 2 * nc);
      finish_timing(true, 1);
      copy_out(out->buf.data() + total - 2 * nc, staged, 2 * nc);
      kept_tiled = true;
      kept_nc = nc;
      kept_w.assign(w, w + nc * nf);
      kept_mu.assign(mu ? mu : w, mu ? mu + nf : w);
      kept_has_mu = mu != nullptr;
      return true;
    }
    kept_tiled = false;
    HIP_OK(hipSetDevice(device));
    const int nb = pick_nb(nc);
    const int nfp = 16 * nb;
    // keep == false, or no room for Y: loss-only pass, completion recomputes the full pass.
    // With a communicator the ranks agree (once) on keeping Y: the two completions issue
    // different all-reduces.
    // Where the fused pass may form G on int8 digits (fused_g8.inc), the completion recomputes
    // the fused pass instead of forming G from the kept Y on fp64 MFMA: the accepted try's G then
    // has the bits of the fused pass at its W (decided from the shape alone: rank-consistent)
    if (g_stage_ == 0 && nb == 8 && !need_h && (d.kind == DENS_TANH || d.kind == DENS_EXP)) keep = false;
    bool store = keep && ensure_ybuf(nb);
    if (coll_ && keep) store = agree_once(ybuf_agreed_, store, "a kept Y buffer (completion from Y)");
    out->nc = nc;
    out->has_h = need_h;
    out->buf.assign(EvalStats::size(nc, need_h), 0.0);
    const size_t total = EvalStats::size(nc, need_h);
    double* st = ensure(d_stats, cap_stats, total);
    double* st_rows = st + total - 2 * nc;  // [Σℓ | Σy²] are the last 2·nc entries
    HIP_OK(hipEventRecord(ev[0], stream));
    const double* dmu = resident_mu(mu);  // null: X is centred in place
    std::vector<double> wp((size_t)16 * nb * nfp, 0.0);
    for (size_t i = 0; i < nc; ++i)
      for (size_t k = 0; k < nf; ++k) wp[i * nfp + k] = w[i * nf + k];
    ensure(d_w, cap_w, wp.size());
    HIP_OK(hipMemcpyAsync(d_w, wp.data(), wp.size() * sizeof(double), hipMemcpyHostToDevice, stream));
    kept_nc_pending = nc;
    d_wsl_ready_ = false;
    // the int8 stage only where the fused pass at this W runs it too (no H): a try's
    // loss-only pass and its full evaluation must give the same bits
    if (dmu == nullptr && oz_any(nc) && !need_h && ensure_xsl()) {
      upload_wsl(w, nc);
      d_wsl_ready_ = true;
    }
#define PC_LOSS(NBV, Q)                                                                       \
  switch (d.kind) {                                                                             \
    case DENS_TANH: launch_loss<NBV, DENS_TANH, Q>(dmu, d.alpha, store, st_rows); break;         \
    case DENS_EXP: launch_loss<NBV, DENS_EXP, Q>(dmu, d.alpha, store, st_rows); break;           \
    default: launch_loss<NBV, DENS_CUBE, Q>(dmu, d.alpha, store, st_rows); break;                \
  }
    // Σy² only where it is read (non-orthogonal: need_h) or asked for
    const bool q = need_h || want_y2;
    switch (nb) {
      case 1: if (q) { PC_LOSS(1, true); } else { PC_LOSS(1, false); } break;
      case 2: if (q) { PC_LOSS(2, true); } else { PC_LOSS(2, false); } break;
      case 4: if (q) { PC_LOSS(4, true); } else { PC_LOSS(4, false); } break;
      default: if (q) { PC_LOSS(8, true); } else { PC_LOSS(8, false); } break;
    }
#undef PC_LOSS
    allreduce(st_rows, 2 * nc, "loss");
    const double* staged = d2h_enqueue(st_rows, 2 * nc);
    finish_timing(true, 1);
    copy_out(out->buf.data() + total - 2 * nc, staged, 2 * nc);
    kept_nc = nc;
    kept_nb = nb;
    kept_tiled = !store;  // "recompute" completion
    if (!store) {
      kept_w.assign(w, w + nc * nf);
      kept_mu.assign(mu ? mu : w, mu ? mu + nf : w);
      kept_has_mu = mu != nullptr;
    }
    return true;
  }

  template <int NB>
  void dispatch_fromy(pc_density d, bool need_h, double* st) {
    if constexpr (NB == 8) {  // H at NB = 8 does not fit the register budget: never split (fused_ok)
      if (need_h) throw computation_error("split evaluation with H needs nc <= 64");
    } else if (need_h) {
      switch (d.kind) {
        case DENS_TANH: launch_fromy<NB, true, DENS_TANH>(d.alpha, st); return;
        case DENS_EXP: launch_fromy<NB, true, DENS_EXP>(d.alpha, st); return;
        default: launch_fromy<NB, true, DENS_CUBE>(d.alpha, st); return;
      }
    }
    switch (d.kind) {
      case DENS_TANH: launch_fromy<NB, false, DENS_TANH>(d.alpha, st); break;
      case DENS_EXP: launch_fromy<NB, false, DENS_EXP>(d.alpha, st); break;
      default: launch_fromy<NB, false, DENS_CUBE>(d.alpha, st); break;
    }
  }

  void eval_complete_into(pc_density d, bool need_h, double* stats) override {
    if (kept_nc == 0) throw computation_error("no kept evaluation to complete");
    EvalStats tmp;
    tmp.nc = kept_nc;
    tmp.has_h = need_h;
    tmp.buf.assign(EvalStats::size(kept_nc, need_h), 0.0);
    eval_complete(d, need_h, &tmp);
    const size_t e1 = (need_h ? 2 : 1) * kept_nc * kept_nc + kept_nc;
    std::memcpy(stats, tmp.buf.data(), e1 * sizeof(double));
  }

  bool kept_tiled = false, kept_has_mu = false;
  std::vector<double> kept_w, kept_mu;

  void eval_complete(pc_density d, bool need_h, EvalStats* out) override {
    HIP_OK(hipSetDevice(device));
    if (kept_tiled) {  // recompute phase 1 in full mode + phase 2 at the kept W
      const size_t nc = kept_nc;
      const size_t total = EvalStats::size(nc, need_h);
      std::vector<double> full(total);
      run_eval(kept_w.data(), nc, kept_has_mu ? kept_mu.data() : nullptr, d.kind, d.alpha, need_h, full.data());
      const size_t e1 = (need_h ? 2 : 1) * nc * nc + nc;
      std::memcpy(out->buf.data(), full.data(), e1 * sizeof(double));
      return;
    }
    const size_t nc = kept_nc;
    const size_t total = EvalStats::size(nc, need_h);
    double* st = ensure(d_stats, cap_stats, total);
    const size_t e1 = (need_h ? 2 : 1) * nc * nc + nc;
    HIP_OK(hipEventRecord(ev[0], stream));
    switch (kept_nb) {
      case 1: dispatch_fromy<1>(d, need_h, st); break;
      case 2: dispatch_fromy<2>(d, need_h, st); break;
      case 4: dispatch_fromy<4>(d, need_h, st); break;
      default: dispatch_fromy<8>(d, need_h, st); break;
    }
    allreduce(st, e1, need_h ? "complete+H" : "complete");
    const double* staged = d2h_enqueue(st, e1);
    finish_timing(true, 2);
    copy_out(out->buf.data(), staged, e1);
  }

  void sources(const double* w, size_t nc, const double* mu, double* out) override {
    HIP_OK(hipSetDevice(device));
    resident_mu(mu);  // X is centred in place: Y = W·X
    const uint64_t CH = 1ull << 20;
    m4_full_ = nullptr;  // d_chunk is reused
    double* Y = ensure(d_chunk, cap_chunk, nc * CH);  // first: a failed allocation releases the image
    const bool oz = ystore_oz_ok(nc);
    if (oz) upload_wsl(w, nc);
    else ystore_upload(w, nc, nf);
    for (uint64_t c0 = 0; c0 < n_local_; c0 += CH) {
      const uint64_t cn = std::min<uint64_t>(CH, n_local_ - c0);
      if (oz) ystore_oz_run(c0 / 16, cn, nc, Y, CH);
      else ystore_run(X + c0, ldx, nf, nc, cn, Y, CH);
      HIP_OK(hipMemcpy2DAsync(out + c0, n_local_ * sizeof(double), Y, CH * sizeof(double), cn * sizeof(double), nc,
                              hipMemcpyDeviceToHost, stream));
    }
    sync();
  }

  // Sources kept in HBM (S = W·(X − μ), nc × ldx, row-major, zero padding past
  // n_local): the whole shard in one k_ystore pass — for callers that consume
  // the sources on the device; *kernel_ms = the pass's HIP-event time.
  double* d_src = nullptr; size_t cap_src = 0;
  const double* sources_resident(const double* w, size_t nc, const double* mu, double* kernel_ms) {
    HIP_OK(hipSetDevice(device));
    resident_mu(mu);
    double* S = ensure(d_src, cap_src, nc * ldx);  // first: a failed allocation releases the image
    const bool oz = ystore_oz_ok(nc);
    if (oz) upload_wsl(w, nc);
    else ystore_upload(w, nc, nf);
    if (ldx > n_local_)  // the padding columns read as zero, like X's
      HIP_OK(hipMemset2DAsync(S + n_local_, ldx * sizeof(double), 0, (ldx - n_local_) * sizeof(double), nc, stream));
    HIP_OK(hipEventRecord(ev[1], stream));
    if (oz) ystore_oz_run(0, n_local_, nc, S, ldx);
    else ystore_run(X, ldx, nf, nc, n_local_, S, ldx);
    HIP_OK(hipEventRecord(ev[2], stream));
    sync();
    float a = 0;
    HIP_OK(hipEventElapsedTime(&a, ev[1], ev[2]));
    if (kernel_ms) *kernel_ms = a;
    return S;
  }

  // JADE sweeps as one cooperative launch (jade_sweeps.inc): the np cumulant
  // matrices stay in the LDS of ≤ #CU workgroups for the whole run. Only when
  // they fit (n ≲ 66 on MI355X: np·npos·8 B over 256 CUs) and the device can
  // co-schedule the grid; otherwise the host runs the sweeps.
  bool jade_sweeps(const double* A, size_t n, size_t max_iter, double tol, double* v_out, JadeSweepLog* log) override {
    return jade_sweeps_impl(A, n, 0.0, max_iter, tol, v_out, log);
  }
  // the cumulant matrices from the M the last moments4 call left in d_chunk (m4_full_)
  bool jade_sweeps_moments(size_t n, double t, size_t max_iter, double tol, double* v_out,
                           JadeSweepLog* log) override {
    if (!m4_full_ || m4_nc_ != n) return false;
    return jade_sweeps_impl(nullptr, n, t, max_iter, tol, v_out, log);
  }
  // M of the last moments4 call, its pair lists (inside d_chunk; cleared by every other user)
  const double* m4_full_ = nullptr;
  const int *m4_pi_ = nullptr, *m4_pj_ = nullptr;
  size_t m4_nc_ = 0;
  bool jade_sweeps_impl(const double* A, size_t n, double t, size_t max_iter, double tol, double* v_out,
                        JadeSweepLog* log) {
    HIP_OK(hipSetDevice(device));
    if (n < 2 || n > 256) return false;
    const size_t np = n * (n + 1) / 2, npos = np;
    // matrices per workgroup fixed by the shape, not by this device's CU count: the g-sum
    // grouping (and so every angle's bits) is then the same on any device that can hold the
    // grid; one that cannot (fewer CUs, a partition) runs the host sweeps instead
    const size_t mw = (np + JS_MAX_WG - 1) / JS_MAX_WG;
    const size_t G = (np + mw - 1) / mw;
    const size_t lds = (npos * mw + 4) * sizeof(double);
    if (lds > 160 * 1024 || G > (size_t)n_cu || G > (size_t)JS_MAX_WG || (n - 2) * mw > (size_t)JS_ROT_ELEMS)
      return false;
    int coop = 0;
    HIP_OK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, device));
    if (!coop) return false;
    const int th = JS_THREADS;
    const void* kern = (const void*)k_jade_sweeps<JS_THREADS>;
    lds_attr(kern, (int)lds);
    int per_cu = 0;
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, th, lds));
    if ((size_t)per_cu * n_cu < G) return false;
    // A [npos][np] as the host built it; workgroup g loads matrices g·mw … g·mw + mw − 1
    std::vector<double> eye(n * n, 0.0);
    for (size_t i = 0; i < n; ++i) eye[i * n + i] = 1.0;
    // One context-owned buffer (ensure: kept across calls, freed with the context), so an
    // error anywhere below — a throwing HIP_OK, a refused launch — leaks nothing:
    // [A: npos·np][V: n·n][granules: 2·3·G {value, seq} pairs][θ log: cap + 1][sweep counts]
    const int theta_cap = (int)std::min<size_t>(max_iter / 10, 1u << 16);
    const size_t off_v = npos * np, off_g = off_v + n * n, off_th = off_g + 2 * G * 3 * 2,
                 off_sw = off_th + (size_t)theta_cap + 1, total = off_sw + 2;
    double* base = ensure(d_jade, cap_jade, total);
    double *d_a = base, *d_v = base + off_v, *d_g = base + off_g, *d_th = base + off_th;
    int* d_sw = (int*)(base + off_sw);
    // granule tags start at seq0 (0; PICARD_JADE_BAR_BASE presets it, a test hook:
    // the sweeps must not depend on it)
    unsigned long long seq0 = 0;
    if (const char* e = std::getenv("PICARD_JADE_BAR_BASE")) seq0 = std::strtoull(e, nullptr, 0);
    long long max_pairs = (long long)std::min<size_t>(jade_max_pairs(), (size_t)LLONG_MAX);
    HIP_OK(hipMemsetAsync(d_g, 0, 2 * G * 3 * 2 * sizeof(double), stream));  // tags 0 ≠ any seq ≥ seq0 + 1
    HIP_OK(hipMemsetAsync(d_sw, 0, 4 * sizeof(int), stream));  // sweeps, converged, stalled
    if (A) {
      HIP_OK(hipMemcpyAsync(d_a, A, npos * np * sizeof(double), hipMemcpyHostToDevice, stream));
    } else {
      k_jade_cumulants<<<(unsigned)((np * np + 255) / 256), 256, 0, stream>>>(m4_full_, m4_pi_, m4_pj_, (int)np, t, d_a);
      HIP_OK(hipGetLastError());
    }
    HIP_OK(hipMemcpyAsync(d_v, eye.data(), n * n * sizeof(double), hipMemcpyHostToDevice, stream));
    int np_i = (int)np, n_i = (int)n, npos_i = (int)npos, mw_i = (int)mw, it_i = (int)std::min<size_t>(max_iter, 1u << 30);
    double tol_d = tol;
    // The kernel needs its G workgroups co-resident (each waits for the others' granules;
    // jade_sweeps.inc), not a grid barrier: occupancy was checked above. A context alone on its
    // device launches it plainly; contexts that share the device (an in-process rank group, or
    // several contexts of one process) use the cooperative launch, whose admission guarantees
    // co-residency against each other's sweeps. (A rocprofv3-traced process that ran a
    // cooperative launch crashed in HIP's exit handler: DESIGN.md §6.) A plain launch that is
    // not co-resident after all (another process holding CUs) cannot hang: each workgroup's
    // wait is bounded (JS_POLL_CAP) and a stalled grid reports it. A refused launch is not
    // an error: the host sweeps run instead (PICARD_TEST_JADE_REFUSE=1 refuses every launch,
    // a test hook).
    const bool coop_launch = (coll_ && std::strcmp(coll_->kind(), "local") == 0) || ctxs_on_device(device) > 1;
    // test hooks of the bounded wait (jade_sweeps.inc): a lower poll cap, a withheld publish
    unsigned poll_cap = JS_POLL_CAP;
    int stall_wg = -1;
    if (const char* e = std::getenv("PICARD_TEST_JADE_POLL_CAP")) poll_cap = (unsigned)std::max(1L, std::atol(e));
    if (const char* e = std::getenv("PICARD_TEST_JADE_STALL")) stall_wg = std::atoi(e);
    hipError_t le = hipSuccess;
    if (std::getenv("PICARD_TEST_JADE_REFUSE") && std::atoi(std::getenv("PICARD_TEST_JADE_REFUSE")) != 0) {
      le = hipErrorCooperativeLaunchTooLarge;
    } else if (coop_launch) {
      void* args[] = {&d_a, &np_i, &n_i,  &npos_i, &mw_i, &it_i, &tol_d, &d_v,      &d_g,
                      &d_sw, &d_th, (void*)&theta_cap, &seq0, &max_pairs, &poll_cap, &stall_wg};
      le = hipLaunchCooperativeKernel(kern, dim3((unsigned)G), dim3((unsigned)th), args, (unsigned)lds, stream);
    } else {
      k_jade_sweeps<JS_THREADS><<<dim3((unsigned)G), dim3((unsigned)th), lds, stream>>>(
          d_a, np_i, n_i, npos_i, mw_i, it_i, tol_d, d_v, d_g, d_sw, d_th, theta_cap, seq0, max_pairs, poll_cap, stall_wg);
      le = hipGetLastError();
    }
    last_jade_coop_ = coop_launch;
    if (le != hipSuccess) {
      (void)hipGetLastError();
      sync();  // the queued copies into the buffer are done before it is reused
      return false;
    }
    int sw[3] = {0, 0, 0};
    HIP_OK(hipMemcpyAsync(v_out, d_v, n * n * sizeof(double), hipMemcpyDeviceToHost, stream));
    HIP_OK(hipMemcpyAsync(sw, d_sw, 3 * sizeof(int), hipMemcpyDeviceToHost, stream));
    sync();
    // a workgroup gave up waiting for the others' granules (the grid was not co-resident:
    // JS_POLL_CAP): V is partial, the host sweeps run instead
    if (sw[2] != 0) return false;
    log->sweeps = (size_t)sw[0];
    log->converged = sw[1] != 0;
    log->theta10.assign(std::min<size_t>(log->sweeps / 10, (size_t)theta_cap), 0.0);
    if (!log->theta10.empty())
      HIP_OK(hipMemcpy(log->theta10.data(), d_th, log->theta10.size() * sizeof(double), hipMemcpyDeviceToHost));
    return true;
  }
  bool last_jade_coop_ = false;

  // expm(a) (n × n) by k_expm_ps (expm.inc): the host matrix_exp's bits, or false (the caller
  // forms it on the host) for a shape or a series the kernel leaves to the host, a stalled grid,
  // or PICARD_DEVICE_EXPM=0. Tags of the grid barrier continue from the last call (xm_seq_).
  const bool device_expm_ = !(std::getenv("PICARD_DEVICE_EXPM") && std::atoi(std::getenv("PICARD_DEVICE_EXPM")) == 0);
  unsigned long long xm_seq_ = 0;
  size_t xm_n_ = 0;
  // below this n the host's products are faster than the kernel's latency-bound steps (measured:
  // n = 64 host 0.05 ms, device 0.12–0.14 ms); PICARD_DEVICE_EXPM_MIN_N overrides (the tests: 32)
  size_t xm_min_n_ = std::getenv("PICARD_DEVICE_EXPM_MIN_N") ? (size_t)std::atoi(std::getenv("PICARD_DEVICE_EXPM_MIN_N")) : 96;
  double* d_xm = nullptr; size_t cap_xm = 0;
  PinSlot pin_xm_, pin_xmo_{nullptr, 0, nullptr, false, hipHostMallocCoherent};
  uint64_t n_device_expm_ = 0;
  bool device_matrix_exp(const double* a, size_t n, double* out) override {
    if (!device_expm_ || n < xm_min_n_ || n > (size_t)XM_MAXN || n % 32 != 0) return false;
    HIP_OK(hipSetDevice(device));
    const size_t nn = n * n, G = (n / 32) * (n / 32);
    // device: [A | work: P1…P4, R0, R1 | granules: 2·3·G {value, tag}]; E and the status word are
    // stored by the kernel straight into coherent pinned host memory (no D2H copy on the timeline)
    const size_t off_w = nn, off_g = 7 * nn, total = off_g + 2 * 3 * G * 2;
    const size_t cap0 = cap_xm;
    double* base = ensure(d_xm, cap_xm, total);
    // a new buffer (or a new n: the granules moved) starts with tag 0 everywhere, below any seq0
    if (cap_xm != cap0 || n != xm_n_) HIP_OK(hipMemsetAsync(base + off_g, 0, 2 * 3 * G * 2 * sizeof(double), stream));
    xm_n_ = n;
    double* h = (double*)pin_acquire(pin_xm_, nn * sizeof(double));
    std::memcpy(h, a, nn * sizeof(double));
    HIP_OK(hipMemcpyAsync(base, h, nn * sizeof(double), hipMemcpyHostToDevice, stream));
    pin_release(pin_xm_);
    double* o = (double*)pin_acquire(pin_xmo_, (nn + 1) * sizeof(double));
    lds_attr((const void*)k_expm_ps, XM_LDS);
    const unsigned long long seq0 = xm_seq_ + 1;
    xm_seq_ += 128;  // more than the barriers of one call (≤ 65)
    HIP_OK(hipEventRecord(ev[1], stream));
    k_expm_ps<<<(unsigned)(8 * G), XM_THREADS, XM_LDS, stream>>>(base, (int)n, base + off_w, o, (int*)(o + nn),
                                                                 base + off_g, seq0, 1u << 20);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ev[2], stream));
    pin_release(pin_xmo_);
    sync();
    int st = 0;
    std::memcpy(&st, o + nn, sizeof(int));
    if (std::getenv("PICARD_TRACE_EXPM")) {
      float km = 0.f;
      HIP_OK(hipEventElapsedTime(&km, ev[1], ev[2]));
      std::fprintf(stderr, "[picard-expm] n %zu kernel %.3f ms status %d\n", n, km, st);
    }
    if (st != 0) {
      if (std::getenv("PICARD_TRACE"))
        std::fprintf(stderr, "[picard-expm] n %zu: device map declined (status %d: 1 = the host's series, 2 = stalled grid)\n", n, st);
      return false;
    }
    std::memcpy(out, o, nn * sizeof(double));
    ++n_device_expm_;
    return true;
  }
  double* d_jade = nullptr; size_t cap_jade = 0;  // the JADE sweeps' buffer (jade_sweeps_impl)

  void moments4(const double* w, size_t nc, const double* mu, double* out) override {
    HIP_OK(hipSetDevice(device));
    const int np = (int)(nc * (nc + 1) / 2);
    std::vector<int> pi(np), pj(np);
    {
      int q = 0;
      for (int i = 0; i < (int)nc; ++i)
        for (int j = i; j < (int)nc; ++j) { pi[q] = i; pj[q] = j; ++q; }
    }
    resident_mu(mu);  // X is centred in place: Y = W·X
    ystore_upload(w, nc, nf);
    const bool mfma_path = nc <= 64;  // larger nc: the VALU tile kernel (symmetric upper tiles)
    const uint64_t CH = mfma_path ? (1ull << 22) : (1ull << 16);
    // (R, C) pair orders and the staircase patches of k_moments4_patch
    std::vector<int> ri(np), rj(np), ci(np), cj(np);
    {
      int q = 0;
      for (int b = 0; b < (int)nc; ++b)
        for (int a = 0; a <= b; ++a) { ri[q] = a; rj[q] = b; ++q; }
      q = 0;
      for (int c = 0; c < (int)nc; ++c)
        for (int d = c; d < (int)nc; ++d) { ci[q] = c; cj[q] = d; ++q; }
    }
    const int nrg = (np + 63) / 64, nqc = (np + 31) / 32;
    std::vector<int> packs;
    std::vector<unsigned char> pmask((size_t)nrg * nqc, 0);
    for (int g = 0; g < nrg; ++g) {
      const int bmin = rj[g * 64];  // rows are ordered by b
      for (int h = 0; h < nqc; ++h) {
        const int cmax = ci[std::min(np, h * 32 + 32) - 1];  // columns by c
        if (bmin <= cmax) { packs.push_back(g << 16 | h); pmask[(size_t)g * nqc + h] = 1; }
      }
    }
    while (packs.size() % M4_PACK) packs.push_back(-1);  // idle waves
    const int npack = (int)(packs.size() / M4_PACK);
    // splits: the item count (npack · nsplit) that fills whole rounds of one workgroup
    // per CU best, at ≥ 2 rounds
    int nsplit = 1;
    if (mfma_path) {
      double best = -1;
      for (int s = 1; s <= 48; ++s) {
        const double items = (double)npack * s, rounds = std::ceil(items / n_cu);
        if (rounds < 2) continue;
        const double fill = items / (rounds * n_cu);
        if (fill > best + 1e-9) { best = fill; nsplit = s; }
      }
    }
    const size_t slab_stride = (size_t)np * np;
    auto dsz = [](size_t bytes) { return (bytes + sizeof(double) - 1) / sizeof(double); };
    const size_t ints = dsz((6 * (size_t)np + packs.size()) * sizeof(int) + pmask.size());
    const size_t need = nc * CH + (mfma_path ? 2 : 1) * (size_t)np * np + ints + (mfma_path ? nsplit * slab_stride : 0);
    m4_full_ = nullptr;
    double* Y = ensure(d_chunk, cap_chunk, need);
    double* acc = Y + nc * CH;
    double* full = mfma_path ? acc + (size_t)np * np : acc;  // the lexicographic M (fill target)
    int* dpi = reinterpret_cast<int*>(full + (size_t)np * np);
    int* dpj = dpi + np;
    int* dri = dpj + np;
    int* drj = dri + np;
    int* dci = drj + np;
    int* dcj = dci + np;
    int* dpk = dcj + np;
    unsigned char* dtm = reinterpret_cast<unsigned char*>(dpk + packs.size());
    double* slabs = full + (size_t)np * np + ints;
    HIP_OK(hipMemcpyAsync(dpi, pi.data(), np * sizeof(int), hipMemcpyHostToDevice, stream));
    HIP_OK(hipMemcpyAsync(dpj, pj.data(), np * sizeof(int), hipMemcpyHostToDevice, stream));
    HIP_OK(hipMemcpyAsync(dri, ri.data(), np * sizeof(int), hipMemcpyHostToDevice, stream));
    HIP_OK(hipMemcpyAsync(drj, rj.data(), np * sizeof(int), hipMemcpyHostToDevice, stream));
    HIP_OK(hipMemcpyAsync(dci, ci.data(), np * sizeof(int), hipMemcpyHostToDevice, stream));
    HIP_OK(hipMemcpyAsync(dcj, cj.data(), np * sizeof(int), hipMemcpyHostToDevice, stream));
    HIP_OK(hipMemcpyAsync(dpk, packs.data(), packs.size() * sizeof(int), hipMemcpyHostToDevice, stream));
    HIP_OK(hipMemcpyAsync(dtm, pmask.data(), pmask.size(), hipMemcpyHostToDevice, stream));
    HIP_OK(hipMemsetAsync(acc, 0, (size_t)np * np * sizeof(double), stream));
    // the host image vectors must outlive the async copies
    sync();
    const int tiles = (np + 31) / 32;
    bool first = true;
    for (uint64_t c0 = 0; c0 < n_local_; c0 += CH) {
      const uint64_t cn = std::min<uint64_t>(CH, n_local_ - c0);
      ystore_run(X + c0, ldx, nf, nc, cn, Y, CH);
      if (mfma_path) {
        const uint64_t n_stage = (cn + M4_STAGE - 1) / M4_STAGE;
        if (cn % M4_STAGE)  // the last stage reads zeros past cn (CH is a multiple of M4_STAGE)
          HIP_OK(hipMemset2DAsync(Y + cn, CH * sizeof(double), 0, (n_stage * M4_STAGE - cn) * sizeof(double), nc,
                                  stream));
        const uint64_t spb = (n_stage + nsplit - 1) / nsplit;
        const uint64_t per_xcd = ((uint64_t)npack * nsplit + 7) / 8;
        const size_t lds = (size_t)2 * M4_STAGE_DBL * sizeof(double);
        lds_attr((const void*)k_moments4_patch, (int)lds);
        k_moments4_patch<<<(unsigned)(8 * per_xcd), FUSED_THREADS, lds, stream>>>(
            Y, CH, n_stage, (int)nc, dri, drj, dci, dcj, np, dpk, npack, nsplit, spb, per_xcd, slabs, slab_stride);
        HIP_OK(hipGetLastError());
        k_moments4_reduce<<<(unsigned)(((size_t)np * np + 255) / 256), 256, 0, stream>>>(slabs, nsplit, slab_stride, np,
                                                                                         dtm, first ? 0 : 1, acc);
      } else {
        k_moments4<<<tiles * tiles, 256, 0, stream>>>(Y, CH, cn, (int)nc, dpi, dpj, np, acc);
      }
      HIP_OK(hipGetLastError());
      first = false;
    }
    allreduce(acc, (size_t)np * np, "moments4");
    if (mfma_path) {
      k_moments4_fill<<<(unsigned)(((size_t)np * np + 255) / 256), 256, 0, stream>>>(acc, dpi, dpj, (int)nc, np, full);
      HIP_OK(hipGetLastError());
    }
    HIP_OK(hipMemcpyAsync(out, full, (size_t)np * np * sizeof(double), hipMemcpyDeviceToHost, stream));
    sync();
    if (mfma_path) {  // the lexicographic M stays for jade_sweeps_moments (the VALU path fills one triangle)
      m4_full_ = full;
      m4_pi_ = dpi;
      m4_pj_ = dpj;
      m4_nc_ = nc;
    }
    if (!mfma_path)
      for (int p = 0; p < np; ++p)  // mirror the upper tiles
        for (int q = 0; q < p; ++q) out[(size_t)p * np + q] = out[(size_t)q * np + p];
  }

};

// factory + thin accessors used by capi.cpp
Evaluator* make_device_ctx(int device, int rank, int world, const char* uid, std::shared_ptr<LocalGroup> grp) {
  return new DeviceCtx(device, rank, world, uid, std::move(grp));
}
// [0] all-reduces issued, [1] capability agreements asked, [2] screen agreement, [3] kept-Y
// agreement (0 not asked, 1 every rank, -1 not every rank), [4] 1 if the group was aborted,
// [5] world size, [6] 1 RCCL / 2 in-process group / 0 none
void device_ctx_comm_stats(const Evaluator* e, int64_t* out) {
  auto* d = static_cast<const DeviceCtx*>(e);
  out[0] = d->coll_ ? (int64_t)d->coll_->n_allreduce : 0;
  out[1] = (int64_t)d->n_agree_;
  out[2] = d->screen_agreed_;
  out[3] = d->ybuf_agreed_;
  out[4] = d->coll_ && d->coll_->aborted() ? 1 : 0;
  out[5] = d->world;
  out[6] = !d->coll_ ? 0 : std::strcmp(d->coll_->kind(), "rccl") == 0 ? 1 : 2;
}
// [0..2] ms in hipMalloc / hipFree / hipMemGetInfo, [3..5] their counts, [6..8] the largest
// single call of each
void device_ctx_alloc_stats(const Evaluator* e, double* out) {
  auto* d = static_cast<const DeviceCtx*>(e);
  for (int k = 0; k < 3; ++k) {
    out[k] = d->as_.ms[k];
    out[3 + k] = (double)d->as_.n[k];
    out[6 + k] = d->as_.mx[k];
  }
}
void device_last_teardown(double* out) {
  std::lock_guard<std::mutex> lk(g_teardown_mu);
  for (int k = 0; k < 4; ++k) out[k] = g_teardown[k];
}
// [0] ms inside all-reduces (see DeviceCtx::allreduce), [1] all-reduces timed
void device_ctx_comm_timing(const Evaluator* e, double* out) {
  auto* d = static_cast<const DeviceCtx*>(e);
  out[0] = d->ar_ms_;
  out[1] = (double)d->ar_timed_;
}
// drop the HBM caches (int8 digit image, kept-Y buffer): later passes run without them
void device_ctx_release_caches(Evaluator* e) {
  auto* d = static_cast<DeviceCtx*>(e);
  HIP_OK(hipSetDevice(d->device));
  d->release_xsl();
  d->kept_nc = 0;  // a kept evaluation cannot be completed from a freed Y
  if (d->d_ybuf) {
    d->sync();
    HIP_OK(hipFree(d->d_ybuf));
    d->d_ybuf = nullptr;
    d->cap_ybuf = 0;
  }
  // the multi-try pass's y fragments: slot 1's buffer is freed, and neither slot may be read
  // again (slot 0 lives in d_tbuf, which stays allocated but is no longer a promised cache)
  if (d->d_ybuf2) {
    d->sync();
    HIP_OK(d->t_free(d->d_ybuf2));
    d->d_ybuf2 = nullptr;
    d->cap_ybuf2 = 0;
  }
  d->ytile_[0].valid = false;
  d->ytile_[1].valid = false;
}
void device_ctx_load(Evaluator* e, const double* x, uint64_t nf, uint64_t nl, uint64_t nt, uint64_t t0) {
  static_cast<DeviceCtx*>(e)->load(x, nf, nl, nt, t0);
}
void device_ctx_generate(Evaluator* e, uint64_t nf, uint64_t nt, uint64_t seed, double* a_out) {
  static_cast<DeviceCtx*>(e)->generate(nf, nt, seed, a_out);
}
void device_ctx_download(Evaluator* e, double* out) { static_cast<DeviceCtx*>(e)->download(out); }
const double* device_ctx_sources_resident(Evaluator* e, const double* w, size_t nc, const double* mu, double* ms,
                                          uint64_t* ld) {
  auto* d = static_cast<DeviceCtx*>(e);
  *ld = d->ldx;
  return d->sources_resident(w, nc, mu, ms);
}
uint64_t device_ctx_t0(const Evaluator* e) { return static_cast<const DeviceCtx*>(e)->t0; }
void device_ctx_timing(const Evaluator* e, double* k, double* c) {
  auto* d = static_cast<const DeviceCtx*>(e);
  *k = d->last_kernel_ms;
  *c = d->last_call_ms;
}
void device_ctx_kernel_stats(Evaluator* e, double* kernel_ms, double* call_ms, uint64_t* n, int reset) {
  auto* d = static_cast<DeviceCtx*>(e);
  *kernel_ms = d->sum_kernel_ms;
  *call_ms = d->sum_call_ms;
  *n = d->n_kernel;
  if (reset) { d->sum_kernel_ms = 0; d->sum_call_ms = 0; d->n_kernel = 0; }
}
void device_ctx_kernel_breakdown(Evaluator* e, double* ms, uint64_t* n, int reset) {
  auto* d = static_cast<DeviceCtx*>(e);
  ms[0] = d->sum_kernel_ms; n[0] = d->n_kernel;
  ms[1] = d->sum_loss_ms; n[1] = d->n_loss;
  ms[2] = d->sum_fromy_ms; n[2] = d->n_fromy;
  ms[3] = d->sum_multi_ms; n[3] = d->n_multi;
  if (reset) {
    d->sum_kernel_ms = d->sum_loss_ms = d->sum_fromy_ms = d->sum_split_ms = d->sum_call_ms = d->sum_multi_ms = 0;
    d->n_kernel = d->n_loss = d->n_fromy = d->n_split = d->n_multi = 0;
  }
}
void device_ctx_set_g_stage(Evaluator* e, int mode) { static_cast<DeviceCtx*>(e)->g_stage_ = mode; }
uint64_t device_ctx_g8_passes(const Evaluator* e) { return static_cast<const DeviceCtx*>(e)->n_g8_passes_; }
uint64_t device_ctx_multi_ybuf_passes(const Evaluator* e) {
  return static_cast<const DeviceCtx*>(e)->n_multi_ybuf_;
}
void device_ctx_set_y_stage(Evaluator* e, int mode) {
  auto* d = static_cast<DeviceCtx*>(e);
  d->y_stage_ = mode;
}
uint64_t device_ctx_int8_passes(const Evaluator* e) { return static_cast<const DeviceCtx*>(e)->n_int8_passes_; }
// the screen's statistical-bound inputs (tests): false without an int8 digit image
bool device_ctx_screen_digit_gram(Evaluator* e, double* lam, double* s4) {
  DeviceCtx* c = static_cast<DeviceCtx*>(e);
  if (!c->ensure_xsl() || !c->ensure_digit_gram()) return false;
  for (int b = 0; b < OZ_SLICES; ++b) lam[b] = c->xg_lam_[b];
  *s4 = c->xsc_s4_;
  return true;
}
void device_ctx_screen_stats(Evaluator* e, double* ms, uint64_t* n, int reset) {
  auto* d = static_cast<DeviceCtx*>(e);
  *ms = d->sum_screen_ms;
  *n = d->n_screen;
  if (reset) { d->sum_screen_ms = 0; d->n_screen = 0; d->n_screen_tries = 0; d->n_screen_products = 0; }
}
uint64_t device_ctx_screen_tries(const Evaluator* e) { return static_cast<const DeviceCtx*>(e)->n_screen_tries; }
uint64_t device_ctx_screen_products(const Evaluator* e) { return static_cast<const DeviceCtx*>(e)->n_screen_products; }
void device_check_f32_transc(int device, double* out4) {
  HIP_OK(hipSetDevice(device));
  const int nblk = 2048;
  double* d = nullptr;
  HIP_OK(hipMalloc(&d, nblk * 4 * sizeof(double)));
  k_check_f32_transc<<<nblk, 256>>>(d);
  HIP_OK(hipGetLastError());
  std::vector<double> h(nblk * 4);
  HIP_OK(hipMemcpy(h.data(), d, h.size() * sizeof(double), hipMemcpyDeviceToHost));
  (void)hipFree(d);
  out4[0] = out4[1] = out4[2] = 0.0;
  out4[3] = 1.0;
  for (int b = 0; b < nblk; ++b) {
    for (int c = 0; c < 3; ++c) out4[c] = std::max(out4[c], h[b * 4 + c]);
    out4[3] = std::min(out4[3], h[b * 4 + 3]);
  }
}
void device_synchronize(int device) {
  HIP_OK(hipSetDevice(device));
  HIP_OK(hipDeviceSynchronize());
}
void device_mem_info(int device, uint64_t* free_b, uint64_t* total_b) {
  HIP_OK(hipSetDevice(device));
  size_t f = 0, t = 0;
  HIP_OK(hipMemGetInfo(&f, &t));
  if (free_b) *free_b = f;
  if (total_b) *total_b = t;
}
void device_ctx_raw_eval(Evaluator* e, const double* w, size_t nc, const double* mu, int dens, double alpha,
                         bool need_h, double* stats) {
  static_cast<DeviceCtx*>(e)->run_eval(w, nc, mu, dens, alpha, need_h, stats);
}

}  // namespace pcamd
