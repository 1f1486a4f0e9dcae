// The scalar part of matrix_exp (math.rs:38-74, host_linalg.cpp): the scaling exponent and the
// Paterson–Stockmeyer plan (extra halvings t, Taylor degree m) chosen from the ∞-norms of
// B … B⁴. Shared by the host (matrix_exp) and the device (k_expm_ps, expm.inc): the functions
// are constexpr, which hipcc compiles for both sides, and every operation is one IEEE operation
// in the order written (neither caller fuses them: the host has no FMA in generic code, the
// device kernel turns contraction off), so both sides make the same choice from the same norms.
#pragma once

namespace pcamd {

// 2^e, exact for −1074 ≤ e ≤ 1023 (products of powers of two)
constexpr double pc_pow2(int e) {
  double r = 1.0, b = e >= 0 ? 2.0 : 0.5;
  for (int k = e >= 0 ? e : -e; k > 0; --k) r *= b;
  return r;
}

// ceil(log2 x) for 1e-300 < x < 1e300, exactly (a power of two gives its own exponent)
constexpr int pc_ceil_log2(double x) {
  int e = 0;
  double p = 1.0;  // p = 2^e
  while (p < x) { p *= 2.0; ++e; }
  while (p * 0.5 >= x) { p *= 0.5; --e; }
  return e;  // 2^(e-1) < x ≤ 2^e
}

struct ExpmPlan {
  bool converged;  // the reference's 30-term series converges: Paterson–Stockmeyer with (t, m)
  int t, m;
};

constexpr int EXPM_KMAX = 90, EXPM_TMAX = 6;

// tails[m] = Σ_{k>m} bound(k)/k! at scale 2^-t (m = 0 … 31), ‖B^k‖ ≤ ν_4^⌊k/4⌋·ν_(k mod 4), for
// nu[k] = ‖B^k‖∞ (k = 1 … 4; nu[0] = 1) of B = A / 2^s. One t per call: the device forms the
// seven rows in parallel.
constexpr void expm_tails(const double (&nu)[5], int t, double (&tails)[32]) {
  const double f = pc_pow2(-t);
  const double fr[4] = {1.0, f, f * f, f * f * f};
  const double b4 = nu[4] * fr[2] * fr[2];
  double term[EXPM_KMAX + 1] = {};
  double inv_fact = 1.0, p4 = 1.0;
  for (int k = 1; k <= EXPM_KMAX; ++k) {
    inv_fact /= (double)k;
    if (k % 4 == 0) p4 *= b4;
    term[k] = p4 * nu[k % 4] * fr[k % 4] * inv_fact;
    if (k % 4 == 3 && p4 * inv_fact < 1e-250) break;  // the rest is negligible (and no subnormals)
  }
  double sum = 0.0;
  for (int k = EXPM_KMAX; k > 31; --k) sum += term[k];
  for (int m = 31; m >= 0; --m) {
    tails[m] = sum;
    if (m > 0) sum += term[m];
  }
}

// the plan from the tails of t = 0 … EXPM_TMAX
constexpr ExpmPlan expm_select(double nu4, const double (&tails)[EXPM_TMAX + 1][32]) {
  ExpmPlan p{false, 0, 30};
  const bool finite = nu4 - nu4 == 0.0;  // not NaN, not ±inf
  if (!(finite && tails[0][30] < 1e-17)) return p;
  p.converged = true;
  int best_cost = 1 << 30;
  for (int tt = 0; tt <= EXPM_TMAX; ++tt)
    for (int mm = 1; mm <= 30; ++mm)
      if (tails[tt][mm] < 1e-17) {
        if (mm / 4 + tt < best_cost) best_cost = mm / 4 + tt, p.t = tt, p.m = mm;
        break;
      }
  return p;
}

constexpr ExpmPlan expm_plan(const double (&nu)[5]) {
  double tails[EXPM_TMAX + 1][32] = {};
  for (int t = 0; t <= EXPM_TMAX; ++t) expm_tails(nu, t, tails[t]);
  return expm_select(nu[4], tails);
}

}  // namespace pcamd
