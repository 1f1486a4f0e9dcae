// Host N×N linear algebra; see host_linalg.hpp.
#include "host_linalg.hpp"
#include "expm_plan.hpp"

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>

namespace pcamd {

// C = A·B for the small dense N×N products of the host driver (matrix_exp's
// 30-term Taylor series is the biggest user: ~40 products of N×N per line-search
// try). Register-blocked 4 rows × 32 columns with fma, every element summed over
// p in increasing order (so any thread count gives the same bits, as the
// lockstep multi-rank drivers require). Compiled for AVX-512 and AVX2 (both
// with FMA) plus a plain fallback; the variant is picked once from cpuid.
namespace {
constexpr size_t MB = 4, NBW = 32;

#define PC_MM_BLOCK_BODY                                                           \
  double acc[MB][NBW] = {};                                                        \
  for (size_t p = 0; p < k; ++p) {                                                 \
    const double* bp = B + p * m + j0;                                             \
    for (size_t r = 0; r < MB; ++r) {                                              \
      const double a = A[(i0 + r) * k + p];                                       \
      for (size_t j = 0; j < NBW; ++j) acc[r][j] = __builtin_fma(a, bp[j], acc[r][j]); \
    }                                                                              \
  }                                                                                \
  for (size_t r = 0; r < MB; ++r)                                                  \
    for (size_t j = 0; j < NBW; ++j) C[(i0 + r) * m + j0 + j] = acc[r][j];

__attribute__((target("avx512f,avx512vl,fma"))) void mm_block_avx512(const double* A, const double* B, double* C,
                                                                     size_t k, size_t m, size_t i0, size_t j0) {
  PC_MM_BLOCK_BODY
}
__attribute__((target("avx2,fma"))) void mm_block_avx2(const double* A, const double* B, double* C, size_t k,
                                                        size_t m, size_t i0, size_t j0) {
  PC_MM_BLOCK_BODY
}
void mm_block_plain(const double* A, const double* B, double* C, size_t k, size_t m, size_t i0, size_t j0) {
  PC_MM_BLOCK_BODY
}
#undef PC_MM_BLOCK_BODY

using mm_block_fn = void (*)(const double*, const double*, double*, size_t, size_t, size_t, size_t);
mm_block_fn pick_mm_block() {
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("fma"))
    return mm_block_avx512;
  if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) return mm_block_avx2;
  return mm_block_plain;
}
const mm_block_fn mm_block = pick_mm_block();

void mm_edge(const double* A, const double* B, double* C, size_t k, size_t m, size_t i0, size_t i1, size_t j0,
             size_t j1) {
  for (size_t i = i0; i < i1; ++i)
    for (size_t j = j0; j < j1; ++j) {
      double s = 0.0;
      for (size_t p = 0; p < k; ++p) s += A[i * k + p] * B[p * m + j];
      C[i * m + j] = s;
    }
}
// ---- JADE sweep kernels (host_solver.cpp: Solver::jade), same dispatch ----
#define PC_GIVENS_BODY                                   \
  for (size_t m = 0; m < len; ++m) {                     \
    const double x = a[m], y = b[m];                     \
    a[m] = c * x - s * y;                                \
    b[m] = s * x + c * y;                                \
  }
__attribute__((target("avx512f,avx512vl"))) void givens_avx512(double* a, double* b, size_t len, double c, double s) {
  PC_GIVENS_BODY
}
__attribute__((target("avx2"))) void givens_avx2(double* a, double* b, size_t len, double c, double s) {
  PC_GIVENS_BODY
}
void givens_plain(double* a, double* b, size_t len, double c, double s) { PC_GIVENS_BODY }
#undef PC_GIVENS_BODY

// g-sums over 8 fixed lanes (m mod 8), combined in a fixed order: the same
// value whichever instruction set runs it
#define PC_GSUM_BODY                                                          \
  double s00[8] = {}, s01[8] = {}, s11[8] = {};                              \
  size_t m = 0;                                                               \
  for (; m + 8 <= len; m += 8)                                                \
    for (int j = 0; j < 8; ++j) {                                             \
      const double hpq = apq[m + j] + apq[m + j], hd = app[m + j] - aqq[m + j]; \
      s00[j] += hpq * hpq;                                                    \
      s01[j] += hpq * hd;                                                     \
      s11[j] += hd * hd;                                                      \
    }                                                                         \
  for (int j = 0; m < len; ++m, ++j) {                                        \
    const double hpq = apq[m] + apq[m], hd = app[m] - aqq[m];                 \
    s00[j] += hpq * hpq;                                                      \
    s01[j] += hpq * hd;                                                       \
    s11[j] += hd * hd;                                                        \
  }                                                                           \
  g[0] = ((s00[0] + s00[1]) + (s00[2] + s00[3])) + ((s00[4] + s00[5]) + (s00[6] + s00[7])); \
  g[1] = ((s01[0] + s01[1]) + (s01[2] + s01[3])) + ((s01[4] + s01[5]) + (s01[6] + s01[7])); \
  g[2] = ((s11[0] + s11[1]) + (s11[2] + s11[3])) + ((s11[4] + s11[5]) + (s11[6] + s11[7]));
__attribute__((target("avx512f,avx512vl"))) void gsum_avx512(const double* apq, const double* app,
                                                             const double* aqq, size_t len, double* g) {
  PC_GSUM_BODY
}
__attribute__((target("avx2"))) void gsum_avx2(const double* apq, const double* app, const double* aqq, size_t len,
                                              double* g) {
  PC_GSUM_BODY
}
void gsum_plain(const double* apq, const double* app, const double* aqq, size_t len, double* g) { PC_GSUM_BODY }
#undef PC_GSUM_BODY

using givens_fn = void (*)(double*, double*, size_t, double, double);
using gsum_fn = void (*)(const double*, const double*, const double*, size_t, double*);
const givens_fn givens_impl = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl")
                                  ? givens_avx512
                                  : __builtin_cpu_supports("avx2") ? givens_avx2 : givens_plain;
const gsum_fn gsum_impl = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl")
                              ? gsum_avx512
                              : __builtin_cpu_supports("avx2") ? gsum_avx2 : gsum_plain;
}  // namespace

void givens_rows(double* a, double* b, size_t len, double c, double s) { givens_impl(a, b, len, c, s); }
void jade_gsums(const double* apq, const double* app, const double* aqq, size_t len, double* g) {
  gsum_impl(apq, app, aqq, len, g);
}

Mat matmul(const Mat& a, const Mat& b) {
  Mat c(a.rows, b.cols);
  const size_t n = a.rows, k = a.cols, m = b.cols;
  const double* A = a.data();
  const double* B = b.data();
  double* C = c.data();
  if (m < NBW) {  // tiny (C1-sized) products: plain i-k-j
    for (size_t i = 0; i < n; ++i)
      for (size_t p = 0; p < k; ++p) {
        const double aip = A[i * k + p];
        for (size_t j = 0; j < m; ++j) C[i * m + j] += aip * B[p * m + j];
      }
    return c;
  }
  const size_t nb = n / MB, mb = m / NBW;
  const long tiles = (long)(nb * mb);
#pragma omp parallel if (n * k * m > (1u << 20))
  {
#pragma omp for schedule(static) nowait
    for (long t = 0; t < tiles; ++t) mm_block(A, B, C, k, m, (size_t)(t / mb) * MB, (size_t)(t % mb) * NBW);
#pragma omp single nowait
    {
      if (mb * NBW < m) mm_edge(A, B, C, k, m, 0, nb * MB, mb * NBW, m);
      if (nb * MB < n) mm_edge(A, B, C, k, m, nb * MB, n, 0, m);
    }
  }
  return c;
}

Mat transpose(const Mat& a) {
  Mat t(a.cols, a.rows);
  for (size_t i = 0; i < a.rows; ++i)
    for (size_t j = 0; j < a.cols; ++j) t(j, i) = a(i, j);
  return t;
}

Mat matmul_nt(const Mat& a, const Mat& b) { return matmul(a, transpose(b)); }

Mat add(const Mat& a, const Mat& b) {
  Mat c = a;
  for (size_t i = 0; i < c.a.size(); ++i) c.a[i] += b.a[i];
  return c;
}

Mat sub(const Mat& a, const Mat& b) {
  Mat c = a;
  for (size_t i = 0; i < c.a.size(); ++i) c.a[i] -= b.a[i];
  return c;
}

Mat scale(const Mat& a, double s) {
  Mat c = a;
  for (double& v : c.a) v *= s;
  return c;
}

double max_abs(const Mat& a) {
  // fold(0.0, f64::max): NaN entries are skipped by f64::max (core.rs:289)
  // (f > m ? f : m) is fmax here: m starts at 0 and never becomes NaN, and a NaN f
  // compares false. Unlike std::fmax it is inlined (no libm call per element).
  double m = 0.0;
  for (double v : a.a) {
    const double f = std::fabs(v);
    m = f > m ? f : m;
  }
  return m;
}

double dot_sum(const Mat& a, const Mat& b) {
  // (a * b).sum() of the reference: ndarray sums a contiguous array in 8 interleaved partial
  // sums (numeric_util::unrolled_fold), combined as ((((0 + (p0+p4)) + (p1+p5)) + (p2+p6)) +
  // (p3+p7)), then the < 8 remaining elements in order. Eight independent chains instead of one
  // dependent add per element (the L-BFGS recursion takes 2m of these per iteration).
  const double* x = a.data();
  const double* y = b.data();
  const size_t n = a.a.size();
  double p[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  size_t i = 0;
  for (; i + 8 <= n; i += 8)
    for (int j = 0; j < 8; ++j) p[j] += x[i + j] * y[i + j];
  double s = 0.0;
  s = s + (p[0] + p[4]);
  s = s + (p[1] + p[5]);
  s = s + (p[2] + p[6]);
  s = s + (p[3] + p[7]);
  for (; i < n; ++i) s += x[i] * y[i];
  return s;
}

namespace {
// Householder tridiagonalisation + implicit QL with shifts (the EISPACK
// tred2/tql2 pair, as in LAPACK's dsteqr path that ndarray-linalg's eigh
// reaches): O(n³) with a small constant — the cyclic Jacobi below costs
// ~1.2 s at n = 256 (BASELINE C4's whitening and w_init decorrelation).
// v: row-major n×n, in = symmetric matrix, out = eigenvectors (columns);
// d = eigenvalues (unsorted).
void eigh_tridiag_ql(std::vector<double>& v, size_t n, std::vector<double>& d) {
  std::vector<double> e(n, 0.0);
  d.assign(n, 0.0);
  auto V = [&](size_t r, size_t c) -> double& { return v[r * n + c]; };
  for (size_t j = 0; j < n; ++j) d[j] = V(n - 1, j);
  for (size_t i = n - 1; i > 0; --i) {  // tred2
    double scale = 0.0, h = 0.0;
    for (size_t k = 0; k < i; ++k) scale += std::fabs(d[k]);
    if (scale == 0.0) {
      e[i] = d[i - 1];
      for (size_t j = 0; j < i; ++j) {
        d[j] = V(i - 1, j);
        V(i, j) = 0.0;
        V(j, i) = 0.0;
      }
    } else {
      for (size_t k = 0; k < i; ++k) {
        d[k] /= scale;
        h += d[k] * d[k];
      }
      double f = d[i - 1];
      double g = std::sqrt(h);
      if (f > 0) g = -g;
      e[i] = scale * g;
      h -= f * g;
      d[i - 1] = f - g;
      for (size_t j = 0; j < i; ++j) e[j] = 0.0;
      for (size_t j = 0; j < i; ++j) {
        f = d[j];
        V(j, i) = f;
        g = e[j] + V(j, j) * f;
        for (size_t k = j + 1; k < i; ++k) {
          g += V(k, j) * d[k];
          e[k] += V(k, j) * f;
        }
        e[j] = g;
      }
      f = 0.0;
      for (size_t j = 0; j < i; ++j) {
        e[j] /= h;
        f += e[j] * d[j];
      }
      const double hh = f / (h + h);
      for (size_t j = 0; j < i; ++j) e[j] -= hh * d[j];
      for (size_t j = 0; j < i; ++j) {
        f = d[j];
        g = e[j];
        for (size_t k = j; k < i; ++k) V(k, j) -= (f * e[k] + g * d[k]);
        d[j] = V(i - 1, j);
        V(i, j) = 0.0;
      }
    }
    d[i] = h;
  }
  for (size_t i = 0; i + 1 < n; ++i) {  // accumulate the transformations
    V(n - 1, i) = V(i, i);
    V(i, i) = 1.0;
    const double h = d[i + 1];
    if (h != 0.0) {
      for (size_t k = 0; k <= i; ++k) d[k] = V(k, i + 1) / h;
      for (size_t j = 0; j <= i; ++j) {
        double g = 0.0;
        for (size_t k = 0; k <= i; ++k) g += V(k, i + 1) * V(k, j);
        for (size_t k = 0; k <= i; ++k) V(k, j) -= g * d[k];
      }
    }
    for (size_t k = 0; k <= i; ++k) V(k, i + 1) = 0.0;
  }
  for (size_t j = 0; j < n; ++j) {
    d[j] = V(n - 1, j);
    V(n - 1, j) = 0.0;
  }
  V(n - 1, n - 1) = 1.0;
  e[0] = 0.0;
  // tql2 on a column-major copy (rotations touch two contiguous columns)
  std::vector<double> z(n * n);
  for (size_t r = 0; r < n; ++r)
    for (size_t c = 0; c < n; ++c) z[c * n + r] = V(r, c);
  for (size_t i = 1; i < n; ++i) e[i - 1] = e[i];
  e[n - 1] = 0.0;
  double f = 0.0, tst1 = 0.0;
  const double eps = std::ldexp(1.0, -52);
  for (size_t l = 0; l < n; ++l) {
    tst1 = std::fmax(tst1, std::fabs(d[l]) + std::fabs(e[l]));
    size_t m = l;
    while (m < n) {
      if (std::fabs(e[m]) <= eps * tst1) break;
      ++m;
    }
    if (m == n) m = n - 1;
    if (m > l) {
      int iter = 0;
      do {
        if (++iter > 60) break;
        double g = d[l];
        double p = (d[l + 1] - g) / (2.0 * e[l]);
        double r = std::hypot(p, 1.0);
        if (p < 0) r = -r;
        d[l] = e[l] / (p + r);
        d[l + 1] = e[l] * (p + r);
        const double dl1 = d[l + 1];
        double h = g - d[l];
        for (size_t i = l + 2; i < n; ++i) d[i] -= h;
        f += h;
        p = d[m];
        double c = 1.0, c2 = c, c3 = c, s = 0.0, s2 = 0.0;
        const double el1 = e[l + 1];
        for (size_t ii = m; ii-- > l;) {
          c3 = c2;
          c2 = c;
          s2 = s;
          g = c * e[ii];
          h = c * p;
          r = std::hypot(p, e[ii]);
          e[ii + 1] = s * r;
          s = e[ii] / r;
          c = p / r;
          p = c * d[ii] - s * g;
          d[ii + 1] = h + s * (c * g + s * d[ii]);
          double* zi = z.data() + ii * n;
          double* zi1 = zi + n;
          for (size_t k = 0; k < n; ++k) {
            h = zi1[k];
            zi1[k] = s * zi[k] + c * h;
            zi[k] = c * zi[k] - s * h;
          }
        }
        p = -s * s2 * c3 * el1 * e[l] / dl1;
        e[l] = s * p;
        d[l] = c * p;
      } while (std::fabs(e[l]) > eps * tst1);
    }
    d[l] += f;
    e[l] = 0.0;
  }
  for (size_t r = 0; r < n; ++r)
    for (size_t c = 0; c < n; ++c) V(r, c) = z[c * n + r];
}
}  // namespace

void eigh(const Mat& s_in, std::vector<double>* vals, Mat* vecs) {
  const size_t n = s_in.rows;
  if (n > 64) {  // symmetrised from the lower triangle (UPLO::Lower, math.rs:16)
    std::vector<double> v(n * n), d;
    for (size_t i = 0; i < n; ++i)
      for (size_t j = 0; j < n; ++j) v[i * n + j] = i >= j ? s_in(i, j) : s_in(j, i);
    eigh_tridiag_ql(v, n, d);
    std::vector<size_t> order(n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return d[x] < d[y]; });
    vals->assign(n, 0.0);
    *vecs = Mat(n, n);
    for (size_t c = 0; c < n; ++c) {
      (*vals)[c] = d[order[c]];
      for (size_t r = 0; r < n; ++r) (*vecs)(r, c) = v[r * n + order[c]];
    }
    return;
  }
  // n ≤ 64: cyclic Jacobi (milliseconds; small eigenvalues to high relative accuracy)
  Mat a = s_in;
  // symmetrise from the lower triangle (UPLO::Lower, math.rs:16)
  for (size_t i = 0; i < n; ++i)
    for (size_t j = i + 1; j < n; ++j) a(i, j) = a(j, i);
  Mat v = Mat::eye(n);
  for (int sweep = 0; sweep < 100; ++sweep) {
    double off = 0.0, diag = 0.0;
    for (size_t i = 0; i < n; ++i) {
      diag += a(i, i) * a(i, i);
      for (size_t j = i + 1; j < n; ++j) off += a(i, j) * a(i, j);
    }
    if (off <= 1e-32 * diag || off == 0.0) break;
    for (size_t p = 0; p < n; ++p) {
      for (size_t q = p + 1; q < n; ++q) {
        const double apq = a(p, q);
        if (apq == 0.0) continue;
        const double app = a(p, p), aqq = a(q, q);
        if (std::fabs(apq) < 1e-300) { a(p, q) = a(q, p) = 0.0; continue; }
        const double theta = (aqq - app) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0);
        const double sn = t * c;
        for (size_t k = 0; k < n; ++k) {
          const double akp = a(k, p), akq = a(k, q);
          a(k, p) = c * akp - sn * akq;
          a(k, q) = sn * akp + c * akq;
        }
        for (size_t k = 0; k < n; ++k) {
          const double apk = a(p, k), aqk = a(q, k);
          a(p, k) = c * apk - sn * aqk;
          a(q, k) = sn * apk + c * aqk;
        }
        a(p, q) = a(q, p) = 0.0;
        for (size_t k = 0; k < n; ++k) {
          const double vkp = v(k, p), vkq = v(k, q);
          v(k, p) = c * vkp - sn * vkq;
          v(k, q) = sn * vkp + c * vkq;
        }
      }
    }
  }
  std::vector<size_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return a(x, x) < a(y, y); });
  vals->assign(n, 0.0);
  *vecs = Mat(n, n);
  for (size_t c = 0; c < n; ++c) {
    (*vals)[c] = a(order[c], order[c]);
    for (size_t r = 0; r < n; ++r) (*vecs)(r, c) = v(r, order[c]);
  }
}

bool sym_decorrelation(const Mat& w, Mat* out) {
  Mat ww_t = matmul_nt(w, w);
  std::vector<double> ev;
  Mat u;
  eigh(ww_t, &ev, &u);
  double mn = std::numeric_limits<double>::infinity();
  for (double e : ev) mn = std::fmin(mn, e);
  if (mn < 1e-10) return false;
  Mat scaled = u;
  for (size_t r = 0; r < u.rows; ++r)
    for (size_t c = 0; c < u.cols; ++c) scaled(r, c) *= 1.0 / std::sqrt(ev[c]);
  *out = matmul(matmul_nt(scaled, u), w);
  return true;
}

static double norm_inf(const Mat& m) {  // max row sum (contiguous rows)
  double r = 0.0;
  for (size_t i = 0; i < m.rows; ++i) {
    const double* p = m.data() + i * m.cols;
    double s = 0.0;
    for (size_t j = 0; j < m.cols; ++j) s += std::fabs(p[j]);
    r = std::fmax(r, s);
  }
  return r;
}

Mat matrix_exp(const Mat& a) {
  const size_t n = a.rows;
  const double norm = max_abs(a);
  if (norm < 1e-15) return Mat::eye(n);
  // s = max(⌈log2 ‖A‖max⌉, 0), exactly (expm_plan.hpp: the device map k_expm_ps makes the same choice)
  const int s = std::max(pc_ceil_log2(norm), 0);
  const double sc = std::ldexp(1.0, s);
  Mat as = a;
  for (double& v : as.a) v /= sc;
  // math.rs:38-74 sums the series term by term until max|term| < 1e-16 (at most 30 terms), then
  // squares s times. Where that series converges within its 30 terms it is exp(as) to rounding,
  // and the same value comes from far fewer products (Paterson–Stockmeyer):
  // * the powers B^1 … B^4 of B = as (3 products) and their ∞-norms ν_k bound every power,
  //   ‖B^k‖ ≤ ν_4^⌊k/4⌋·ν_(k mod 4) — for the skew-symmetric directions of the orthogonal
  //   search (normal matrices) ν_4^(1/4) is close to the spectral radius, far below ‖B‖;
  // * the series converged if Σ_{k>30} ‖B^k‖/k! < 1e-17 by that bound; otherwise the reference
  //   stops at its 30-term cap short of exp(as), and the term-by-term loop below restates that
  //   truncated value;
  // * else halve B t more times (its powers scale exactly by 2^-kt) and pick the degree m whose
  //   remainder bound is below 1e-17, (t, m) minimising ⌊m/4⌋ + t products: a Horner recursion
  //   in B^4 over blocks Σ_{i<4} B^i/(4j+i)!, then s + t squarings. The powers of two 2^-it are
  //   folded into the block coefficients and the Horner step (exact).
  //   The plan (t, m) is expm_plan (expm_plan.hpp), shared with the device.
  std::vector<Mat> pw(5);
  pw[1] = as;
  double nu[5] = {1.0, norm_inf(as), 0.0, 0.0, 0.0};
  for (int k = 2; k <= 4; ++k) {
    pw[k] = matmul(pw[k - 1], as);
    nu[k] = norm_inf(pw[k]);
  }
  const ExpmPlan plan = expm_plan(nu);
  if (plan.converged) {
    const int t = plan.t, m = plan.m;
    // B̃ = 2^-t·B: B̃^(4j+i) = (f4·B^4)^j·f^i·B^i, so R_nb = block_nb and R_j = R_(j+1)·(f4·B^4) +
    // block_j with block_j = Σ_{i<4, 4j+i ≤ m} f^i/(4j+i)!·B^i (B^0 = I)
    const double f = std::ldexp(1.0, -t), f4 = std::ldexp(1.0, -4 * t);
    std::vector<double> cf(m + 1);  // 1/k!
    cf[0] = 1.0;
    for (int k = 1; k <= m; ++k) cf[k] = cf[k - 1] / (double)k;
    // R ← g·R + block_j in one sweep (g = f4 after a Horner product, else 1)
    auto add_block = [&](Mat& r, int j, double g) {
      double ci[4] = {0.0, 0.0, 0.0, 0.0}, fi = 1.0;
      for (int i = 0; i < 4 && 4 * j + i <= m; ++i, fi *= f) ci[i] = cf[4 * j + i] * fi;
      double* o = r.data();
      const double *p1 = pw[1].data(), *p2 = pw[2].data(), *p3 = pw[3].data();
      for (size_t e = 0; e < n * n; ++e) o[e] = g * o[e] + (ci[1] * p1[e] + ci[2] * p2[e] + ci[3] * p3[e]);
      for (size_t d = 0; d < n; ++d) o[d * n + d] += ci[0];
    };
    const int nb = m / 4;
    Mat result(n, n);
    int j = nb;
    if (m % 4 == 0) {  // the top block is cf[m]·I: R_(nb−1) = cf[m]·f4·B^4 + block_(nb−1), no product
      const double top = cf[m] * f4;
      for (size_t e = 0; e < n * n; ++e) result.a[e] = top * pw[4].a[e];
      --j;
    }
    add_block(result, j, 1.0);
    for (--j; j >= 0; --j) {
      result = matmul(result, pw[4]);
      add_block(result, j, f4);
    }
    for (int i = 0; i < s + t; ++i) result = matmul(result, result);
    return result;
  }
  Mat result = Mat::eye(n), term = Mat::eye(n);
  for (int k = 1; k <= 30; ++k) {
    term = matmul(term, as);
    // term /= k; result += term; max|term| — one sweep, same per-element operations, split
    // over the threads (16K divisions per term at N=128 outweighed the threaded product;
    // the max of the per-thread maxima is exact in any order, none of them is NaN).
    const double kd = (double)k;
    double m = 0.0;
    const long ne = (long)term.a.size();
#pragma omp parallel for schedule(static) reduction(max : m) if (ne >= 8192)
    for (long i = 0; i < ne; ++i) {
      const double v = term.a[i] / kd;
      term.a[i] = v;
      result.a[i] += v;
      const double f = std::fabs(v);
      m = f > m ? f : m;
    }
    if (m < 1e-16) break;
  }
  for (int i = 0; i < s; ++i) result = matmul(result, result);
  return result;
}

void sln_det(const Mat& m, double* sign, double* logabs) {
  const size_t n = m.rows;
  Mat lu = m;
  double sg = 1.0, la = 0.0;
  for (size_t k = 0; k < n; ++k) {
    size_t piv = k;
    double best = std::fabs(lu(k, k));
    for (size_t i = k + 1; i < n; ++i)
      if (std::fabs(lu(i, k)) > best) { best = std::fabs(lu(i, k)); piv = i; }
    if (best == 0.0) { *sign = 0.0; *logabs = -std::numeric_limits<double>::infinity(); return; }
    if (piv != k) {
      for (size_t j = 0; j < n; ++j) std::swap(lu(k, j), lu(piv, j));
      sg = -sg;
    }
    const double d = lu(k, k);
    for (size_t i = k + 1; i < n; ++i) {
      const double f = lu(i, k) / d;
      lu(i, k) = f;
      for (size_t j = k + 1; j < n; ++j) lu(i, j) -= f * lu(k, j);
    }
  }
  for (size_t k = 0; k < n; ++k) {
    const double d = lu(k, k);
    if (d < 0) sg = -sg;
    la += std::log(std::fabs(d));
  }
  *sign = sg;
  *logabs = la;
}

Mat skew_symmetric(const Mat& a) {
  Mat r(a.rows, a.cols);
  for (size_t i = 0; i < a.rows; ++i)
    for (size_t j = 0; j < a.cols; ++j) r(i, j) = (a(i, j) - a(j, i)) / 2.0;
  return r;
}

bool invert_matrix(const Mat& m, Mat* out) {
  const size_t n = m.rows;
  if (n != m.cols) return false;
  Mat aug(n, 2 * n);
  for (size_t i = 0; i < n; ++i) {
    for (size_t j = 0; j < n; ++j) aug(i, j) = m(i, j);
    aug(i, n + i) = 1.0;
  }
  for (size_t i = 0; i < n; ++i) {
    size_t max_row = i;
    for (size_t k = i + 1; k < n; ++k)
      if (std::fabs(aug(k, i)) > std::fabs(aug(max_row, i))) max_row = k;
    for (size_t j = 0; j < 2 * n; ++j) std::swap(aug(i, j), aug(max_row, j));
    if (std::fabs(aug(i, i)) < 1e-15) return false;
    const double pivot = aug(i, i);
    for (size_t j = 0; j < 2 * n; ++j) aug(i, j) /= pivot;
    for (size_t k = 0; k < n; ++k) {
      if (k == i) continue;
      const double f = aug(k, i);
      for (size_t j = 0; j < 2 * n; ++j) aug(k, j) -= f * aug(i, j);
    }
  }
  *out = Mat(n, n);
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) (*out)(i, j) = aug(i, n + j);
  return true;
}

// W's radix-256 digits for the int8 Y stage (DeviceCtx::upload_wsl, ozaki.inc "Layout"): per
// row i, scale sc[i] = 2^(f_i − 12) with max_k |w_ik| < 2^f_i, and 7 signed digits per weight
// of 64·w·2^-f_i by a shifter rint (exact for |v| < 2^51), ±128/±129 folded into the digit
// above; img[wave][digit][kstep][lane][16 B] as the i8 MFMA B operand. A NaN / ±inf weight
// makes the row's scale NaN (zero digits), as the fp64 stage would give NaN.
// dn2 (optional, [nc][7]): Σ_k w_a,ik² per row and digit level a (exact integers), for the
// line-search screen's statistical bound (DeviceCtx::screen_rank_bound).
void oz_split_rows(const double* w, size_t nc, size_t nf, uint8_t* img, double* sc, int ksw, double* dn2) {
  constexpr double SH = 0x1.8p52;
  constexpr int OZ_SLICES = 7;
  // rows are independent (each writes its own digit bytes and scale): split over the threads
#pragma omp parallel for schedule(static) if (nc * nf >= 4096)
  for (long ii = 0; ii < (long)nc; ++ii) {
    const size_t i = (size_t)ii;
    double mx = 0.0;
    bool bad = false;  // a NaN / ±inf weight: the row's scale becomes NaN (y = NaN, as in fp64)
    for (size_t k = 0; k < nf; ++k) {
      const double f = std::fabs(w[i * nf + k]);
      bad |= !std::isfinite(w[i * nf + k]);
      mx = f > mx ? f : mx;  // = fmax (NaN rows are flagged by bad), without a libm call
    }
    if (dn2)
      for (int a = 0; a < OZ_SLICES; ++a) dn2[i * OZ_SLICES + a] = 0.0;
    if (bad) {
      sc[i] = std::nan("");
      continue;  // zero digits
    }
    int e = 0;
    if (mx > 0.0) (void)std::frexp(mx, &e);
    sc[i] = std::ldexp(1.0, e - 12);
    const bool tiny = 6 - e > 1000;  // a row of subnormal size: 2^(6 − e) would overflow
    const double s6 = tiny ? 0.0 : std::ldexp(1.0, 6 - e);
    const size_t wave = i >> 4, n = i & 15;
    for (size_t k = 0; k < nf; ++k) {
      double v = tiny ? std::ldexp(w[i * nf + k], 6 - e) : w[i * nf + k] * s6;
      int dg[OZ_SLICES];
      for (int a = 0; a < OZ_SLICES; ++a) {
        const double r = (v + SH) - SH;
        dg[a] = (int)r;
        v = (v - r) * 256.0;
      }
      for (int a = OZ_SLICES - 1; a > 0; --a) {
        if (dg[a] > 127) { dg[a] -= 256; dg[a - 1] += 1; }
        else if (dg[a] < -128) { dg[a] += 256; dg[a - 1] -= 1; }
      }
      const size_t s = k >> 6, lane = n + 16 * ((k >> 4) & 3), j = k & 15;
      for (int a = 0; a < OZ_SLICES; ++a)
        img[(((wave * OZ_SLICES + a) * ksw + s) * 64 + lane) * 16 + j] = (uint8_t)(int8_t)dg[a];
      if (dn2)
        for (int a = 0; a < OZ_SLICES; ++a) dn2[i * OZ_SLICES + a] += (double)(dg[a] * dg[a]);
    }
  }
}

}  // namespace pcamd
