// Host Picard driver over an Evaluator. Statement order follows the
// reference so that the host-side N×N arithmetic is the reference's:
//   src/solver.rs:45-189 (fit_with_config), :218-249 (ica_par)
//   src/core.rs:39-96 (compute_loss), :99-150 (line_search), :162-401 (run)
//   src/lbfgs.rs:84-171, src/whitening.rs:48-107, src/jade.rs:22-197
// Every N×T quantity comes from the Evaluator (one fused device pass).
#include "host_solver.hpp"
#include "host_rng.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <omp.h>
#include <pthread.h>
#include <sched.h>
#include <sys/resource.h>
#include <thread>

namespace pcamd {

std::string rust_e4(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "inf" : "-inf";
  char buf[64];
  std::snprintf(buf, sizeof buf, "%.4e", v);
  std::string s(buf);
  size_t e = s.find('e');
  int ex = std::atoi(s.c_str() + e + 1);
  return s.substr(0, e) + "e" + std::to_string(ex);
}

// ---------------------------------------------------------------- lbfgs.rs
// Elementwise N×N updates of the host driver split over the team at N ≥ 256 (each element's
// arithmetic is unchanged, so any split gives the same bits); reductions stay serial.
constexpr size_t ELEMWISE_PAR = 65536;

Mat compute_direction(const Mat& g, const Mat& h, const std::vector<double>& h_off,
                      const LbfgsMemory& mem, bool ortho) {
  Mat q = g;
  const size_t k = mem.len();
  std::vector<double> alpha_list(k);
  const long ne = (long)q.a.size();
  for (size_t ii = k; ii-- > 0;) {  // .rev()
    const double alpha = mem.r_list[ii] * dot_sum(mem.s_list[ii], q);
    alpha_list[ii] = alpha;
    const Mat& y = mem.y_list[ii];
#pragma omp parallel for schedule(static) if (ne >= (long)ELEMWISE_PAR)
    for (long e = 0; e < ne; ++e) q.a[e] = q.a[e] - alpha * y.a[e];
  }
  Mat z;
  if (ortho) {
    Mat zq(q.rows, q.cols);
    for (size_t e = 0; e < q.a.size(); ++e) zq.a[e] = q.a[e] / h.a[e];
    z = Mat(q.rows, q.cols);
    for (size_t i = 0; i < q.rows; ++i)
      for (size_t j = 0; j < q.cols; ++j) z(i, j) = (zq(i, j) - zq(j, i)) / 2.0;
  } else {
    z = solve_hessian_system(h, h_off, q);
  }
  for (size_t ii = 0; ii < k; ++ii) {
    const double beta = mem.r_list[ii] * dot_sum(mem.y_list[ii], z);
    const Mat& s = mem.s_list[ii];
    const double f = alpha_list[ii] - beta;
#pragma omp parallel for schedule(static) if (ne >= (long)ELEMWISE_PAR)
    for (long e = 0; e < ne; ++e) z.a[e] = z.a[e] + f * s.a[e];
  }
  for (double& v : z.a) v = -v;
  return z;
}

Mat solve_hessian_system(const Mat& h, const std::vector<double>& h_off, const Mat& g) {
  const size_t n = h.rows;
  Mat r(n, n);
#pragma omp parallel for schedule(static) if (n * n >= ELEMWISE_PAR)
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) {
      const double det = h(i, j) * h(j, i) - h_off[i] * h_off[j];
      if (std::fabs(det) > 1e-15) r(i, j) = (h(j, i) * g(i, j) - h_off[i] * g(j, i)) / det;
    }
  return r;
}

void regularize_hessian(Mat& h, const std::vector<double>& h_off, double lambda_min) {
  const size_t n = h.rows;
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) {
      if (i == j) continue;
      const double diff = h(i, j) - h(j, i);
      const double discr = std::sqrt(diff * diff + 4.0 * h_off[i] * h_off[j]);
      const double eig = 0.5 * (h(i, j) + h(j, i) - discr);
      if (eig < lambda_min) h(i, j) += lambda_min - eig;
    }
}

// ------------------------------------------------------------- Solver
// Host team of the driving thread: the N×N work (Taylor series, log-determinants, L-BFGS, the
// digit split of W) gains nothing past a few threads at N ≤ 256, and a team as wide as the
// process's CPU share leaves no core for the line-search helper and the HIP runtime threads:
// on a 16-CPU box the one-rank-of-8 C3 shard measured host time per iteration mean 1.4-2.0 ms,
// p90 3-5 ms with 16 threads against 0.84-0.88 / 1.1-1.2 ms with 8 (profiles/r03_h). With 8
// ranks per node, 8 teams as wide as the node would oversubscribe it 8×. The team is
// min(the calling thread's OMP max threads at this call, cap), cap = 8 or PICARD_HOST_THREADS;
// only the cap is read once, so a caller's smaller setting for one fit does not shrink later
// fits.
static int host_team_cap() {
  static const int cap = [] {
    if (const char* e = std::getenv("PICARD_HOST_THREADS")) {
      const int c = std::atoi(e);
      if (c > 0) return c;
    }
    return 8;
  }();
  return cap;
}
static int host_team_threads() { return std::max(1, std::min(omp_get_max_threads(), host_team_cap())); }

// The calling thread's OpenMP team for the solver's host work, the caller's own setting
// restored on exit: the library leaves a caller's OpenMP state as it found it.
class TeamGuard {
 public:
  explicit TeamGuard(int n) : prev_(omp_get_max_threads()) { omp_set_num_threads(n); }
  ~TeamGuard() { omp_set_num_threads(prev_); }
  TeamGuard(const TeamGuard&) = delete;
  TeamGuard& operator=(const TeamGuard&) = delete;

 private:
  const int prev_;
};

Solver::Solver(Evaluator* ev, const pc_config& cfg) : ev_(ev), cfg_(cfg) {
  TeamGuard team(host_team_threads());
  // config.rs:104-142
  if (cfg.max_iter == 0) throw invalid_config("max_iter", "must be greater than 0");
  if (!(cfg.tol > 0.0)) throw invalid_config("tol", "must be positive");
  if (!(cfg.lambda_min > 0.0)) throw invalid_config("lambda_min", "must be positive");
  if (cfg.m == 0) throw invalid_config("m", "L-BFGS memory size must be at least 1");
  if (cfg.has_fastica_it && cfg.has_jade_it)
    throw invalid_config("jade_it", "cannot use both fastica_it and jade_it; choose one warm start method");
  if (cfg.density.kind < PC_DENSITY_TANH || cfg.density.kind > PC_DENSITY_CUBE)
    throw invalid_config("density", "unknown density kind");
  if (cfg.w_init) {
    w_init_user_.assign(cfg.w_init, cfg.w_init + cfg.w_init_rows * cfg.w_init_cols);
    cfg_.w_init = nullptr;
  }
  nf_ = ev->n_features();
  T_ = ev->n_samples();
  const uint64_t n = nf_, p = T_;
  if (n == 0 || p == 0) throw invalid_dimensions("Input matrix cannot be empty");  // solver.rs:50-54

  // solver.rs:56-60: StdRng::seed_from_u64(seed), or an unseeded (OS-entropy) stream
  RustStdRng rng{cfg.has_random_state ? cfg.random_state
                                      : (uint64_t)std::random_device{}() << 32 ^ std::random_device{}()};
  const uint64_t mn = n < p ? n : p;
  uint64_t ncomp = cfg.has_n_components ? cfg.n_components : mn;
  if (ncomp > mn) ncomp = mn;  // solver.rs:63
  extended_ = cfg.has_extended ? (cfg.extended != 0) : (cfg.ortho != 0);  // config.rs:99-101
  if (cfg.density.kind != PC_DENSITY_TANH && extended_ && !cfg.ortho)  // solver.rs:69-74
    std::fprintf(stderr,
                 "Warning: Using a density other than tanh with extended=true and ortho=false "
                 "may result in incorrect estimation or numerical overflow\n");
  const double pf = (double)p;
  // setup phases for PICARD_TRACE (ms since the constructor started)
  const auto ts0 = std::chrono::steady_clock::now();
  double tsm[5] = {0, 0, 0, 0, 0};  // rowsum, Gram, eigh, w_init + warm start, initial pass
  auto lap = [&](int i) { tsm[i] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts0).count(); };
  // center: whitening.rs:24-35 (μ folded into every pass; X is never copied)
  if (cfg.centering) {
    mu_.assign(n, 0.0);
    ev->rowsum(mu_.data());
    lap(0);
    for (double& v : mu_) v /= pf;
    has_mu_ = true;
  }
  const double* mu = has_mu_ ? mu_.data() : nullptr;
  // whiten: whitening.rs:48-116 via the Gram X·Xᵀ = U S² Uᵀ
  if (cfg.whiten) {
    if (ncomp > n) {
      throw invalid_dimensions("n_components (" + std::to_string(ncomp) +
                               ") cannot exceed n_features (" + std::to_string(n) + ")");
    }
    gram_ = Mat(n, n);
    ev->gram(mu, gram_.data());
    lap(1);
    has_gram_ = true;
    std::vector<double> lam;
    Mat u;
    eigh(gram_, &lam, &u);
    lap(2);
    // descending singular values s_i = sqrt(λ), columns of U in that order
    std::vector<double> s(n);
    Mat ud(n, n);
    for (size_t c = 0; c < n; ++c) {
      const size_t src = n - 1 - c;
      s[c] = std::sqrt(std::fmax(lam[src], 0.0));
      for (size_t r = 0; r < n; ++r) ud(r, c) = u(r, src);
    }
    double min_sv = std::numeric_limits<double>::infinity();
    for (size_t i = 0; i < ncomp; ++i) min_sv = std::fmin(min_sv, s[i]);
    if (min_sv < 1e-10) throw singular_matrix();  // whitening.rs:72-79
    gram_cond_ = (s[0] / min_sv) * (s[0] / min_sv);
    const double sc = std::sqrt(pf);
    K_ = Mat(ncomp, n);
    for (size_t i = 0; i < ncomp; ++i)
      for (size_t j = 0; j < n; ++j) K_(i, j) = ud(j, i) / s[i] * sc;
    for (size_t i = 0; i < ncomp; ++i) {  // whitening.rs:93-107 (max_by keeps the last max)
      size_t mi = 0;
      double best = -1.0;
      for (size_t j = 0; j < n; ++j)
        if (std::fabs(K_(i, j)) >= best) { best = std::fabs(K_(i, j)); mi = j; }
      if (K_(i, mi) < 0.0)
        for (size_t j = 0; j < n; ++j) K_(i, j) = -K_(i, j);
    }
    has_k_ = true;
  }
  nc_ = has_k_ ? ncomp : n;  // solver.rs:95
  // w_init: solver.rs:98-121
  if (cfg.w_init != nullptr) {
    if (cfg.w_init_rows != nc_ || cfg.w_init_cols != nc_)
      throw invalid_dimensions("w_init shape [" + std::to_string(cfg.w_init_rows) + ", " +
                               std::to_string(cfg.w_init_cols) + "] doesn't match expected (" +
                               std::to_string(nc_) + ", " + std::to_string(nc_) + ")");
    w_init_ = Mat(nc_, nc_);
    w_init_.a = w_init_user_;
  } else {
    Mat w(nc_, nc_);  // solver.rs:112-118: StandardNormal draws, row-major
    for (size_t i = 0; i < nc_ * nc_; ++i) w.a[i] = rng.standard_normal();
    if (!sym_decorrelation(w, &w_init_)) throw singular_matrix();
  }
  // warm starts: solver.rs:124-137
  if (cfg.has_jade_it) {
    if (cfg.verbose) std::printf("Running %llu iterations of JADE...\n", (unsigned long long)cfg.jade_it);
    w_init_ = jade(cfg.jade_it, 1e-6);
  } else if (cfg.has_fastica_it) {
    if (cfg.verbose) std::printf("Running %llu iterations of FastICA...\n", (unsigned long long)cfg.fastica_it);
    w_init_ = ica_par(w_init_);
  }
  lap(3);
  // x1 = w_init·x1 (solver.rs:140), kept as the composed map P
  P_ = has_k_ ? matmul(w_init_, K_) : w_init_;
  has_cov_ = extended_ && cfg.whiten;  // solver.rs:143-147
  if (cfg.verbose) {
    std::printf("Running Picard...\n");
    std::fflush(stdout);
  }
  trace_ = std::getenv("PICARD_TRACE") != nullptr;
  keep_y_ = std::getenv("PICARD_KEEP_Y") != nullptr;
  no_multi_ = std::getenv("PICARD_NO_MULTI") != nullptr;
  if (const char* e = std::getenv("PICARD_CVX")) cvx_on_ = std::atoi(e) != 0;
  if (const char* e = std::getenv("PICARD_MULTI_GROUP")) multi_group_ = (size_t)std::max(0, std::atoi(e));
  split_first_ = std::getenv("PICARD_SPLIT_FIRST") != nullptr;
  init_core();
  lap(4);
  for (int i = 0; i < 5; ++i) setup_ms_[i] = tsm[i];
  if (trace_)
    std::fprintf(stderr, "[picard-trace] setup ms (cumulative): rowsum %.3f gram %.3f eigh %.3f w_init %.3f initial pass %.3f\n",
                 tsm[0], tsm[1], tsm[2], tsm[3], tsm[4]);
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void Solver::evaluate(const Mat& w_core, EvalStats* out) {
  Mat wt = matmul(w_core, P_);
  // Σy² is read only by the extended non-orthogonal loss and Hessian (core.rs:79-81, :251)
  ev_->want_y2 = !cfg_.ortho && extended_;
  const double t0 = now_ms();
  ev_->eval(wt.data(), nc_, has_mu_ ? mu_.data() : nullptr, cfg_.density, !cfg_.ortho, out);
  eval_ms_ += now_ms() - t0;
  ++last_evals_;
  ++total_evals_;
  if (!cfg_.ortho) {  // the next non-ortho search starts from this W: keep W·P for it
    wp_cache_src_ = w_core;
    wp_cache_ = std::move(wt);
  }
}

bool Solver::evaluate_loss(const Mat& w_core, EvalStats* out) {
  Mat wt = matmul(w_core, P_);
  ev_->want_y2 = !cfg_.ortho && extended_;
  const double t0 = now_ms();
  const bool partial =
      ev_->eval_loss(wt.data(), nc_, has_mu_ ? mu_.data() : nullptr, cfg_.density, !cfg_.ortho, out, keep_y_);
  eval_ms_ += now_ms() - t0;
  ++last_evals_;
  ++total_evals_;
  return partial;
}

void Solver::complete(EvalStats* out) {
  const double t0 = now_ms();
  ev_->eval_complete(cfg_.density, !cfg_.ortho, out);
  eval_ms_ += now_ms() - t0;
  ++total_completions_;
}

// core.rs:39-85 + loss_to_f64 core.rs:90-96, from the pass's per-row sums
double Solver::loss_of(const EvalStats& s, const Mat& w, const std::vector<double>& signs, bool* singular,
                       double sg, double la) {
  const double t = (double)T_;
  const bool ortho = cfg_.ortho != 0;
  double loss = 0.0;
  *singular = false;
  if (!ortho) {
    if (std::isnan(sg)) sln_det(w, &sg, &la);  // not given by the caller
    if (sg == 0.0) { *singular = true; return 1e15; }
    loss = -la;
  }
  const double* ll = s.ll();
  const double* y2 = s.y2();
  for (size_t i = 0; i < nc_; ++i) {
    loss += signs[i] * ll[i] / t;
    if (extended_ && !ortho) loss += 0.5 * y2[i] / t;
  }
  return loss;
}

void Solver::init_core() {  // core.rs:175-209
  const size_t n = nc_;
  W_ = Mat::eye(n);
  signs_.assign(n, 1.0);
  old_signs_ = signs_;
  last_evals_ = 0;
  evaluate(W_, &S_);
  bool singular;
  current_loss_ = loss_of(S_, W_, signs_, &singular);
  if (singular) throw singular_matrix();
  gradient_norm_ = 1.0;
  converged_ = false;
  if (extended_) {
    if (has_cov_) {
      C_ = Mat::eye(n);
    } else {  // Y·Yᵀ/T of x1 = P·(X−μ): P·Gram·Pᵀ/T (core.rs:202)
      if (!has_gram_) {
        gram_ = Mat(nf_, nf_);
        ev_->gram(has_mu_ ? mu_.data() : nullptr, gram_.data());
        has_gram_ = true;
      }
      C_ = matmul_nt(matmul(P_, gram_), P_);
      for (double& v : C_.a) v /= (double)T_;
    }
  } else {
    C_ = Mat::eye(n);
  }
  // whitened covariance for the curvature rejection (orthogonal tanh searches only): used
  // only when it computes to I within 1e-3 and the kept part of the Gram has condition number
  // below 1e10 (C1's rounding, ≈ 1e-13·cond relative, then stays far inside Cy's 1 % margin)
  if (cfg_.ortho && has_k_ && has_gram_ && cfg_.density.kind == PC_DENSITY_TANH && cfg_.density.alpha > 0.0) {
    C1_ = matmul_nt(matmul(P_, gram_), P_);
    for (double& v : C1_.a) v /= (double)T_;
    double dev = 0.0;
    for (size_t i = 0; i < n; ++i)
      for (size_t j = 0; j < n; ++j) dev = std::fmax(dev, std::fabs(C1_(i, j) - (i == j ? 1.0 : 0.0)));
    curv_ok_ = dev < 1e-3 && gram_cond_ < 1e10;
  }
}

// Curvature rejection (schedule only, no decision changes). Along the try path
// W(α) = expm(αD)·W, y_t(α) = E·y_t with E = expm(αD) orthogonal and commuting with D (D
// skew-symmetric), so with Cy = Σ_t y_t y_tᵀ/T = W·C1·Wᵀ the sums A_k = Σ_t‖D^k y_t‖²/T =
// tr(D^k·Cy·D^kᵀ) (A_0 = N_eff) do not depend on α. For the tanh density ℓ′ = tanh(a·y)
// (|ℓ′| ≤ a|y|) and 0 ≤ ℓ″ ≤ a. The orthogonal loss L(α) = Σ_i s_i Σ_t ℓ(y_it)/T has
// L′(0) = ⟨g, D⟩ = slope and L″ = u + v with
//   u(α) = Σ_t Σ_i s_i ℓ″(y_it)(D y_t)_i² / T   ≥ −a·A_1⁻, A_1⁻ = min(A_1, λmax(Cy)·Σ_{i: s_i < 0} (D·Dᵀ)_ii)
//          (0 when every s_i = +1; both terms bound the negative rows at every α, below);
//   v(α) = Σ_t Σ_i s_i ℓ′(y_it)(D² y_t)_i / T,  v(0) = ⟨g_s, D²⟩ (g_s = s_i·G_ij/T, the
//          signed gradient before the skew part), |v′| ≤ a·√(A_1·A_2) + a·√(A_0·A_3) = K_3,
//          |v| ≤ a·√(A_0·A_2)   (Cauchy–Schwarz over t).
// So L″(β) ≥ m(β) = max(q − β·K_3, −M) with q = v(0) − a·A_1⁻, M = a·A_1⁻ + a·√(A_0·A_2), and
//   L(α) − L(0) ≥ α·slope + ∫_0^α (α − β)·m(β) dβ,
// integrated in closed form on the two pieces of m (the line q − β·K_3 down to β* = (q + M)/K_3,
// the floor −M after it). Its two extremes are the earlier bounds α·slope − α²·M/2 and
// α·slope + α²·q/2 − α³·K_3/6, and it is at least the larger of them.
// When it exceeds the rounding of both exact losses (passes and W(α); far above the kernels'
// 1e-10 relative sum error), the exact pass at α would reject the try (core.rs:127-140), so it
// need not run. Cy carries a 1 % margin (C1's rounding is ≈ 1e-13·cond(Gram) relative, and the
// rejection is off above cond 1e10); slope and v(0) are lowered by their rounding bounds.
void Solver::set_curvature(const Mat& g, const Mat& gs, const Mat& d, double slope) {
  ls_curv_ = 0.0;
  if (!curv_ok_ || !(slope > 0.0)) return;
  const size_t n = nc_;
  for (size_t i = 0; i < n; ++i)
    if (!(signs_[i] == 1.0 || signs_[i] == -1.0)) return;
  Mat cy = matmul_nt(matmul(W_, C1_), W_);
  for (double& v : cy.a) v *= 1.01;
  double a0 = 0.0;
  for (size_t i = 0; i < n; ++i) a0 += cy(i, i);
  const Mat d2 = matmul(d, d), d3 = matmul(d2, d);
  const Mat dcy = matmul(d, cy);
  const double a1 = std::fabs(dot_sum(dcy, d));              // tr(D·Cy·Dᵀ) = Σ (D·Cy)∘D
  // A1⁻ bounds Σ_{s_i<0} (E·D·Cy·Dᵀ·Eᵀ)_ii at EVERY α (E = expm(αD)): a partial diagonal sum
  // is not rotation-invariant, but D·Cy·Dᵀ ≤ λmax(Cy)·D·Dᵀ and E·D·Dᵀ·Eᵀ = D·Dᵀ (E commutes
  // with D and is orthogonal), so A1⁻ = λ·Σ_{s_i<0} (D·Dᵀ)_ii with λ ≥ λmax(Cy) from
  // Gershgorin, capped by the invariant full trace A1 (exact for any Cy, not only
  // an isotropic one)
  double lam = 0.0;
  for (size_t i = 0; i < n; ++i) {
    double r = 0.0;
    for (size_t j = 0; j < n; ++j) r += std::fabs(cy(i, j));
    lam = std::fmax(lam, r);
  }
  double ddn = 0.0;
  for (size_t i = 0; i < n; ++i)
    if (signs_[i] < 0.0)
      for (size_t j = 0; j < n; ++j) ddn += d(i, j) * d(i, j);
  const double a1n = std::fmin(a1, lam * ddn);
  const double a2 = std::fabs(dot_sum(matmul(d2, cy), d2));  // tr(D²·Cy·D²ᵀ)
  const double a3 = std::fabs(dot_sum(matmul(d3, cy), d3));  // tr(D³·Cy·D³ᵀ)
  double gd = 0.0, gd2 = 0.0, v0 = 0.0;
  for (size_t e = 0; e < g.a.size(); ++e) gd += std::fabs(g.a[e] * d.a[e]);
  for (size_t e = 0; e < gs.a.size(); ++e) {
    v0 += gs.a[e] * d2.a[e];
    gd2 += std::fabs(gs.a[e] * d2.a[e]);
  }
  const double a = cfg_.density.alpha;
  ls_slope_ = slope - 1e-10 * gd;
  ls_curv_ = a * (a1n + std::sqrt(a0 * a2));
  ls_q_ = v0 - 1e-10 * gd2 - a * a1n;
  ls_k3_ = a * (std::sqrt(a1 * a2) + std::sqrt(a0 * a3));
  // |Σ_i ℓ_i| ≤ Σ|y_i| + N·ln2/a ≤ √(N·N_eff) + N·ln2/a per sample
  ls_slack_ = 2.0 * (3e-10 * (std::sqrt((double)n * a0) + (double)n * 0.6931471805599453 / a) + 1e-9);
  if (!std::isfinite(ls_curv_) || !std::isfinite(ls_slope_) || !std::isfinite(ls_q_) || !std::isfinite(ls_k3_) ||
      !(ls_slope_ > 0.0))
    ls_curv_ = 0.0;
}

double Solver::curvature_lower_bound(double alpha) const {
  // b: where m(β) meets its floor, within [0, α]
  double b = ls_k3_ > 0.0 ? (ls_q_ + ls_curv_) / ls_k3_ : (ls_q_ + ls_curv_ >= 0.0 ? alpha : 0.0);
  b = std::fmin(std::fmax(b, 0.0), alpha);
  const double r = alpha - b;
  return alpha * ls_slope_ + ls_q_ * b * (alpha - 0.5 * b) - ls_k3_ * b * b * (0.5 * alpha - b / 3.0) -
         0.5 * ls_curv_ * r * r;
}

// Convexity rejection (schedule only, no decision changes), non-orthogonal searches with the
// tanh density and every s_i = +1 (not extended). Along the try path W(α) = (I + αD)·W
// (core.rs:121) the sources y_t(α) = y_t + α·D·y_t are affine in α, so the density part of the
// loss (core.rs:39-85), f(α) = Σ_i Σ_t ℓ(y_it(α))/T with ℓ″ = a·(1 − tanh²(a·y)) ≥ 0, is convex:
//   f(α) ≥ f(0) + α·f′(0),  f′(0) = Σ_ij D_ij·G_ij/T  (G = ψ·Yᵀ of the current W's pass).
// The log-determinant part is −log|det W| − log|det(I + αD)|, and Hadamard's inequality gives
// log|det(I + αD)| ≤ Σ_k ½·log‖e_k + α·D_k‖² (D_k: row k). So
//   L(α) − L(0) ≥ B(α) = α·f′(0) − Σ_k ½·log((1 + α·D_kk)² + α²·Σ_{j≠k} D_kj²),
// which is α·⟨g, D⟩ − O(α²) with ⟨g, D⟩ = f′(0) − tr D the search's slope: positive at small α
// along a non-descent direction (a third of C4's failed searches). Where B(α) exceeds the
// rounding of both computed losses (the pass's G entries to 1e-10 of Σ_t|ψ_i·y_j| ≤ T·√(Σy_j²/T)
// as |ψ| ≤ 1; the density sums to 1e-9 of Σ|ℓ| with |ℓ(y)| ≤ |y| + ln2/a; each log|det| to 1e-9
// per row — all far above the kernels' and the LU's actual rounding), the exact pass at α would
// reject the try (core.rs:127-140). Returns how many leading tries (α = 1, ½, …) remain once the
// trailing tries that the bound rejects are dropped; tries between the first and the last
// rejection still run. When none remains, the search fails without a pass, as it would with
// every pass run (its result is then discarded for the gradient fallback, core.rs:349-364).
size_t Solver::convexity_trim(const Mat& d, size_t tries, double* b_first) const {
  const size_t n = nc_;
  *b_first = 0.0;
  if (!cvx_on_ || cfg_.ortho || extended_ || cfg_.density.kind != PC_DENSITY_TANH || !(cfg_.density.alpha > 0.0) ||
      tries == 0)
    return tries;
  for (size_t i = 0; i < n; ++i)
    if (signs_[i] != 1.0) return tries;
  const double t = (double)T_, a = cfg_.density.alpha;
  const double* g = S_.G();
  const double* y2 = S_.y2();
  std::vector<double> ry(n), dkk(n), off(n);
  double sry = 0.0;
  for (size_t j = 0; j < n; ++j) {
    const double q = y2[j] / t;
    if (!(q > 0.0) || !std::isfinite(q)) return tries;  // Σy² not computed by this pass
    ry[j] = std::sqrt(q);
    sry += ry[j];
  }
  double fp = 0.0, dabs = 0.0;  // f′(0); Σ_ij |D_ij|·√(Σy_j²/T) ≥ Σ_i E|(D·y)_i|
  for (size_t i = 0; i < n; ++i) {
    double o = 0.0;
    for (size_t j = 0; j < n; ++j) {
      const double v = d(i, j);
      fp += v * (g[i * n + j] / t);
      dabs += std::fabs(v) * ry[j];
      if (j != i) o += v * v;
    }
    dkk[i] = d(i, i);
    off[i] = o;
  }
  if (!std::isfinite(fp) || !std::isfinite(dabs)) return tries;
  auto bound = [&](double al) {
    double h = 0.0;  // Σ_k ½·log‖e_k + α·D_k‖², each row's square sum a sum of non-negative terms
    for (size_t k = 0; k < n; ++k) {
      const double u = 1.0 + al * dkk[k];
      h += 0.5 * std::log((u * u + al * al * off[k]) * (1.0 + 1e-12));
    }
    const double slack = al * 1e-10 * dabs + 2e-9 * (sry + al * dabs + (double)n * 0.6931471805599453 / a) +
                         2e-9 * (double)n + 1e-12;
    return al * fp - h - slack;  // −inf row terms (a zero row of I + αD: W(α) singular) reject
  };
  size_t keep = tries;
  double al = std::ldexp(1.0, -(int)(tries - 1));
  double b = 0.0;
  while (keep > 0 && (b = bound(al)) > 0.0) {
    *b_first = b;
    --keep;
    al *= 2.0;
  }
  return keep;
}

// Orthogonal line search, host side: W_k = expm(α_k·D)·W (core.rs:118-125) for
// α_k = 2^-k. Try 0's map is on the critical path; a helper thread forms the
// maps of tries 1, 2, … while the device evaluates the earlier tries, so the
// N³ Taylor series (math.rs:38-74) is hidden behind the passes. Same operations
// in the same order as the serial loop: identical bits.
// One persistent helper per solver. A search submits (D, W, tries) under a new
// generation number; the helper forms its maps in order and drops a job as soon
// as a newer one arrives. A finished search never waits for it (a stale
// matrix_exp just completes in the background), which a per-search thread that
// is joined at the end would do: up to one N³ series per iteration.
// The helper runs single-threaded: a second OpenMP team beside the driving thread's
// oversubscribes the host's cores (measured: try 1's map 3.6x slower with half the threads
// here), and its maps were never waited for (PICARD_TRACE map_wait_ms = 0 at C3 / 8).
class TransformWorker {
 public:
  TransformWorker() : nthreads_(1) {
    th_ = std::thread([this] { run(); });
  }
  ~TransformWorker() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void submit(const Mat& d, const Mat& w, size_t tries) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      ++gen_;
      d_ = d;
      w_ = w;
      tries_ = tries;
      out_.assign(tries, Mat());
      ready_.assign(tries, 0);
    }
    cv_.notify_all();
  }
  Mat get(size_t k, double* wait_ms) {
    const double t0 = now_ms();
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return ready_[k] != 0; });
    *wait_ms += now_ms() - t0;
    return out_[k];
  }

 private:
  const int nthreads_;
  void run() {
    // below the driving thread's priority: woken by submit() right after try 1's map, a helper of
    // equal weight was often placed on the driving thread's core and ran its whole job (all the
    // later tries' maps) before the driver could launch try 1's pass — 0.8–1.2 ms of host time in
    // about half the iterations of a traced N = 64 fit on the 8-core container; at nice +10 the
    // driver keeps its core (Linux: setpriority on PRIO_PROCESS 0 applies to the calling thread)
    setpriority(PRIO_PROCESS, 0, 10);
    omp_set_num_threads(nthreads_);
    uint64_t done_gen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || gen_ != done_gen; });
      if (stop_) return;
      const uint64_t g = gen_;
      const Mat d = d_, w = w_;
      const size_t tries = tries_;
      double alpha = 1.0;
      for (size_t k = 1; k < tries; ++k) {
        alpha /= 2.0;
        lk.unlock();
        Mat wk = matmul(matrix_exp(scale(d, alpha)), w);
        lk.lock();
        if (stop_ || gen_ != g) break;  // superseded: drop the rest of this job
        out_[k] = std::move(wk);
        ready_[k] = 1;
        cv_.notify_all();
      }
      done_gen = g;
    }
  }
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  uint64_t gen_ = 0;
  Mat d_, w_;
  size_t tries_ = 0;
  std::vector<Mat> out_;
  std::vector<char> ready_;
};

Solver::~Solver() = default;

// screen / full-pass time ratio of the first-try policy, from the pass shape alone (every rank
// computes the same value): kernel time ∝ nc²·T (MI355X, C3 = 128² × 1e8: screen 18.6 ms, fused
// pass 84 ms) plus a fixed cost per call (≈ 0.08 / 0.10 ms: launches, copies, synchronisation).
// C3: 0.22; C2 (64² × 1e6): 0.41.
static double screen_cost_ratio(size_t nc, uint64_t t) {
  const double w = (double)nc * (double)nc * (double)t / (128.0 * 128.0 * 1e8);
  return (18.6 * w + 0.08) / (84.0 * w + 0.10);
}

// The device share of an evaluator call that ran `hook_ms` of the caller's host work while its
// pass was in flight (Evaluator::overlap_): the whole call while the hook hid behind the pass;
// once the hook outlasts the pass's kernel time, the excess is host time. Without a
// kernel time the call counts as device time.
double Solver::device_share(double call_ms, double hook_ms) const {
  const double k = ev_->last_pass_kernel_ms();
  if (!(hook_ms > 0.0) || !(k >= 0.0)) return call_ms;
  return std::fmin(call_ms, std::fmax(call_ms - hook_ms, k));
}

Solver::LsResult Solver::line_search(const Mat& direction, size_t tries, bool multi_first,
                                     bool first_loss_only, bool full_first) {  // core.rs:99-150
  // Evaluation schedule: a try is a full fused pass, or a loss-only pass
  // completed (G, H, Σψ′) only if that try becomes the new iterate (both
  // bit-identical). Non-ortho searches evaluate their tries in one multi-α pass
  // (from try 1 when `multi_first`, else from try 2), which forms Y_α as Y + αZ
  // and so agrees with per-try passes to rounding.
  const size_t n = nc_;
  const bool ortho = cfg_.ortho != 0;
  double alpha = 1.0;
  LsResult r{false, W_, S_, current_loss_, Mat(), false, 0, false, false};
  if (!ortho && !full_first) {  // the trailing tries the convexity bound rejects run no pass
    double b = 0.0;
    const size_t keep = convexity_trim(direction, tries, &b);
    if (keep < tries) {
      cvx_skips_ += tries - keep;
      if (trace_)
        std::fprintf(stderr, "[picard-cvx] tries %zu-%zu rejected by the convexity bound (at alpha %.3e: %.3e)\n",
                     keep + 1, tries, std::ldexp(1.0, -(int)keep), b);
      tries = keep;
    }
  }
  // a paired screen's second try (Evaluator::eval_loss_screen2): its rows, for try pair_k
  std::vector<double> pair_ll, pair_bnd;
  size_t pair_k = tries;
  // the previous screened try of this search: its margin (estimate − current loss) and the
  // bound of its first-level screen (schedule only, below)
  double prev_margin = -1.0, prev_eb0 = 0.0;
  for (size_t k = 0; k < tries; ++k) {
    Mat transform;
    if (ortho) {
      if (k == 0) {
        // the helper starts on try 2's map while this thread forms try 1's: a paired screen
        // needs both at once (it waited 0.33–0.41 ms for try 2's map when submitted after)
        if (tries > 1) {
          if (!ahead_) {
            ahead_.reset(new TransformWorker());
            // the helper keeps a core of its own: this thread's OpenMP team gives one up. A
            // stale helper map (a search that ended early) otherwise shares a core with a team
            // thread, and every barrier of the team's N³ products waits for that thread (one
            // rank of C3/8: a fallback's try-1 Taylor series took 9.4 ms instead of 0.2)
            omp_set_num_threads(std::max(1, host_team_threads() - 1));
          }
          ahead_->submit(direction, W_, tries);
        }
        // try 1's map is on the critical path: expm(α·D) where the passes run when the evaluator
        // can (DeviceCtx: k_expm_ps, the host's bits), else on the host
        const double tm = now_ms();
        const Mat da = scale(direction, alpha);
        Mat e(n, n);
        if (!ev_->device_matrix_exp(da.data(), n, e.data())) e = matrix_exp(da);
        r.w = matmul(e, W_);
        map1_ms_ = now_ms() - tm;
      } else {
        r.w = ahead_->get(k, &ahead_wait_ms_);
      }
    } else if (no_multi_ || !(k == 1 || (k == 0 && multi_first))) {  // (a multi-try pass forms it below)
      transform = Mat::eye(n);
      for (size_t e = 0; e < transform.a.size(); ++e) transform.a[e] += alpha * direction.a[e];
      r.w = matmul(transform, W_);
    }
    if (!ortho && !no_multi_ && (k == 1 || (k == 0 && multi_first))) {
      // Non-ortho: Y_α = Y + α·Z is linear in α, so the remaining tries share
      // one pass (see eval_loss_multi); only the accepted try is evaluated in full.
      const size_t na = tries - k;
      std::vector<double> alphas(na), ll(na * n), y2(na * n), bnd;
      for (size_t j = 0; j < na; ++j) alphas[j] = j == 0 ? alpha : alphas[j - 1] / 2.0;
      const bool cached = wp_cache_src_.a.size() == W_.a.size() &&
                          std::memcmp(wp_cache_src_.a.data(), W_.a.data(), W_.a.size() * sizeof(double)) == 0;
      const Mat wt = cached ? wp_cache_ : matmul(W_, P_);  // (the same product, evaluate())
      Mat zt = matmul(matmul(direction, W_), P_);
      // without Σy² in the loss (not extended), the tries may come with a bound instead of
      // exact sums (fp32 row terms); every decision is then taken on exact values (below)
      bool bounded = false;
      const double tmp0 = now_ms();
      if (!extended_ && multi_bound_on_) {
        bnd.assign(na * n, 0.0);
        bounded = ev_->eval_loss_multi_bound(wt.data(), zt.data(), n, has_mu_ ? mu_.data() : nullptr, cfg_.density,
                                             alphas.data(), (int)na, ll.data(), bnd.data());
      }
      // Staged tries (exact path; schedule only): the pass's cost grows with its tries (each is
      // a density evaluation per element), and a search is usually decided by an early try, so
      // the first pass covers the first multi_group_ tries and a second pass the rest only if
      // none of them is accepted. Each try's sums do not depend on which others share its pass
      // (k_multi_loss2*: per-try accumulators, the same arithmetic per try), so every decision
      // is the one-pass schedule's.
      const size_t g1 = bounded || multi_group_ == 0 ? na : std::min(na, multi_group_);
      size_t j0 = 0, nj = g1;
      // every try's W_j = (I + α_j D)·W and log|det W_j| (core.rs:121-125, :43-47), formed for a
      // pass's tries at once on the host threads — while the device runs that pass (the
      // evaluator's overlap hook), else right after it; each is the same serial arithmetic as
      // the per-try path, and the walk below accepts in the reference order
      std::vector<Mat> wj(na);
      std::vector<double> dsg(na), dla(na);
      auto form_tries = [&](size_t a0, size_t cnt) {
#pragma omp parallel for schedule(dynamic, 1) if (cnt > 1)
        for (size_t j = a0; j < a0 + cnt; ++j) {
          Mat tj = Mat::eye(n);
          for (size_t e = 0; e < tj.a.size(); ++e) tj.a[e] += alphas[j] * direction.a[e];
          wj[j] = matmul(tj, W_);
          sln_det(wj[j], &dsg[j], &dla[j]);
        }
      };
      struct HookGuard {  // never leave a hook on the evaluator that refers to this frame
        Evaluator* ev;
        ~HookGuard() { ev->overlap_ = nullptr; }
      } hook_guard{ev_};
      double hook_ms = 0.0;  // the overlapped host work: booked as host time where it outlasts the pass
      if (bounded) form_tries(0, nj);
      else ev_->overlap_ = [&, nj] {
        const double th = now_ms();
        form_tries(0, nj);
        hook_ms = now_ms() - th;
      };
      const bool multi_ran = bounded || ev_->eval_loss_multi(wt.data(), zt.data(), n, has_mu_ ? mu_.data() : nullptr,
                                                             cfg_.density, alphas.data(), (int)nj, ll.data(), y2.data());
      eval_ms_ += device_share(now_ms() - tmp0, hook_ms);  // the multi-try pass is device time
      ev_->run_overlap();  // (not run by the evaluator)
      if (!multi_ran) r.w = wj[0];  // try k on its own pass (below)
      if (multi_ran) {
        EvalStats ls;
        ls.nc = n;
        ls.has_h = false;
        ls.buf.assign(EvalStats::size(n, false), 0.0);
        EvalStats last_full;  // bounded: the exact pass of the LAST try, if one ran and rejected it
        bool have_last_full = false;
        for (;;) {  // one pass over tries j0 … j0 + nj − 1
          ++last_evals_;
          ++total_evals_;
          for (size_t j = j0; j < j0 + nj; ++j) {
            const double a = alphas[j];
            r.w = std::move(wj[j]);
            std::memcpy(const_cast<double*>(ls.ll()), ll.data() + j * n, n * sizeof(double));
            std::memcpy(const_cast<double*>(ls.y2()), y2.data() + j * n, n * sizeof(double));
            r.tries = k + j + 1;
            bool singular;
            const double loss = loss_of(ls, r.w, signs_, &singular, dsg[j], dla[j]);
            if (bounded) {
              // core.rs:127-140 on the exact loss: a try whose lower bound cannot beat the
              // current loss fails; the first one that might is evaluated in full (that pass is
              // the new iterate if it is accepted) and decided on its exact loss
              double eb = 0.0;
              for (size_t i = 0; i < n; ++i) eb += std::fabs(signs_[i]) * bnd[j * n + i] / (double)T_;
              if (!singular && loss - eb < current_loss_) {
                EvalStats full;
                evaluate(r.w, &full);
                const double exact = loss_of(full, r.w, signs_, &singular, dsg[j], dla[j]);
                if (exact < current_loss_) {
                  r.stats = std::move(full);
                  r.partial = false;
                  r.loss = exact;
                  r.success = true;
                  r.step = scale(direction, a);
                  return r;
                }
                multi_bound_on_ = false;  // a full pass spent on a rejected try: exact tries from now on
                if (j + 1 == na) {  // kept below: step() needs no second pass at the same W
                  last_full = std::move(full);
                  have_last_full = true;
                }
              }
            } else if (loss < current_loss_) {
              evaluate(r.w, &r.stats);  // the new iterate: full pass at W_k
              r.partial = false;
              r.loss = loss_of(r.stats, r.w, signs_, &singular, dsg[j], dla[j]);  // (its log|det| is formed)
              r.success = true;
              r.step = scale(direction, a);
              return r;
            }
            alpha = a / 2.0;
          }
          j0 += nj;
          if (j0 >= na) break;
          nj = na - j0;  // the remaining tries in one more pass
          ++multi_second_passes_;
          const double tmp1 = now_ms();
          hook_ms = 0.0;
          ev_->overlap_ = [&, j0, nj] {
            const double th = now_ms();
            form_tries(j0, nj);
            hook_ms = now_ms() - th;
          };
          if (!ev_->eval_loss_multi(wt.data(), zt.data(), n, has_mu_ ? mu_.data() : nullptr, cfg_.density,
                                    alphas.data() + j0, (int)nj, ll.data() + j0 * n, y2.data() + j0 * n))
            throw computation_error("multi-try pass refused after an earlier one ran");
          eval_ms_ += device_share(now_ms() - tmp1, hook_ms);
          ev_->run_overlap();
        }
        // no try accepted: the caller evaluates the last try in full if it keeps it — unless
        // the bounded path already ran that pass (its exact statistics and loss are kept)
        bool singular;
        if (have_last_full) {
          r.stats = std::move(last_full);
          r.needs_full = false;
          r.loss = loss_of(r.stats, r.w, signs_, &singular, dsg[na - 1], dla[na - 1]);
        } else {
          r.stats = ls;
          r.needs_full = true;
          r.loss = loss_of(ls, r.w, signs_, &singular, dsg[na - 1], dla[na - 1]);
          r.det_sg = dsg[na - 1];  // step() evaluates this W in full and takes its loss again
          r.det_la = dla[na - 1];
        }
        r.partial = false;
        r.step = scale(direction, alpha);
        return r;
      }
      no_multi_ = true;  // evaluator cannot: per-try passes from now on
    }
    r.tries = k + 1;
    // Curvature rejection (set_curvature): once the evaluator has shown that it screens (so
    // the exact-every-try modes keep every pass), a try the bound already rejects needs no pass
    if (ortho && ls_curv_ > 0.0 && screen_seen_ && curvature_lower_bound(alpha) > ls_slack_) {
      if (k == 0 && !first_loss_only && !full_first) first_n_[first_cell_] += 1.0;
      ++curv_skips_;
      r.screened_out = true;  // no exact statistics for this W
      if (trace_)
        std::fprintf(stderr, "[picard-curv] try %zu alpha %.3e lower bound %.3e reject\n", k + 1, alpha,
                     curvature_lower_bound(alpha));
      alpha /= 2.0;
      continue;
    }
    // Orthogonal searches screen their tries when the evaluator has a screen. Try 1 of a
    // descent direction (⟨g, D⟩ < 0) is accepted with some probability p: screening it
    // costs t_s + p·t_f against t_f for a full pass, so it is screened only while the
    // running estimate of p is below 1 − t_s/t_f. p is estimated per cell (step(): whether
    // Picard's quadratic model along D predicts a decrease at α = 1, and whether the previous
    // search was accepted at try 1) over this fit's first tries.
    // t_s/t_f: screen_cost_ratio (rank-independent; see below).
    // The gradient fallback (full_first) is accepted at try 1 almost always: full pass.
    // Schedule only: no decision changes.
    bool screen = ortho && !keep_y_ && screen_ok_;
    const bool first_policy = k == 0 && !first_loss_only && !full_first;
    // A later try of a descent search (its first try failed) where Picard's quadratic model
    // still predicts a decrease, α·slope + α²·qh/2 < 0: the same estimate as try 1's cells
    // (Beta(9, 1) prior, own counts). On the traced proxy fit it named the accepted try of
    // every such search it reached (profiles/r04_k). Schedule only.
    const bool later_policy = k > 0 && !first_loss_only && !full_first && pred_slope_ < 0.0 && pred_qh_ > 0.0 &&
                              pred_slope_ + 0.5 * alpha * pred_qh_ < 0.0;
    bool later_full = false;
    if (screen && later_policy && (later_acc_ + 9.0) / (later_n_ + 10.0) >= 1.0 - screen_cost_ratio(n, T_)) {
      screen = false;
      later_full = true;
    }
    if (screen && k == 0) {
      if (full_first) {
        screen = false;
      } else if (first_policy) {
        // t_s/t_f is a model of the shape, not the measured means: with one RCCL
        // communicator every rank must take the same branch (the screen and the full
        // pass issue different all-reduces), and p_acc is built from decisions alone.
        // p per policy cell, Beta-prior mean: Beta(9, 1) where the model predicts a decrease
        // (a full pass from the start; two early failures bring screening back), else Beta(1, 1)
        const int c = first_cell_;
        const double p_acc = c >= 2 ? (first_acc_[c] + 9.0) / (first_n_[c] + 10.0) : (first_acc_[c] + 1.0) / (first_n_[c] + 2.0);
        screen = p_acc < 1.0 - screen_cost_ratio(n, T_);
      }
    }
    if (later_full || (!screen && k == 0 && !first_loss_only && (first_full_ || !split_first_))) {
      if (later_full && trace_) std::fprintf(stderr, "[picard-model] try %zu alpha %.3e full pass\n", k + 1, alpha);
      evaluate(r.w, &r.stats);
      r.partial = false;
    } else if (screen) {
      // Screen (Evaluator::eval_loss_screen): a cheaper pass plus a rigorous bound on
      // the exact Σℓ. If even the most favourable exact loss cannot beat the current
      // one, the try fails exactly as core.rs:127-140 would decide; otherwise the exact
      // evaluation runs as a full pass (it also yields G if the try is accepted).
      bool rejected = false, screened = false;
      std::vector<double> ll(n), bnd(n);
      const Mat wt = matmul(r.w, P_);
      ev_->want_y2 = false;
      const double t0 = now_ms();
      const double* mu = has_mu_ ? mu_.data() : nullptr;
      bool got = false;
      const char* via = "";
      // Schedule only: the previous try of this search was screened with a margin m, and
      // halving α roughly halves it; when m/2 falls below 1.25× the first-level bound that try
      // had, the first level would almost surely leave this try undecided, so the screen starts
      // one level finer (it issues the same collectives on every rank: margins and bounds are
      // reduced statistics). The decision itself is unchanged: every level is rigorous.
      int level0 = 0;
      if (pair_k != k && k > 0 && prev_margin > 0.0 && 0.5 * prev_margin < 1.25 * prev_eb0) level0 = 1;
      if (level0 == 1 && ev_->eval_loss_screen_fine(1, wt.data(), n, mu, cfg_.density, ll.data(), bnd.data())) {
        got = true;
        via = " (finer first)";
        eval_ms_ += now_ms() - t0;
        ++screen_passes_;
      } else {
        level0 = 0;
      }
      if (got) {
      } else if (pair_k == k) {  // screened with the previous try's pass
        via = " (paired)";
        ll = pair_ll;
        bnd = pair_bnd;
        pair_k = tries;
        got = true;
      } else if (pairs_ok_ && k + 1 < tries && ahead_ &&
                 (first_loss_only ? !(ls_curv_ > 0.0 && curvature_lower_bound(alpha / 2.0) > ls_slack_)
                                  : descent_pair_ && !full_first && pred_slope_ < 0.0 && pred_qh_ > 0.0 &&
                                        0.5 * alpha >= descent_pair_factor_ * -pred_slope_ / pred_qh_ &&
                                        (k == 0 || (prev_margin > 0.0 && 0.25 * prev_margin > 2.5 * prev_eb0)))) {
        // Schedule only: a non-descent direction (⟨g, D⟩ ≥ 0) almost surely fails every try,
        // and its next try will be screened too (not rejected by curvature), so both tries go
        // in one pass — half the bytes per try for a screen whose clock the memory side's power
        // holds down. Each try's rows are those of its own screen (the same
        // arithmetic per W), so every decision is unchanged.
        // An overshooting descent search pairs its tries the same way while Picard's quadratic
        // model puts the loss's zero crossing α₀ = 2|slope|/qh at most half the next try's α (so
        // neither try is predicted to descend, and the next try takes no model full pass; on C3 the
        // accepted try of a descent search lay within 2.5·α₀, the pair's first try is ≥ 4·α₀)
        // and the previous try's margin, at least halving per try, leaves the next one decided
        // at the first level with room (m/4 > 2.5× its bound). C3's two overshooting searches
        // (7 rejected tries each) ran 7 single screens. PICARD_DESCENT_PAIR=0: singles.
        const Mat wt2 = matmul(ahead_->get(k + 1, &ahead_wait_ms_), P_);
        pair_ll.assign(n, 0.0);
        pair_bnd.assign(n, 0.0);
        if (ev_->eval_loss_screen2(wt.data(), wt2.data(), n, mu, cfg_.density, ll.data(), bnd.data(), pair_ll.data(),
                                   pair_bnd.data())) {
          pair_k = k + 1;
          ++screen_pairs_;
          via = first_loss_only ? " (pair)" : " (pair, descent)";
          got = true;
          eval_ms_ += now_ms() - t0;
          ++screen_passes_;
        } else {
          pairs_ok_ = false;  // not available here: single screens from now on
        }
      }
      if (!got && ev_->eval_loss_screen(wt.data(), n, mu, cfg_.density, ll.data(), bnd.data())) {
        got = true;
        eval_ms_ += now_ms() - t0;
        ++screen_passes_;
      }
      if (got) {
        screened = true;
        screen_seen_ = true;
        double lo = 0.0, eb = 0.0;
        for (size_t i = 0; i < n; ++i) {
          lo += (signs_[i] * ll[i] - std::fabs(signs_[i]) * bnd[i]) / (double)T_;
          eb += std::fabs(signs_[i]) * bnd[i] / (double)T_;
        }
        rejected = !(lo < current_loss_);  // exact loss ≥ lo ≥ current: the try fails
        if (trace_)
          std::fprintf(stderr, "[picard-screen] try %zu alpha %.3e margin %.3e bound %.3e ratio %.3e %s%s\n", k + 1, alpha,
                       lo + eb - current_loss_, eb, (lo + eb - current_loss_) / eb, rejected ? "reject" : "exact", via);
        prev_margin = lo + eb - current_loss_;
        if (level0 == 0) prev_eb0 = eb;
        // undecided, but the estimate lies above the current loss (a likely rejection): the
        // finer screens in turn, while the evaluator has them, before the full pass. Their
        // inputs are the reduced statistics, so every rank takes the same branch.
        for (int level = level0 + 1; !rejected && lo + eb > current_loss_; ++level) {
          const double tf = now_ms();
          if (!ev_->eval_loss_screen_fine(level, wt.data(), n, mu, cfg_.density, ll.data(), bnd.data())) break;
          eval_ms_ += now_ms() - tf;  // device time (host_ms counted it before round 5)
          ++screen_passes_;
          lo = 0.0;
          eb = 0.0;
          for (size_t i = 0; i < n; ++i) {
            lo += (signs_[i] * ll[i] - std::fabs(signs_[i]) * bnd[i]) / (double)T_;
            eb += std::fabs(signs_[i]) * bnd[i] / (double)T_;
          }
          rejected = !(lo < current_loss_);
          prev_margin = lo + eb - current_loss_;
          if (trace_)
            std::fprintf(stderr, "[picard-screen] fine%d try %zu alpha %.3e margin %.3e bound %.3e ratio %.3e %s\n", level,
                         k + 1, alpha, lo + eb - current_loss_, eb, (lo + eb - current_loss_) / eb,
                         rejected ? "reject" : "exact");
        }
      }
      if (rejected) {
        if (first_policy) first_n_[first_cell_] += 1.0;
        if (later_policy) later_n_ += 1.0;
        ++screen_rejects_;
        r.screened_out = true;  // no exact statistics for this W
        alpha /= 2.0;
        continue;
      }
      if (screened) {
        evaluate(r.w, &r.stats);
        r.partial = false;
      } else {
        screen_ok_ = false;  // this evaluator has no screen: the schedule above from now on
        if (k == 0 && !first_loss_only && (first_full_ || !split_first_)) {
          evaluate(r.w, &r.stats);
          r.partial = false;
        } else {
          r.partial = evaluate_loss(r.w, &r.stats);
        }
      }
    } else {
      r.partial = evaluate_loss(r.w, &r.stats);
    }
    r.screened_out = false;
    bool singular;
    r.loss = loss_of(r.stats, r.w, signs_, &singular);
    const bool accepted = r.loss < current_loss_;
    if (first_policy) {
      first_n_[first_cell_] += 1.0;
      if (accepted) first_acc_[first_cell_] += 1.0;
    }
    if (later_policy) {
      later_n_ += 1.0;
      if (accepted) later_acc_ += 1.0;
    }
    if (accepted) {
      r.success = true;
      r.step = scale(direction, alpha);
      return r;
    }
    alpha /= 2.0;
  }
  r.step = scale(direction, alpha);
  return r;
}

bool Solver::step() {
  // with the line-search helper running, its core is taken out of the team (see line_search)
  TeamGuard team(ahead_ ? std::max(1, host_team_threads() - 1) : host_team_threads());
  if (done_) return true;
  const double step_t0 = now_ms(), eval_t0 = eval_ms_, wait_t0 = ahead_wait_ms_;
  const size_t n = nc_;
  const double t_f = (double)T_;
  const bool ortho = cfg_.ortho != 0;
  last_evals_ = 0;
  n_iter_ = iter_;
  // core.rs:215-218 from the pass statistics of the current Y
  Mat g(n, n);
  for (size_t e = 0; e < n * n; ++e) g.a[e] = S_.G()[e] / t_f;
  std::vector<double> dmean(n);
  for (size_t i = 0; i < n; ++i) dmean[i] = S_.dpsi()[i] / t_f;
  bool sign_change = false;
  if (extended_) {  // core.rs:225-253
    for (size_t i = 0; i < n; ++i) {
      const double k = dmean[i] * C_(i, i) - g(i, i);
      signs_[i] = std::isnan(k) ? k : std::copysign(1.0, k);  // f64::signum
    }
    if (iter_ > 0)
      for (size_t i = 0; i < n; ++i)
        if (signs_[i] != old_signs_[i]) sign_change = true;
    old_signs_ = signs_;
    for (size_t i = 0; i < n; ++i) {
      for (size_t j = 0; j < n; ++j) g(i, j) *= signs_[i];
      dmean[i] *= signs_[i];  // mean(s_i ψ′_i) = s_i mean(ψ′_i): sign flips are exact
    }
    if (!ortho) g = add(g, C_);
  }
  std::vector<double> h_off(n, 1.0);  // core.rs:256-260
  if (ortho)
    for (size_t i = 0; i < n; ++i) h_off[i] = g(i, i);
  Mat h(n, n);
  if (ortho) {  // core.rs:263-272
    for (size_t i = 0; i < n; ++i)
      for (size_t j = 0; j < n; ++j) {
        const double v = 0.5 * (dmean[i] + dmean[j] - h_off[i] - h_off[j]);
        h(i, j) = std::fmax(v, cfg_.lambda_min);
      }
  } else {  // core.rs:274-275: ψ′ (signed, +1 when extended) · (Y∘Y)ᵀ / T
    const double* hr = S_.H();
    const double* y2 = S_.y2();
    for (size_t i = 0; i < n; ++i)
      for (size_t j = 0; j < n; ++j) {
        const double v = extended_ ? signs_[i] * hr[i * n + j] + y2[j] : hr[i * n + j];
        h(i, j) = v / t_f;
      }
    regularize_hessian(h, h_off, cfg_.lambda_min);
  }
  const Mat gs = g;  // signed gradient before the skew part (curvature rejection)
  if (ortho) {  // core.rs:280-286
    g = skew_symmetric(g);
  } else {
    for (size_t i = 0; i < n; ++i) g(i, i) -= 1.0;
  }
  gradient_norm_ = max_abs(g);  // core.rs:289
  if (gradient_norm_ < cfg_.tol) {
    converged_ = true;
    done_ = true;
    return true;
  }
  if (iter_ > 0 && has_prev_step_) {  // core.rs:296-313
    has_prev_step_ = false;
    if (has_g_old_) {
      Mat y_diff = sub(g, g_old_);
      const double r = 1.0 / dot_sum(prev_step_, y_diff);
      if (std::isfinite(r)) {
        mem_.s_list.push_back(prev_step_);
        mem_.y_list.push_back(y_diff);
        mem_.r_list.push_back(r);
        if (mem_.s_list.size() > cfg_.m) {
          mem_.s_list.pop_front();
          mem_.y_list.pop_front();
          mem_.r_list.pop_front();
        }
      }
    }
  }
  g_old_ = g;
  has_g_old_ = true;
  if (extended_ && sign_change) {  // core.rs:317-331: no extra pass (per-row sums kept)
    bool singular;
    current_loss_ = loss_of(S_, W_, signs_, &singular);
    mem_.clear();
  }
  const double t_grad = now_ms();
  Mat direction = compute_direction(g, h, h_off, mem_, ortho);  // core.rs:334
  const double t_dir = now_ms();
  // non-ortho: all tries in one multi-α pass unless the last search accepted at try 1
  // Schedule only (never a decision): the first try's pass also yields the next
  // gradient if it is accepted, so it is a full fused pass — unless the search
  // direction is not a descent direction (⟨g, D⟩ ≥ 0: the loss rises for small
  // α and the whole search almost surely fails), where a loss-only pass avoids
  // the wasted G stage. An accepted try is completed either way.
  const double slope = dot_sum(g, direction);
  set_curvature(g, gs, direction, slope);
  const double t_curv = now_ms();
  // First-try policy cell (schedule only): Picard's quadratic model along D, L(α) − L(0) ≈
  // α·slope + α²·qh/2 with qh = Σ h_ij·D_ij² (the Hessian approximation that preconditions D),
  // predicts a decrease at α = 1 when slope + qh/2 < 0 — exactly −slope/2 for the plain Newton
  // step. On the traced C3 and proxy fits every first try with that prediction was accepted (34),
  // and 17 of 19 without it that followed an accepted search failed (profiles/r04_j). Computed
  // from rank-identical data.
  {
    double qh = 0.0;
    if (ortho)
      for (size_t e = 0; e < n * n; ++e) qh += h.a[e] * direction.a[e] * direction.a[e];
    const bool model_decrease = ortho && slope < 0.0 && slope + 0.5 * qh < 0.0;
    first_cell_ = (model_decrease ? 2 : 0) + (first_full_ ? 1 : 0);
    pred_slope_ = ortho ? slope : 0.0;
    pred_qh_ = ortho ? qh : 0.0;
    if (trace_ && ortho)
      std::fprintf(stderr, "[picard-pred] iter %zu slope %.6e qh %.6e model %.3e first_full %d cell %d\n", iter_ + 1, slope,
                   qh, slope + 0.5 * qh, first_full_ ? 1 : 0, first_cell_);
  }
  const double t_ls0 = now_ms(), e_ls0 = eval_ms_;
  LsResult res = line_search(direction, cfg_.ls_tries, !first_full_, ortho && slope >= 0.0);
  const double ls_host = (now_ms() - t_ls0) - (eval_ms_ - e_ls0);
  const size_t first_tries = res.tries;
  const bool first_ok = res.success;
  first_full_ = res.success && res.tries == 1;
  if (!res.success) {  // core.rs:349-364
    mem_.clear();
    ls_curv_ = 0.0;  // the gradient direction descends: nothing to reject by curvature
    res = line_search(scale(g, -1.0), 10, false, false, true);
  }
  if (res.partial) complete(&res.stats);  // the new iterate needs G (H), Σψ′
  if (res.needs_full || res.screened_out) {  // rejected multi-try / screened last try kept as the iterate
    evaluate(res.w, &res.stats);
    bool singular;
    res.loss = loss_of(res.stats, res.w, signs_, &singular, res.det_sg, res.det_la);
  }
  {
    const double step_ms = now_ms() - step_t0, dev_ms = eval_ms_ - eval_t0;
    last_timing_[0] = step_ms;
    last_timing_[1] = dev_ms;
    last_timing_[2] = step_ms - dev_ms;
    last_timing_[3] = ahead_wait_ms_ - wait_t0;
  }
  if (trace_) {
    const double step_ms = now_ms() - step_t0, dev_ms = eval_ms_ - eval_t0;
    std::fprintf(stderr, "[picard-host] iter %zu grad_ms %.3f dir_ms %.3f curv_ms %.3f ls_host_ms %.3f\n", iter_ + 1,
                 t_grad - step_t0, t_dir - t_grad, t_curv - t_dir, ls_host);
    std::fprintf(stderr, "[picard-trace] iter %zu gnorm %.3e first_ls_tries %zu ok %d fallback %d fb_tries %zu partial %d slope %.3e"
                 " step_ms %.3f eval_ms %.3f host_ms %.3f map1_ms %.3f map_wait_ms %.3f screens %llu rejected %llu"
                 " curv_skips %llu screen_pairs %llu cvx_skips %llu\n",
                 iter_ + 1, gradient_norm_, first_tries, first_ok ? 1 : 0, first_ok ? 0 : 1, first_ok ? 0 : res.tries,
                 res.partial ? 1 : 0, slope, step_ms, dev_ms, step_ms - dev_ms, map1_ms_, ahead_wait_ms_ - wait_t0,
                 (unsigned long long)screen_passes_, (unsigned long long)screen_rejects_,
                 (unsigned long long)curv_skips_, (unsigned long long)screen_pairs_, (unsigned long long)cvx_skips_);
  }
  prev_step_ = std::move(res.step);
  has_prev_step_ = true;
  W_ = std::move(res.w);
  S_ = std::move(res.stats);
  if (extended_ && has_cov_) C_ = matmul_nt(W_, W_);  // core.rs:375-379 with cov = I
  current_loss_ = res.loss;
  if (cfg_.verbose)
    std::printf("iteration %zu, gradient norm = %s, loss = %s\n", iter_ + 1, rust_e4(gradient_norm_).c_str(),
                rust_e4(current_loss_).c_str());
  if (cfg_.verbose) std::fflush(stdout);
  ++iter_;
  if (iter_ >= cfg_.max_iter) done_ = true;
  return done_;
}

static double* dup(const double* p, size_t n) {
  double* q = new double[n];
  std::memcpy(q, p, n * sizeof(double));
  return q;
}

void Solver::finish(pc_result* out) {
  TeamGuard team(ahead_ ? std::max(1, host_team_threads() - 1) : host_team_threads());
  std::memset(out, 0, sizeof *out);
  Mat w = matmul(W_, w_init_);  // solver.rs:169
  if (!converged_ && cfg_.verbose)
    std::fprintf(stderr, "Warning: PICARD did not converge. Final gradient norm: %s, tolerance: %s\n",
                 rust_e4(gradient_norm_).c_str(), rust_e4(cfg_.tol).c_str());
  if (has_k_) {
    out->whitening = dup(K_.data(), K_.a.size());
    out->whitening_rows = K_.rows;
    out->whitening_cols = K_.cols;
  }
  out->unmixing = dup(w.data(), w.a.size());
  out->unmixing_rows = out->unmixing_cols = nc_;
  if (cfg_.want_sources) {
    const uint64_t nl = ev_->n_local();
    out->sources = new double[nc_ * nl];
    out->sources_rows = nc_;
    out->sources_cols = nl;
    Mat wt = matmul(W_, P_);
    ev_->sources(wt.data(), nc_, has_mu_ ? mu_.data() : nullptr, out->sources);
  }
  if (has_mu_) {
    out->mean = dup(mu_.data(), mu_.size());
    out->mean_len = mu_.size();
  }
  out->n_iterations = n_iter_ + 1;  // core.rs:396
  out->converged = converged_;
  out->gradient_norm = gradient_norm_;
  if (extended_) {
    out->signs = dup(signs_.data(), signs_.size());
    out->signs_len = signs_.size();
  }
  out->n_evaluations = total_evals_;
}

// solver.rs:218-249 on the device: with W orthogonal (it is the output of
// sym_decorrelation), x1 = Wᵀ·(W·x1), so E[g(Wx1) x1ᵀ] = (Σ g(y) yᵀ / p)·W
// comes from the same fused pass as the Picard gradient.
Mat Solver::ica_par(const Mat& w_init) {
  Mat w;
  if (!sym_decorrelation(w_init, &w)) throw singular_matrix();
  const double p = (double)T_;
  const size_t n = nc_;
  Mat base = has_k_ ? K_ : Mat::eye(nf_);
  for (uint64_t it = 0; it < cfg_.fastica_it; ++it) {
    Mat wt = matmul(w, base);
    EvalStats s;
    ev_->eval(wt.data(), n, has_mu_ ? mu_.data() : nullptr, cfg_.density, false, &s);
    Mat graw(n, n);
    graw.a.assign(s.G(), s.G() + n * n);
    Mat c = matmul(graw, w);
    for (double& v : c.a) v /= p;
    for (size_t i = 0; i < n; ++i) {
      const double gm = s.dpsi()[i] / p;
      for (size_t j = 0; j < n; ++j) c(i, j) -= gm * w(i, j);
    }
    if (!sym_decorrelation(c, &w)) throw singular_matrix();
  }
  if (cfg_.verbose) std::printf("FastICA pre-iterations complete.\n");
  return w;
}

// jade.rs:22-72 with the cumulant matrices from the device fourth-moment
// pass (jade.rs:78-131) and the Jacobi sweeps on rotated copies VᵀMV kept
// up to date per Givens rotation (same angles as jade.rs:137-185).
Mat Solver::jade(size_t max_iter, double tol) {
  // the device sweeps (one cooperative launch) unless PICARD_HOST_JADE asks for the
  // host's; either falls back to the host when the device cannot hold the matrices
  const int where = std::getenv("PICARD_HOST_JADE") ? JADE_SWEEPS_AUTO : JADE_SWEEPS_AUTO_DEVICE;
  JadeInfo info;
  Mat w = jade_warm_start(ev_, has_k_ ? K_ : Mat::eye(nf_), nc_, has_mu_ ? mu_.data() : nullptr, (double)T_,
                          max_iter, tol, cfg_.verbose, where, &info);
  if (trace_ || std::getenv("PICARD_TRACE"))
    std::fprintf(stderr, "[picard-trace] jade: moments %.3f s, %s sweeps %.3f s (%zu sweeps)\n", info.moments_s,
                 info.on_device ? "device" : "host", info.sweeps_s, info.sweeps);
  return w;
}

size_t jade_max_pairs() {
  const char* e = std::getenv("PICARD_JADE_MAX_PAIRS");
  return e ? (size_t)std::strtoull(e, nullptr, 0) : SIZE_MAX;
}

Mat jade_warm_start(Evaluator* ev, const Mat& base, size_t n, const double* mu, double T, size_t max_iter,
                    double tol, bool verbose, int where, JadeInfo* info) {
  *info = JadeInfo();
  if (n < 2) return Mat::eye(n);
  const size_t np = n * (n + 1) / 2;
  std::vector<double> m4(np * np);
  const auto tj0 = std::chrono::steady_clock::now();
  ev->moments4(base.data(), n, mu, m4.data());
  const auto tj1 = std::chrono::steady_clock::now();
  info->moments_s = std::chrono::duration<double>(tj1 - tj0).count();
  auto device_done = [&](const JadeSweepLog& log, const Mat& v) {
    if (verbose) {  // jade.rs:57-66
      for (size_t k = 0; k < log.theta10.size(); ++k)
        std::printf("JADE iteration %zu: max angle = %s\n", 10 * (k + 1), rust_e4(log.theta10[k]).c_str());
      if (log.converged) std::printf("JADE converged after %zu iterations\n", log.sweeps);
    }
    info->sweeps = log.sweeps;
    info->converged = log.converged;
    info->on_device = true;
    info->sweeps_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tj1).count();
    Mat w;
    if (!sym_decorrelation(v, &w)) throw singular_matrix();  // jade.rs:69
    return w;
  };
  // The device sweeps on cumulant matrices formed on the device from its copy of M (the same
  // values as the host build below): no host build, no upload
  if (where == JADE_SWEEPS_DEVICE || where == JADE_SWEEPS_AUTO_DEVICE) {
    JadeSweepLog log;
    Mat v = Mat::eye(n);
    if (ev->jade_sweeps_moments(n, T, max_iter, tol, v.data(), &log)) {
      if (verbose) std::printf("JADE: %zu cumulant matrices computed\n", np);
      return device_done(log, v);
    }
  }
  std::vector<size_t> pidx(n * n);
  {
    size_t q = 0;
    for (size_t i = 0; i < n; ++i)
      for (size_t j = i; j < n; ++j) { pidx[i * n + j] = pidx[j * n + i] = q++; }
  }
  const double t = T;
  // Cumulant matrices Q_ij (jade.rs:101-126), symmetrised, stored packed by
  // position: A[pos(k,l)][m] for k ≤ l, matrix index m innermost, so a Givens
  // step on (p, q) streams 2n contiguous rows of length np and the g-sums of
  // jade.rs:137-167 are three contiguous dot products.
  auto pos = [n](size_t k, size_t l) {  // k ≤ l
    return k * n - k * (k - 1) / 2 + (l - k);
  };
  const size_t npos = n * (n + 1) / 2;
  std::vector<double> A(npos * np);
  {
    std::vector<std::pair<size_t, size_t>> mpairs;
    for (size_t i = 0; i < n; ++i)
      for (size_t j = i; j < n; ++j) mpairs.emplace_back(i, j);
#pragma omp parallel for schedule(static)
    for (size_t m = 0; m < np; ++m) {
      {
        const size_t i = mpairs[m].first, j = mpairs[m].second;
        const size_t pij = pidx[i * n + j];
        auto q = [&](size_t k, size_t l) {
          const double e = m4[pij * np + pidx[k * n + l]] / t;
          const double d1 = (i == j && k == l) ? 1.0 : 0.0;
          const double d2 = (i == k && j == l) ? 1.0 : 0.0;
          const double d3 = (i == l && j == k) ? 1.0 : 0.0;
          return e - d1 - d2 - d3;
        };
        for (size_t k = 0; k < n; ++k)
          for (size_t l = k; l < n; ++l) A[pos(k, l) * np + m] = (q(k, l) + q(l, k)) / 2.0;
      }
    }
  }
  if (verbose) std::printf("JADE: %zu cumulant matrices computed\n", np);
  Mat v = Mat::eye(n);
  // The sweeps as one cooperative device launch (DeviceCtx::jade_sweeps) where
  // asked for and supported; the host sweeps otherwise.
  if (where == JADE_SWEEPS_DEVICE || where == JADE_SWEEPS_AUTO_DEVICE) {
    JadeSweepLog log;
    if (ev->jade_sweeps(A.data(), n, max_iter, tol, v.data(), &log)) return device_done(log, v);
    if (where == JADE_SWEEPS_DEVICE) throw unsupported("device JADE sweeps not supported for this shape");
  }
  // Sweeps in the reference's cyclic (p, q) order. The np matrices are split
  // into NCH fixed chunks; each thread rotates its chunks and forms their
  // partial g-sums for the NEXT pair, and every thread sums the partials in
  // chunk order to the same angle — one barrier per pair, results independent
  // of the thread count.
  constexpr size_t NCH = 64;
  const size_t nch = std::min<size_t>(NCH, np);
  std::vector<double> gpart(2 * nch * 3, 0.0);
  std::vector<std::pair<size_t, size_t>> pairs;
  for (size_t p = 0; p < n; ++p)
    for (size_t q = p + 1; q < n; ++q) pairs.emplace_back(p, q);
  auto chunk_lo = [&](size_t c) { return c * np / nch; };
  auto partial_g = [&](size_t p, size_t q, size_t c, double* g) {
    const size_t m0 = chunk_lo(c);
    jade_gsums(A.data() + pos(p, q) * np + m0, A.data() + pos(p, p) * np + m0, A.data() + pos(q, q) * np + m0,
               chunk_lo(c + 1) - m0, g);
  };
  size_t sweeps_done = 0;
  bool converged = false;
  // PICARD_JADE_MAX_PAIRS (test hook): stop after that many Givens pairs in all.
  // The sweeps amplify rounding exponentially, so parity
  // with the reference's literal form is checked on prefixes of a sweep.
  const size_t max_pairs = jade_max_pairs();
  // ≤ 8 threads pinned to neighbouring cores (one CCD on EPYC): the per-pair
  // barrier dominates otherwise (C5 on the MI355X host: 8 pinned threads 1.2 s,
  // 16 threads 2.4 s, unpinned 5–7 s). Affinities are restored afterwards.
  const int jade_threads = std::max(1, std::min(8, omp_get_max_threads()));
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  const bool have_mask = sched_getaffinity(0, sizeof allowed, &allowed) == 0;
  std::vector<int> cores;
  if (have_mask) {
    const int here = sched_getcpu();
    const int base = here >= 0 ? here / 8 * 8 : 0;
    for (int c = base; c < CPU_SETSIZE && (int)cores.size() < jade_threads; ++c)
      if (CPU_ISSET(c, &allowed)) cores.push_back(c);
    for (int c = 0; c < base && (int)cores.size() < jade_threads; ++c)
      if (CPU_ISSET(c, &allowed)) cores.push_back(c);
  }
#pragma omp parallel num_threads(jade_threads)
  {
    const int nt = omp_get_num_threads(), tid = omp_get_thread_num();
    const size_t c0 = nch * tid / nt, c1 = nch * (tid + 1) / nt;
    cpu_set_t mine, pin;
    const bool pinned = tid < (int)cores.size() && pthread_getaffinity_np(pthread_self(), sizeof mine, &mine) == 0;
    if (pinned) {
      CPU_ZERO(&pin);
      CPU_SET(cores[tid], &pin);
      (void)pthread_setaffinity_np(pthread_self(), sizeof pin, &pin);
    }
    int buf = 0;
    size_t done_pairs = 0;  // the same count on every thread
    for (size_t c = c0; c < c1; ++c) partial_g(pairs[0].first, pairs[0].second, c, &gpart[(0 * nch + c) * 3]);
#pragma omp barrier
    for (size_t it = 0; it < max_iter && !converged && done_pairs < max_pairs; ++it) {
      double max_theta = 0.0;
      for (size_t pi = 0; pi < pairs.size() && done_pairs < max_pairs; ++pi, ++done_pairs) {
        const size_t p = pairs[pi].first, q = pairs[pi].second;
        double g00 = 0, g01 = 0, g11 = 0;
        for (size_t c = 0; c < nch; ++c) {
          const double* g = &gpart[(buf * nch + c) * 3];
          g00 += g[0]; g01 += g[1]; g11 += g[2];
        }
        const double diff = g11 - g00;
        const double angle = (std::fabs(g01) < 1e-15 && std::fabs(diff) < 1e-15) ? 0.0 : 0.25 * std::atan2(2.0 * g01, diff);
        const double cs = std::cos(angle), sn = std::sin(angle);
        max_theta = std::fmax(max_theta, std::fabs(angle));
        if (tid == 0)
          for (size_t i = 0; i < n; ++i) {  // jade.rs:188-197
            const double vp = v(i, p), vq = v(i, q);
            v(i, p) = cs * vp - sn * vq;
            v(i, q) = sn * vp + cs * vq;
          }
        // A ← Gᵀ A G on this thread's chunks: rows/columns p, q of every matrix
        for (size_t c = c0; c < c1; ++c) {
          const size_t m0 = chunk_lo(c), m1 = chunk_lo(c + 1);
          for (size_t k = 0; k < n; ++k) {
            if (k == p || k == q) continue;
            double* ap = A.data() + (k < p ? pos(k, p) : pos(p, k)) * np;
            double* aq = A.data() + (k < q ? pos(k, q) : pos(q, k)) * np;
            givens_rows(ap + m0, aq + m0, m1 - m0, cs, sn);
          }
          double* app = A.data() + pos(p, p) * np;
          double* apq = A.data() + pos(p, q) * np;
          double* aqq = A.data() + pos(q, q) * np;
          for (size_t m = m0; m < m1; ++m) {  // the 2×2 block: columns, then rows
            const double a = app[m], b = apq[m], d = aqq[m];
            const double pp = cs * a - sn * b, pq = sn * a + cs * b;  // row p after M·G
            const double qp = cs * b - sn * d, qq = sn * b + cs * d;  // row q after M·G
            app[m] = cs * pp - sn * qp;
            apq[m] = cs * pq - sn * qq;
            aqq[m] = sn * pq + cs * qq;
          }
          if (pi + 1 < pairs.size())
            partial_g(pairs[pi + 1].first, pairs[pi + 1].second, c, &gpart[((buf ^ 1) * nch + c) * 3]);
          else
            partial_g(pairs[0].first, pairs[0].second, c, &gpart[((buf ^ 1) * nch + c) * 3]);
        }
        buf ^= 1;
#pragma omp barrier
      }
      if (tid == 0) {
        sweeps_done = it + 1;
        if (verbose && (it + 1) % 10 == 0)
          std::printf("JADE iteration %zu: max angle = %s\n", it + 1, rust_e4(max_theta).c_str());
        if (max_theta < tol) {
          if (verbose) std::printf("JADE converged after %zu iterations\n", it + 1);
          converged = true;
        }
      }
#pragma omp barrier
    }
    if (pinned) (void)pthread_setaffinity_np(pthread_self(), sizeof mine, &mine);
  }
  info->sweeps = sweeps_done;
  info->converged = converged;
  info->sweeps_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tj1).count();
  Mat w;
  if (!sym_decorrelation(v, &w)) throw singular_matrix();  // jade.rs:69
  return w;
}

}  // namespace pcamd
