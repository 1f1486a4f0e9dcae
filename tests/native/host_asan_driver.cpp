// Host-code sanitizer run (AddressSanitizer + UndefinedBehaviorSanitizer on the host sources only;
// no GPU, no HIP call): pc_fit_with_evaluator over C++ callbacks that compute the pass statistics
// of the tanh / exp / cube densities directly (the sums of oracle/picard_oracle.py pass_stats), so
// the solver's whole host pipeline — whitening, warm starts, L-BFGS, both line searches (multi-try
// and screened tries, the curvature and convexity rejections), result assembly — runs under the
// sanitizers. Built and run by tests/test_host_sanitizers.py (make -f tests/native/Makefile.asan).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "picard_mi355x.h"

namespace {

struct Data {
  size_t nf, t;
  std::vector<double> x;  // nf × t, row-major
};

double ell(int kind, double a, double y) {  // density.rs log_lik
  if (kind == PC_DENSITY_TANH) return std::fabs(y) + std::log1p(std::exp(-2.0 * a * std::fabs(y))) / a;
  if (kind == PC_DENSITY_EXP) return -std::exp(-a * y * y / 2.0) / a;
  return y * y * y * y / 4.0;
}
void score(int kind, double a, double y, double* psi, double* dpsi) {  // density.rs score_and_der
  if (kind == PC_DENSITY_TANH) {
    const double s = std::tanh(a * y);
    *psi = s;
    *dpsi = a * (1.0 - s * s);
  } else if (kind == PC_DENSITY_EXP) {
    const double k = std::exp(-a * y * y / 2.0);
    *psi = y * k;
    *dpsi = (1.0 - a * y * y) * k;
  } else {
    *psi = y * y * y;
    *dpsi = 3.0 * y * y;
  }
}

void sources_of(const Data& d, const double* w, size_t nc, const double* mu, std::vector<double>& y) {
  y.assign(nc * d.t, 0.0);
  for (size_t i = 0; i < nc; ++i)
    for (size_t k = 0; k < d.nf; ++k) {
      const double wik = w[i * d.nf + k], m = mu ? mu[k] : 0.0;
      for (size_t s = 0; s < d.t; ++s) y[i * d.t + s] += wik * (d.x[k * d.t + s] - m);
    }
}

int cb_rowsum(void* u, double* out) {
  const Data& d = *(const Data*)u;
  for (size_t k = 0; k < d.nf; ++k) {
    double s = 0.0;
    for (size_t t = 0; t < d.t; ++t) s += d.x[k * d.t + t];
    out[k] = s;
  }
  return 0;
}
int cb_gram(void* u, const double* mu, double* out) {
  const Data& d = *(const Data*)u;
  for (size_t i = 0; i < d.nf; ++i)
    for (size_t j = 0; j < d.nf; ++j) {
      double s = 0.0;
      for (size_t t = 0; t < d.t; ++t)
        s += (d.x[i * d.t + t] - (mu ? mu[i] : 0.0)) * (d.x[j * d.t + t] - (mu ? mu[j] : 0.0));
      out[i * d.nf + j] = s;
    }
  return 0;
}
int cb_eval(void* u, const double* w, uint64_t nc, const double* mu, pc_density dens, uint32_t flags, double* st) {
  const Data& d = *(const Data*)u;
  std::vector<double> y, psi, dpsi;
  sources_of(d, w, nc, mu, y);
  psi.resize(y.size());
  dpsi.resize(y.size());
  for (size_t e = 0; e < y.size(); ++e) score(dens.kind, dens.alpha, y[e], &psi[e], &dpsi[e]);
  const bool h = flags & 1;
  const size_t nn = nc * nc;
  double* G = st;
  double* H = st + nn;
  double* rows = st + (h ? 2 : 1) * nn;
  for (size_t i = 0; i < nc; ++i)
    for (size_t j = 0; j < nc; ++j) {
      double g = 0.0, hh = 0.0;
      for (size_t t = 0; t < d.t; ++t) {
        g += psi[i * d.t + t] * y[j * d.t + t];
        if (h) hh += dpsi[i * d.t + t] * y[j * d.t + t] * y[j * d.t + t];
      }
      G[i * nc + j] = g;
      if (h) H[i * nc + j] = hh;
    }
  for (size_t i = 0; i < nc; ++i) {
    double sd = 0.0, sl = 0.0, sq = 0.0;
    for (size_t t = 0; t < d.t; ++t) {
      const double v = y[i * d.t + t];
      sd += dpsi[i * d.t + t];
      sl += ell(dens.kind, dens.alpha, v);
      sq += v * v;
    }
    rows[i] = sd;
    rows[nc + i] = sl;
    rows[2 * nc + i] = sq;
  }
  return 0;
}
int cb_sources(void* u, const double* w, uint64_t nc, const double* mu, double* out) {
  const Data& d = *(const Data*)u;
  std::vector<double> y;
  sources_of(d, w, nc, mu, y);
  std::memcpy(out, y.data(), y.size() * sizeof(double));
  return 0;
}
int cb_moments4(void* u, const double* w, uint64_t nc, const double* mu, double* out) {
  const Data& d = *(const Data*)u;  // z = [y_i·y_j for i ≤ j] (npair × T), out = z·zᵀ
  std::vector<double> y;
  sources_of(d, w, nc, mu, y);
  const size_t np = nc * (nc + 1) / 2;
  std::vector<double> z(np * d.t);
  size_t q = 0;
  for (size_t i = 0; i < nc; ++i)
    for (size_t j = i; j < nc; ++j, ++q)
      for (size_t t = 0; t < d.t; ++t) z[q * d.t + t] = y[i * d.t + t] * y[j * d.t + t];
  for (size_t a = 0; a < np; ++a)
    for (size_t b = 0; b < np; ++b) {
      double s = 0.0;
      for (size_t t = 0; t < d.t; ++t) s += z[a * d.t + t] * z[b * d.t + t];
      out[a * np + b] = s;
    }
  return 0;
}
int cb_multi(void* u, const double* w, const double* z, uint64_t nc, const double* mu, pc_density dens,
             const double* alphas, uint64_t na, double* ll, double* y2) {
  const Data& d = *(const Data*)u;
  std::vector<double> wa(nc * d.nf), y;
  for (uint64_t j = 0; j < na; ++j) {
    for (size_t e = 0; e < wa.size(); ++e) wa[e] = w[e] + alphas[j] * z[e];
    sources_of(d, wa.data(), nc, mu, y);
    for (size_t i = 0; i < nc; ++i) {
      double sl = 0.0, sq = 0.0;
      for (size_t t = 0; t < d.t; ++t) {
        const double v = y[i * d.t + t];
        sl += ell(dens.kind, dens.alpha, v);
        sq += v * v;
      }
      ll[j * nc + i] = sl;
      y2[j * nc + i] = sq;
    }
  }
  return 0;
}
int cb_screen(void* u, const double* w, uint64_t nc, const double* mu, pc_density dens, double* ll, double* bnd) {
  const Data& d = *(const Data*)u;
  std::vector<double> y;
  sources_of(d, w, nc, mu, y);
  for (size_t i = 0; i < nc; ++i) {
    double sl = 0.0;
    for (size_t t = 0; t < d.t; ++t) sl += ell(dens.kind, dens.alpha, y[i * d.t + t]);
    ll[i] = sl;
    bnd[i] = 1e-9 * std::fabs(sl) + 1e-12;
  }
  return 0;
}

int fit(const Data& d, int ortho, int extended, int kind, bool multi, bool screen, int fastica, int jade = 0) {
  pc_host_evaluator ev{};
  ev.user = (void*)&d;
  ev.n_features = d.nf;
  ev.n_samples = d.t;
  ev.rowsum = cb_rowsum;
  ev.gram = cb_gram;
  ev.eval = cb_eval;
  ev.sources = cb_sources;
  ev.moments4 = cb_moments4;
  ev.eval_loss_multi = multi ? cb_multi : nullptr;
  ev.eval_loss_screen = screen ? cb_screen : nullptr;
  pc_config cfg;
  pc_config_default(&cfg);
  cfg.ortho = ortho;
  cfg.has_extended = 1;
  cfg.extended = extended;
  cfg.density.kind = kind;
  cfg.density.alpha = 1.0;
  cfg.max_iter = 60;
  cfg.has_random_state = 1;
  cfg.random_state = 7;
  cfg.want_sources = 1;
  if (jade) {
    cfg.has_jade_it = 1;
    cfg.jade_it = (uint64_t)jade;
  }
  if (fastica) {
    cfg.has_fastica_it = 1;
    cfg.fastica_it = (uint64_t)fastica;
  }
  pc_result r{};
  char err[512] = {0};
  const int rc = pc_fit_with_evaluator(&ev, &cfg, &r, err, sizeof err);
  std::printf("ortho %d extended %d density %d multi %d screen %d fastica %d jade %d: rc %d iterations %llu converged %d%s%s\n",
              ortho, extended, kind, multi ? 1 : 0, screen ? 1 : 0, fastica, jade, rc, (unsigned long long)r.n_iterations,
              r.converged, rc ? " err: " : "", rc ? err : "");
  if (rc == PC_OK) pc_result_free(&r);
  return rc;
}

}  // namespace

int main() {
  // the bench mixture's shape at a size the callbacks finish in seconds: Laplace sources, a
  // random mixing
  Data d;
  d.nf = std::getenv("PC_DRV_NF") ? (size_t)std::atoi(std::getenv("PC_DRV_NF")) : 8;  // (host-time probes)
  d.t = std::getenv("PC_DRV_T") ? (size_t)std::atoi(std::getenv("PC_DRV_T")) : 3000;
  const int only = std::getenv("PC_DRV_FIT") ? std::atoi(std::getenv("PC_DRV_FIT")) : -1;
  std::mt19937_64 rng(42);
  std::exponential_distribution<double> ex(1.0);
  std::bernoulli_distribution sg(0.5);
  std::normal_distribution<double> nd(0.0, 1.0);
  std::vector<double> s(d.nf * d.t), a(d.nf * d.nf);
  for (double& v : s) v = sg(rng) ? ex(rng) : -ex(rng);
  for (double& v : a) v = nd(rng);
  d.x.assign(d.nf * d.t, 0.0);
  for (size_t i = 0; i < d.nf; ++i)
    for (size_t k = 0; k < d.nf; ++k)
      for (size_t t = 0; t < d.t; ++t) d.x[i * d.t + t] += a[i * d.nf + k] * s[k * d.t + t];
  int bad = 0;
  if (only == 0) return fit(d, 1, 1, PC_DENSITY_TANH, false, true, 0) != PC_OK;  // C3's kind alone
  bad += fit(d, 1, 1, PC_DENSITY_TANH, false, true, 0) != PC_OK;   // screened orthogonal (curvature)
  bad += fit(d, 1, 0, PC_DENSITY_TANH, false, false, 0) != PC_OK;  // every try exact
  bad += fit(d, 0, 0, PC_DENSITY_TANH, true, false, 0) != PC_OK;   // multi-try (convexity)
  bad += fit(d, 0, 1, PC_DENSITY_TANH, true, false, 0) != PC_OK;   // extended non-orthogonal
  bad += fit(d, 0, 0, PC_DENSITY_EXP, false, false, 0) != PC_OK;   // per-try passes
  bad += fit(d, 1, 0, PC_DENSITY_CUBE, false, false, 3) != PC_OK;  // FastICA warm start
  bad += fit(d, 1, 1, PC_DENSITY_TANH, false, true, 0, 20) != PC_OK;  // JADE warm start (host sweeps)
  std::printf("%s\n", bad ? "FAILED" : "all fits ok");
  return bad ? 1 : 0;
}
