// extern "C" boundary (include/picard_mi355x.h). Converts PicardError
// exceptions into pc_status codes + the src/error.rs:44-74 message text.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <utility>

#include "../../include/picard_mi355x.h"
#include "evaluator.hpp"
#include "host_linalg.hpp"
#include "host_solver.hpp"

namespace pcamd {
struct LocalGroup;
std::shared_ptr<LocalGroup> make_local_group(int world);
int local_group_world(const LocalGroup& g);
Evaluator* make_device_ctx(int device, int rank, int world, const char* uid, std::shared_ptr<LocalGroup> grp);
void device_ctx_comm_stats(const Evaluator* e, int64_t* out);
void device_ctx_comm_timing(const Evaluator* e, double* out);
void device_ctx_alloc_stats(const Evaluator* e, double* out);
void device_last_teardown(double* out);
void device_ctx_release_caches(Evaluator* e);
void device_ctx_load(Evaluator* e, const double* x, uint64_t nf, uint64_t nl, uint64_t nt, uint64_t t0);
void device_ctx_generate(Evaluator* e, uint64_t nf, uint64_t nt, uint64_t seed, double* a_out);
void device_ctx_download(Evaluator* e, double* out);
const double* device_ctx_sources_resident(Evaluator* e, const double* w, size_t nc, const double* mu, double* ms,
                                          uint64_t* ld);
uint64_t device_ctx_t0(const Evaluator* e);
void device_ctx_timing(const Evaluator* e, double* k, double* c);
void device_ctx_raw_eval(Evaluator* e, const double* w, size_t nc, const double* mu, int dens, double alpha,
                         bool need_h, double* stats);
int rccl_unique_id(char* out);
void device_ctx_kernel_stats(Evaluator* e, double* kernel_ms, double* call_ms, uint64_t* n, int reset);
void device_synchronize(int device);
void device_mem_info(int device, uint64_t* free_b, uint64_t* total_b);
void device_check_f32_transc(int device, double* out4);
void device_ctx_kernel_breakdown(Evaluator* e, double* ms, uint64_t* n, int reset);
void device_ctx_set_y_stage(Evaluator* e, int mode);
void device_ctx_set_g_stage(Evaluator* e, int mode);
uint64_t device_ctx_g8_passes(const Evaluator* e);
uint64_t device_ctx_multi_ybuf_passes(const Evaluator* e);
uint64_t device_ctx_int8_passes(const Evaluator* e);
void device_ctx_screen_stats(Evaluator* e, double* ms, uint64_t* n, int reset);
bool device_ctx_screen_digit_gram(Evaluator* e, double* lam, double* s4);
uint64_t device_ctx_screen_products(const Evaluator* e);
uint64_t device_ctx_screen_tries(const Evaluator* e);
}  // namespace pcamd

using namespace pcamd;

struct pc_ctx {
  std::unique_ptr<Evaluator> ev;
};
struct pc_solver {
  std::unique_ptr<Solver> s;
  Evaluator* ev = nullptr;  // the context it drives (group abort on failure)
};
struct pc_group {
  std::shared_ptr<LocalGroup> g;
};

namespace {
void set_err(char* err, size_t errlen, const std::string& m) {
  if (err && errlen) {
    std::strncpy(err, m.c_str(), errlen - 1);
    err[errlen - 1] = 0;
  }
}
template <class F>
int guarded(char* err, size_t errlen, F&& f) {
  try {
    f();
    if (err && errlen) err[0] = 0;
    return PC_OK;
  } catch (const PicardError& e) {
    set_err(err, errlen, e.what());
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, errlen, std::string("Computation error: ") + e.what());
    return PC_ERR_COMPUTATION;
  }
}

// The same, for calls on a context of a rank group: an error this rank may be alone in
// seeing (PC_ERR_COMPUTATION: HIP, HBM, a lost capability, a peer's abort) aborts the
// group, so the other ranks' collectives end with an error instead of waiting for this
// rank. Dimension / configuration errors are raised identically on every rank before
// any collective and leave the group usable.
template <class F>
int guarded_on(Evaluator* ev, char* err, size_t errlen, F&& f) {
  char local[512];
  if (!err || !errlen) {
    err = local;
    errlen = sizeof local;
  }
  const int rc = guarded(err, errlen, std::forward<F>(f));
  if (rc == PC_ERR_COMPUTATION && ev) ev->abort_group(err);
  return rc;
}

// Evaluator over caller callbacks (pc_host_evaluator): host-logic tests only.
struct CallbackEvaluator : Evaluator {
  pc_host_evaluator cb;
  explicit CallbackEvaluator(const pc_host_evaluator& c) : cb(c) {}
  uint64_t n_features() const override { return cb.n_features; }
  uint64_t n_samples() const override { return cb.n_samples; }
  uint64_t n_local() const override { return cb.n_samples; }
  void chk(int rc, const char* what) {
    if (rc) throw computation_error(std::string("evaluator callback failed: ") + what);
  }
  void rowsum(double* out) override { chk(cb.rowsum(cb.user, out), "rowsum"); }
  void gram(const double* mu, double* out) override { chk(cb.gram(cb.user, mu, out), "gram"); }
  void eval(const double* w, size_t nc, const double* mu, pc_density d, bool need_h, EvalStats* out) override {
    out->nc = nc;
    out->has_h = need_h;
    out->buf.assign(EvalStats::size(nc, need_h), 0.0);
    chk(cb.eval(cb.user, w, nc, mu, d, need_h ? PC_EVAL_NEED_H : 0u, out->buf.data()), "eval");
  }
  void sources(const double* w, size_t nc, const double* mu, double* out) override {
    chk(cb.sources(cb.user, w, nc, mu, out), "sources");
  }
  void moments4(const double* w, size_t nc, const double* mu, double* out) override {
    if (!cb.moments4) throw computation_error("moments4 callback missing");
    chk(cb.moments4(cb.user, w, nc, mu, out), "moments4");
  }
  bool eval_loss_multi(const double* w, const double* z, size_t nc, const double* mu, pc_density d,
                       const double* alphas, int na, double* ll_out, double* y2_out) override {
    if (!cb.eval_loss_multi) return false;
    chk(cb.eval_loss_multi(cb.user, w, z, nc, mu, d, alphas, (uint64_t)na, ll_out, y2_out), "eval_loss_multi");
    return true;
  }
  bool eval_loss_screen(const double* w, size_t nc, const double* mu, pc_density d, double* ll_out,
                        double* bound_out) override {
    if (!cb.eval_loss_screen) return false;
    chk(cb.eval_loss_screen(cb.user, w, nc, mu, d, ll_out, bound_out), "eval_loss_screen");
    return true;
  }
};

Mat full_unmixing_of(const pc_result* r) {
  Mat w(r->unmixing_rows, r->unmixing_cols);
  std::memcpy(w.data(), r->unmixing, w.a.size() * sizeof(double));
  if (!r->whitening) return w;
  Mat k(r->whitening_rows, r->whitening_cols);
  std::memcpy(k.data(), r->whitening, k.a.size() * sizeof(double));
  return matmul(w, k);
}
}  // namespace

extern "C" {

void pc_config_default(pc_config* c) {  // config.rs:64-85
  std::memset(c, 0, sizeof *c);
  c->density.kind = PC_DENSITY_TANH;
  c->density.alpha = 1.0;
  c->ortho = 1;
  c->whiten = 1;
  c->centering = 1;
  c->max_iter = 500;
  c->tol = 1e-7;
  c->m = 7;
  c->ls_tries = 10;
  c->lambda_min = 0.01;
  c->device = 0;
  c->want_sources = 1;
}

int pc_config_validate(const pc_config* c, char* err, size_t errlen) {  // config.rs:104-142
  return guarded(err, errlen, [&] {
    if (c->max_iter == 0) throw invalid_config("max_iter", "must be greater than 0");
    if (!(c->tol > 0.0)) throw invalid_config("tol", "must be positive");
    if (!(c->lambda_min > 0.0)) throw invalid_config("lambda_min", "must be positive");
    if (c->m == 0) throw invalid_config("m", "L-BFGS memory size must be at least 1");
    if (c->has_fastica_it && c->has_jade_it)
      throw invalid_config("jade_it", "cannot use both fastica_it and jade_it; choose one warm start method");
  });
}

int pc_fit(const double* x, uint64_t nf, uint64_t ns, const pc_config* cfg, pc_result* out, char* err,
           size_t errlen) {
  std::memset(out, 0, sizeof *out);
  return guarded(err, errlen, [&] {
    // validate before touching the device, as solver.rs:46 does first
    char e2[512];
    int rc = pc_config_validate(cfg, e2, sizeof e2);
    if (rc) throw PicardError(rc, e2);
    if (nf == 0 || ns == 0) throw invalid_dimensions("Input matrix cannot be empty");
    std::unique_ptr<Evaluator> ev(make_device_ctx(cfg->device, 0, 1, nullptr, nullptr));
    device_ctx_load(ev.get(), x, nf, ns, ns, 0);
    Solver s(ev.get(), *cfg);
    while (!s.step()) {
    }
    s.finish(out);
  });
}

int pc_fit_default(const double* x, uint64_t nf, uint64_t ns, pc_result* out, char* err, size_t errlen) {
  pc_config c;
  pc_config_default(&c);
  return pc_fit(x, nf, ns, &c, out, err, errlen);
}

int pc_fit_with_evaluator(const pc_host_evaluator* cb, const pc_config* cfg, pc_result* out, char* err,
                          size_t errlen) {
  std::memset(out, 0, sizeof *out);
  return guarded(err, errlen, [&] {
    CallbackEvaluator ev(*cb);
    Solver s(&ev, *cfg);
    while (!s.step()) {
    }
    s.finish(out);
  });
}

int pc_transform(const double* x, uint64_t nf, uint64_t ns, const pc_result* res, double* out, int32_t device,
                 char* err, size_t errlen) {  // solver.rs:199-214
  return guarded(err, errlen, [&] {
    Mat w = full_unmixing_of(res);
    if (w.cols != nf) throw invalid_dimensions("transform: n_features does not match the fitted model");
    std::unique_ptr<Evaluator> ev(make_device_ctx(device, 0, 1, nullptr, nullptr));
    device_ctx_load(ev.get(), x, nf, ns, ns, 0);
    ev->sources(w.data(), w.rows, res->mean, out);
  });
}

int pc_full_unmixing(const pc_result* r, double* out) {  // result.rs:39-44
  Mat w = full_unmixing_of(r);
  std::memcpy(out, w.data(), w.a.size() * sizeof(double));
  return PC_OK;
}

int pc_mixing(const pc_result* r, double* out) {  // result.rs:49-64
  Mat fw = full_unmixing_of(r);
  Mat wt = transpose(fw);
  Mat wtw = matmul(wt, fw);
  Mat inv;
  Mat m = (wtw.rows == wtw.cols && invert_matrix(wtw, &inv)) ? matmul(inv, wt) : wt;
  std::memcpy(out, m.data(), m.a.size() * sizeof(double));
  return PC_OK;
}

void pc_result_free(pc_result* r) {
  if (!r) return;
  delete[] r->whitening;
  delete[] r->unmixing;
  delete[] r->sources;
  delete[] r->mean;
  delete[] r->signs;
  std::memset(r, 0, sizeof *r);
}

double pc_amari_distance(const double* w, const double* a, uint64_t n) {  // utils.rs:82-103
  Mat W(n, n), A(n, n);
  std::memcpy(W.data(), w, n * n * sizeof(double));
  std::memcpy(A.data(), a, n * n * sizeof(double));
  Mat p = matmul(W, A);
  auto s = [&](bool tr) {
    double sum = 0.0;
    for (size_t i = 0; i < n; ++i) {
      double row_sum = 0.0, row_max = 0.0;
      for (size_t j = 0; j < n; ++j) {
        const double v = tr ? std::fabs(p(j, i)) : std::fabs(p(i, j));
        row_sum += v * v;
        row_max = std::fmax(row_max, v * v);
      }
      if (row_max > 1e-15) sum += row_sum / row_max - 1.0;
    }
    return sum;
  };
  return (s(false) + s(true)) / (2.0 * (double)n);
}

void pc_permute(const double* a_in, uint64_t n, int32_t scale, double* out) {  // utils.rs:16-69
  Mat a(n, n);
  std::memcpy(a.data(), a_in, n * n * sizeof(double));
  bool done = false;
  while (!done) {
    done = true;
    for (size_t i = 0; i < n; ++i)
      for (size_t j = 0; j < i; ++j) {
        const double dsq = a(i, i) * a(i, i) + a(j, j) * a(j, j);
        const double osq = a(i, j) * a(i, j) + a(j, i) * a(j, i);
        if (dsq < osq) {
          for (size_t c = 0; c < n; ++c) std::swap(a(i, c), a(j, c));
          done = false;
        }
      }
  }
  if (scale)
    for (size_t i = 0; i < n; ++i) {
      const double d = a(i, i);
      if (std::fabs(d) > 1e-10)
        for (size_t j = 0; j < n; ++j) a(i, j) /= d;
    }
  std::vector<double> cs(n, 0.0);
  for (size_t j = 0; j < n; ++j)
    for (size_t i = 0; i < n; ++i) cs[j] += std::fabs(a(i, j));
  std::vector<size_t> order(n);
  for (size_t i = 0; i < n; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return cs[x] < cs[y]; });
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) out[i * n + j] = a(order[i], order[j]);
}

const char* pc_error_name(int s) {
  switch (s) {
    case PC_OK: return "Ok";
    case PC_ERR_INVALID_DIMENSIONS: return "InvalidDimensions";
    case PC_ERR_SINGULAR_MATRIX: return "SingularMatrix";
    case PC_ERR_COMPUTATION: return "ComputationError";
    case PC_ERR_INVALID_CONFIG: return "InvalidConfig";
    case PC_ERR_NOT_CONVERGED: return "NotConverged";
    case PC_ERR_UNSUPPORTED: return "Unsupported";
    default: return "Unknown";
  }
}

const char* pc_version(void) { return "picard-mi355x 0.3.0 (reference picard-ica 0.1.6)"; }
int pc_abi_version(void) { return PC_ABI_VERSION; }

int pc_rccl_unique_id(char id_out[128]) { return rccl_unique_id(id_out) ? PC_ERR_COMPUTATION : PC_OK; }

int pc_ctx_create(int32_t device, int32_t rank, int32_t world, const char* id, pc_ctx** out, char* err,
                  size_t errlen) {
  *out = nullptr;
  return guarded(err, errlen, [&] {
    if (world < 1 || rank < 0 || rank >= world) throw invalid_dimensions("bad rank / world_size");
    auto* c = new pc_ctx;
    try {
      c->ev.reset(make_device_ctx(device, rank, world, id, nullptr));
    } catch (...) {
      delete c;
      throw;
    }
    *out = c;
  });
}

int pc_group_create_local(int32_t world, pc_group** out, char* err, size_t errlen) {
  *out = nullptr;
  return guarded(err, errlen, [&] {
    auto* g = new pc_group;
    g->g = make_local_group(world);
    *out = g;
  });
}

void pc_group_destroy(pc_group* g) { delete g; }

int pc_ctx_create_in_group(int32_t device, int32_t rank, pc_group* g, pc_ctx** out, char* err, size_t errlen) {
  *out = nullptr;
  return guarded(err, errlen, [&] {
    if (!g) throw invalid_dimensions("no rank group");
    const int world = local_group_world(*g->g);
    if (rank < 0 || rank >= world) throw invalid_dimensions("bad rank / world_size");
    auto* c = new pc_ctx;
    try {
      c->ev.reset(make_device_ctx(device, rank, world, nullptr, g->g));
    } catch (...) {
      delete c;
      throw;
    }
    *out = c;
  });
}

void pc_ctx_comm_stats(const pc_ctx* c, int64_t out[7]) { device_ctx_comm_stats(c->ev.get(), out); }
void pc_ctx_comm_timing(const pc_ctx* c, double out[2]) { device_ctx_comm_timing(c->ev.get(), out); }
void pc_ctx_alloc_stats(const pc_ctx* c, double out[9]) { device_ctx_alloc_stats(c->ev.get(), out); }
void pc_last_teardown(double out[4]) { device_last_teardown(out); }

void pc_ctx_abort(pc_ctx* c, const char* why) { c->ev->abort_group(why ? why : "aborted by the caller"); }

int pc_ctx_release_caches(pc_ctx* c, char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] { device_ctx_release_caches(c->ev.get()); });
}

void pc_ctx_destroy(pc_ctx* c) { delete c; }

int pc_ctx_load(pc_ctx* c, const double* x, uint64_t nf, uint64_t nl, uint64_t nt, uint64_t t0, char* err,
                size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] { device_ctx_load(c->ev.get(), x, nf, nl, nt, t0); });
}

int pc_ctx_generate(pc_ctx* c, uint64_t nf, uint64_t nt, uint64_t seed, double* a_out, char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] { device_ctx_generate(c->ev.get(), nf, nt, seed, a_out); });
}

int pc_ctx_download(pc_ctx* c, double* out) {
  try {
    device_ctx_download(c->ev.get(), out);
    return PC_OK;
  } catch (const PicardError& e) {
    return e.code;
  }
}

uint64_t pc_ctx_n_local(const pc_ctx* c) { return c->ev->n_local(); }
uint64_t pc_ctx_t0(const pc_ctx* c) { return device_ctx_t0(c->ev.get()); }

int pc_ctx_eval(pc_ctx* c, const double* w, uint64_t nc, const double* mu, pc_density d, uint32_t flags,
                double* stats, char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] {
    if (d.kind < 0 || d.kind > PC_DENSITY_CUBE) throw invalid_config("density", "unknown density kind");
    if (nc == 0 || nc > c->ev->n_features()) throw invalid_dimensions("nc must be in 1..=n_features");
    c->ev->want_y2 = (flags & PC_EVAL_SKIP_Y2) == 0;
    device_ctx_raw_eval(c->ev.get(), w, nc, mu, d.kind, d.alpha, (flags & PC_EVAL_NEED_H) != 0, stats);
  });
}

int pc_ctx_eval_loss(pc_ctx* c, const double* w, uint64_t nc, const double* mu, pc_density d, uint32_t flags,
                     double* stats, int32_t* kept, char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] {
    if (d.kind < 0 || d.kind > PC_DENSITY_CUBE) throw invalid_config("density", "unknown density kind");
    if (nc == 0 || nc > c->ev->n_features()) throw invalid_dimensions("nc must be in 1..=n_features");
    const bool h = (flags & PC_EVAL_NEED_H) != 0;
    c->ev->want_y2 = (flags & PC_EVAL_SKIP_Y2) == 0;
    EvalStats st;
    *kept = c->ev->eval_loss(w, nc, mu, d, h, &st) ? 1 : 0;
    const size_t off = *kept ? st.buf.size() - 2 * nc : 0;  // kept: only [Σℓ | Σy²] are written
    std::memcpy(stats + off, st.buf.data() + off, (st.buf.size() - off) * sizeof(double));
  });
}

int pc_ctx_eval_loss_multi(pc_ctx* c, const double* w, const double* z, uint64_t nc, const double* mu,
                           pc_density d, const double* alphas, uint64_t n_alpha, double* ll_out, double* y2_out,
                           char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] {
    if (d.kind < 0 || d.kind > PC_DENSITY_CUBE) throw invalid_config("density", "unknown density kind");
    if (nc == 0 || nc > c->ev->n_features()) throw invalid_dimensions("nc must be in 1..=n_features");
    if (n_alpha == 0) return;
    c->ev->want_y2 = true;  // this entry point returns Σy² (an earlier call may have turned it off)
    if (!c->ev->eval_loss_multi(w, z, nc, mu, d, alphas, (int)n_alpha, ll_out, y2_out))
      throw unsupported("multi-try loss pass not available for this shape");
  });
}

int pc_ctx_eval_loss_multi_bound(pc_ctx* c, const double* w, const double* z, uint64_t nc, const double* mu,
                                 pc_density d, const double* alphas, uint64_t n_alpha, double* ll_out,
                                 double* bnd_out, char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] {
    if (d.kind < 0 || d.kind > PC_DENSITY_CUBE) throw invalid_config("density", "unknown density kind");
    if (nc == 0 || nc > c->ev->n_features()) throw invalid_dimensions("nc must be in 1..=n_features");
    if (n_alpha == 0) return;
    c->ev->want_y2 = false;
    if (!c->ev->eval_loss_multi_bound(w, z, nc, mu, d, alphas, (int)n_alpha, ll_out, bnd_out))
      throw unsupported("bounded multi-try pass not available here");
  });
}

int pc_ctx_eval_complete(pc_ctx* c, pc_density d, uint32_t flags, double* stats, char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] {
    // only the entries [G | H | Σψ′] are written; Σℓ, Σy² of `stats` are left as they are
    c->ev->eval_complete_into(d, (flags & PC_EVAL_NEED_H) != 0, stats);
  });
}

int pc_ctx_rowsum(pc_ctx* c, double* out, char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] { c->ev->rowsum(out); });
}

int pc_ctx_gram(pc_ctx* c, const double* mu, double* out, char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] { c->ev->gram(mu, out); });
}

int pc_ctx_sources(pc_ctx* c, const double* w, uint64_t nc, const double* mu, double* out, char* err,
                   size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] { c->ev->sources(w, nc, mu, out); });
}

int pc_ctx_sources_device(pc_ctx* c, const double* w, uint64_t nc, const double* mu, const double** dev_out,
                          uint64_t* ld_out, double* kernel_ms, char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] {
    uint64_t ld = 0;
    double ms = 0.0;
    const double* p = device_ctx_sources_resident(c->ev.get(), w, nc, mu, &ms, &ld);
    if (dev_out) *dev_out = p;
    if (ld_out) *ld_out = ld;
    if (kernel_ms) *kernel_ms = ms;
  });
}

int pc_ctx_moments4(pc_ctx* c, const double* w, uint64_t nc, const double* mu, double* out, char* err,
                    size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] { c->ev->moments4(w, nc, mu, out); });
}

void pc_ctx_last_timing(const pc_ctx* c, double* k, double* call) { device_ctx_timing(c->ev.get(), k, call); }

void pc_ctx_kernel_stats(pc_ctx* c, double* kernel_ms, double* call_ms, uint64_t* n, int32_t reset) {
  device_ctx_kernel_stats(c->ev.get(), kernel_ms, call_ms, n, reset);
}

void pc_ctx_kernel_breakdown(pc_ctx* c, double ms[4], uint64_t n[4], int32_t reset) {
  device_ctx_kernel_breakdown(c->ev.get(), ms, n, reset);
}

int pc_ctx_set_y_stage(pc_ctx* c, int32_t mode) {
  if (mode != PC_YSTAGE_AUTO && mode != PC_YSTAGE_F64 && mode != PC_YSTAGE_INT8_EXACT) return PC_ERR_INVALID_CONFIG;
  device_ctx_set_y_stage(c->ev.get(), mode);
  return PC_OK;
}

uint64_t pc_ctx_int8_passes(const pc_ctx* c) { return device_ctx_int8_passes(c->ev.get()); }

int pc_ctx_set_g_stage(pc_ctx* c, int32_t mode) {
  if (mode != PC_GSTAGE_AUTO && mode != PC_GSTAGE_F64) return PC_ERR_INVALID_CONFIG;
  device_ctx_set_g_stage(c->ev.get(), mode);
  return PC_OK;
}

uint64_t pc_ctx_g8_passes(const pc_ctx* c) { return device_ctx_g8_passes(c->ev.get()); }
uint64_t pc_ctx_multi_ybuf_passes(const pc_ctx* c) { return device_ctx_multi_ybuf_passes(c->ev.get()); }

int pc_ctx_matrix_exp(pc_ctx* c, const double* a, uint64_t n, double* out, char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] {
    if (!c->ev->device_matrix_exp(a, n, out)) throw unsupported("device matrix exponential for this shape / series");
  });
}

void pc_matrix_exp(const double* a, uint64_t n, double* out) {  // math.rs:38-74
  Mat A(n, n);
  std::memcpy(A.data(), a, n * n * sizeof(double));
  const Mat e = matrix_exp(A);
  std::memcpy(out, e.data(), n * n * sizeof(double));
}

int pc_ctx_eval_loss_screen(pc_ctx* c, const double* w, uint64_t nc, const double* mu, pc_density density,
                            double* ll_out, double* bound_out, char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] {
    if (!c->ev->eval_loss_screen(w, nc, mu, density, ll_out, bound_out))
      throw unsupported("no line-search screen for this shape / density");
  });
}

int pc_ctx_eval_loss_screen2(pc_ctx* c, const double* w1, const double* w2, uint64_t nc, const double* mu,
                             pc_density density, double* ll1, double* bound1, double* ll2, double* bound2,
                             char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] {
    if (!c->ev->eval_loss_screen2(w1, w2, nc, mu, density, ll1, bound1, ll2, bound2))
      throw unsupported("no paired line-search screen for this shape / density");
  });
}

void pc_ctx_screen_stats(pc_ctx* c, double* ms, uint64_t* n, int32_t reset) {
  device_ctx_screen_stats(c->ev.get(), ms, n, reset);
}

uint64_t pc_ctx_screen_tries(const pc_ctx* c) { return device_ctx_screen_tries(c->ev.get()); }
uint64_t pc_ctx_screen_products(const pc_ctx* c) { return device_ctx_screen_products(c->ev.get()); }

int pc_ctx_screen_digit_gram(pc_ctx* c, double* lam, double* s4, char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] {
    if (!device_ctx_screen_digit_gram(c->ev.get(), lam, s4)) throw unsupported("no int8 digit image for this context");
  });
}

int pc_device_check_fp32_transcendentals(int32_t device, double out[4]) {
  try {
    device_check_f32_transc(device, out);
    return PC_OK;
  } catch (const PicardError& e) {
    return e.code;
  }
}

int pc_device_mem_info(int32_t device, uint64_t* free_bytes, uint64_t* total_bytes) {
  try {
    device_mem_info(device, free_bytes, total_bytes);
    return PC_OK;
  } catch (const PicardError& e) {
    return e.code;
  }
}

int pc_device_synchronize(int32_t device) {
  try {
    device_synchronize(device);
    return PC_OK;
  } catch (const PicardError& e) {
    return e.code;
  }
}

int pc_ctx_jade(pc_ctx* c, const double* w, uint64_t nc, const double* mu, uint64_t max_iter, double tol,
                int32_t where, double* w_out, uint64_t sweeps_out[3], char* err, size_t errlen) {
  return guarded_on(c->ev.get(), err, errlen, [&] {
    const uint64_t nf = c->ev->n_features();
    if (nc == 0 || nc > nf) throw invalid_dimensions("n_components must be in 1..=n_features");
    // the cumulants need the fourth moments of ALL samples: a detached shard only has its own
    if (c->ev->partial_sums())
      throw invalid_config("ctx", "a detached shard context returns partial moments; sum pc_ctx_moments4 over the "
                                  "shards and run the sweeps on the host");
    if (where < PC_JADE_AUTO || where > PC_JADE_HOST) throw invalid_config("where", "unknown sweep placement");
    Mat base(nc, nf);
    std::memcpy(base.data(), w, nc * nf * sizeof(double));
    JadeInfo info;
    Mat r = jade_warm_start(c->ev.get(), base, nc, mu, (double)c->ev->n_samples(), max_iter, tol, false, where,
                            &info);
    std::memcpy(w_out, r.data(), nc * nc * sizeof(double));
    if (sweeps_out) {
      sweeps_out[0] = info.sweeps;
      sweeps_out[1] = info.converged ? 1 : 0;
      sweeps_out[2] = info.on_device ? 1 : 0;
    }
  });
}

int pc_solver_create(pc_ctx* c, const pc_config* cfg, pc_solver** out, char* err, size_t errlen) {
  *out = nullptr;
  return guarded_on(c->ev.get(), err, errlen, [&] {
    char e2[512];
    int rc = pc_config_validate(cfg, e2, sizeof e2);
    if (rc) throw PicardError(rc, e2);
    if (c->ev->partial_sums())
      throw invalid_config("ctx", "a detached shard context (world_size > 1 without an RCCL id) returns partial "
                                  "sums; drive the shards with pc_fit_with_evaluator");
    auto* s = new pc_solver;
    s->ev = c->ev.get();
    try {
      s->s.reset(new Solver(c->ev.get(), *cfg));
    } catch (...) {
      delete s;
      throw;
    }
    *out = s;
  });
}

int pc_solver_step(pc_solver* s, int32_t* done, char* err, size_t errlen) {
  return guarded_on(s->ev, err, errlen, [&] { *done = s->s->step() ? 1 : 0; });
}

int pc_solver_finish(pc_solver* s, pc_result* out, char* err, size_t errlen) {
  std::memset(out, 0, sizeof *out);
  return guarded_on(s->ev, err, errlen, [&] { s->s->finish(out); });
}

void pc_solver_destroy(pc_solver* s) { delete s; }

void pc_solver_timing(const pc_solver* s, double out[4]) { s->s->last_timing(out); }
void pc_solver_setup_timing(const pc_solver* s, double out[5]) { s->s->setup_timing(out); }

void pc_solver_last(const pc_solver* s, double* loss, double* gn, uint64_t* n_evals) {
  if (loss) *loss = s->s->last_loss();
  if (gn) *gn = s->s->last_gnorm();
  if (n_evals) *n_evals = s->s->last_evals();
}

}  // extern "C"
