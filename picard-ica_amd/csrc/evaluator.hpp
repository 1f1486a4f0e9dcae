// The operator boundary between the host Picard driver and the device.
// Everything the reference computes over the full N×T data
// (src/core.rs:215-274, :39-85; src/whitening.rs:24-116; src/jade.rs:91-113)
// is one of these calls; everything else is N×N host work.
#pragma once
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/picard_mi355x.h"

namespace pcamd {

// src/error.rs:9-42 as an exception carrying the pc_status code and the
// Display text of src/error.rs:44-74.
struct PicardError : std::runtime_error {
  int code;
  PicardError(int c, const std::string& msg) : std::runtime_error(msg), code(c) {}
};
inline PicardError invalid_dimensions(const std::string& m) {
  return PicardError(PC_ERR_INVALID_DIMENSIONS, "Invalid dimensions: " + m);
}
inline PicardError singular_matrix() {
  return PicardError(PC_ERR_SINGULAR_MATRIX, "Singular matrix encountered during computation");
}
inline PicardError computation_error(const std::string& m) {
  return PicardError(PC_ERR_COMPUTATION, "Computation error: " + m);
}
// A capability miss of the operator boundary (pc_status PC_ERR_UNSUPPORTED): the pass is
// not available here, nothing ran, and a rank group is not aborted (guarded_on).
inline PicardError unsupported(const std::string& m) { return PicardError(PC_ERR_UNSUPPORTED, "Unsupported: " + m); }
inline PicardError invalid_config(const std::string& p, const std::string& m) {
  return PicardError(PC_ERR_INVALID_CONFIG, "Invalid configuration for '" + p + "': " + m);
}

// Packed statistics of one fused pass (see pc_ctx_eval).
struct EvalStats {
  size_t nc = 0;
  bool has_h = false;
  std::vector<double> buf;
  const double* G() const { return buf.data(); }
  const double* H() const { return buf.data() + nc * nc; }
  const double* dpsi() const { return buf.data() + (has_h ? 2 : 1) * nc * nc; }
  const double* ll() const { return dpsi() + nc; }
  const double* y2() const { return dpsi() + 2 * nc; }
  static size_t size(size_t nc, bool h) { return (h ? 2 : 1) * nc * nc + 3 * nc; }
};

struct JadeSweepLog {
  size_t sweeps = 0;
  bool converged = false;
  std::vector<double> theta10;  // max |θ| of sweeps 10, 20, …
};

class Evaluator {
 public:
  virtual ~Evaluator() = default;
  // Σy² (the last nc stats) is always computed with H; without H only if
  // want_y2 (the orthogonal solver never reads it: core.rs:221 computes Y∘Y
  // but only :274 and the extended non-orthogonal loss use it). Otherwise 0.
  bool want_y2 = true;
  // Host work the caller overlaps with its next pass (the non-ortho search's per-try W_j and
  // log|det W_j|): an evaluator that can calls run_overlap() once the pass is enqueued and before
  // it waits for it; the caller runs whatever is still pending after the call itself.
  std::function<void()> overlap_;
  void run_overlap() {
    if (overlap_) {
      auto f = std::move(overlap_);
      overlap_ = nullptr;
      f();
    }
  }
  // kernel time (ms) of the last pass this evaluator ran, < 0 when it does not know: the caller
  // books the part of an overlap hook that outlasted the pass as host time
  virtual double last_pass_kernel_ms() const { return -1.0; }
  virtual uint64_t n_features() const = 0;
  virtual uint64_t n_samples() const = 0;  // global T over all ranks
  // true for a detached shard (world > 1, no communicator): every statistic is
  // this shard's partial sum, so the host driver cannot run on it alone
  virtual bool partial_sums() const { return false; }
  // This rank failed with an error the other ranks may not see (HIP, HBM, a lost
  // capability): end every rank's pending and later collectives with an error instead
  // of leaving them waiting. No-op without a communicator.
  virtual void abort_group(const std::string& why) noexcept { (void)why; }
  virtual void rowsum(double* out) = 0;
  virtual void gram(const double* mu, double* out) = 0;
  virtual void eval(const double* w, size_t nc, const double* mu, pc_density d, bool need_h,
                    EvalStats* out) = 0;
  // this rank's shard of Y = W·(X−μ) (nc × n_local)
  virtual void sources(const double* w, size_t nc, const double* mu, double* out) = 0;
  virtual uint64_t n_local() const = 0;
  virtual void moments4(const double* w, size_t nc, const double* mu, double* out) = 0;
  // Line-search try (core.rs:124-127 only needs Σℓ, Σy²). May compute just
  // those; returns true in that case, and then eval_complete fills G (H) and
  // Σψ′ of the SAME W — from Y kept in HBM when `keep` and there is room,
  // otherwise by recomputing the pass. A device that cannot split falls back
  // to a full pass and returns false.
  virtual bool eval_loss(const double* w, size_t nc, const double* mu, pc_density d, bool need_h,
                         EvalStats* out, bool keep = true) {
    (void)keep;
    eval(w, nc, mu, d, need_h, out);
    return false;
  }
  virtual void eval_complete(pc_density d, bool need_h, EvalStats* out) { (void)d; (void)need_h; (void)out; }
  // Orthogonal line-search screen: Σℓ of a CHEAPER approximation of the loss-only
  // pass at w (ll_out, nc) and, per row, a rigorous bound on how far the exact
  // pass's Σℓ can lie from it (bound_out, nc; any rounding included), both summed
  // over ranks. The solver rejects a try without the exact pass only when even
  // the bound cannot bring its loss below the current one, so no decision of
  // core.rs:127-140 changes. false = no screen here (the try is evaluated exactly).
  virtual bool eval_loss_screen(const double* w, size_t nc, const double* mu, pc_density d, double* ll_out,
                                double* bound_out) {
    (void)w; (void)nc; (void)mu; (void)d; (void)ll_out; (void)bound_out;
    return false;
  }
  // The same on finer (slower, tighter) approximations, level 1, 2, … in turn, for tries the
  // screens so far left undecided although their estimate lies above the current loss.
  // false = no such level. Rank-independent availability (the levels issue collectives).
  virtual bool eval_loss_screen_fine(int level, const double* w, size_t nc, const double* mu, pc_density d,
                                     double* ll_out, double* bound_out) {
    (void)level; (void)w; (void)nc; (void)mu; (void)d; (void)ll_out; (void)bound_out;
    return false;
  }
  // Two tries' screens in one pass (w1, w2: the same shape): each try's [Σℓ, bound] exactly as
  // eval_loss_screen gives it for that W alone. false = not available here (the caller then
  // screens the tries one by one).
  virtual bool eval_loss_screen2(const double* w1, const double* w2, size_t nc, const double* mu, pc_density d,
                                 double* ll1, double* bound1, double* ll2, double* bound2) {
    (void)w1; (void)w2; (void)nc; (void)mu; (void)d; (void)ll1; (void)bound1; (void)ll2; (void)bound2;
    return false;
  }
  // Non-ortho line search: Σℓ and Σy² of Y_j = (W + α_j·Z)·(X−μ) for every α_j
  // in one pass (ll_out, y2_out: [na][nc]). false = not supported here.
  virtual bool eval_loss_multi(const double* w, const double* z, size_t nc, const double* mu, pc_density d,
                               const double* alphas, int na, double* ll_out, double* y2_out) {
    (void)w; (void)z; (void)nc; (void)mu; (void)d; (void)alphas; (void)na; (void)ll_out; (void)y2_out;
    return false;
  }
  // The same tries with a rigorous bound instead of exact sums (tanh, Σy² not needed):
  // |Σℓ_j,i − ll_out[j][i]| ≤ bnd_out[j][i] where Σℓ_j,i is what the exact pass at
  // W + α_j·Z gives. false = not available (the caller uses eval_loss_multi); must be
  // decided from rank-independent inputs only (every rank takes the same branch).
  virtual bool eval_loss_multi_bound(const double* w, const double* z, size_t nc, const double* mu, pc_density d,
                                     const double* alphas, int na, double* ll_out, double* bnd_out) {
    (void)w; (void)z; (void)nc; (void)mu; (void)d; (void)alphas; (void)na; (void)ll_out; (void)bnd_out;
    return false;
  }
  // expm(a) for an n × n a (math.rs:38-74) with the bits of the host's matrix_exp, formed where
  // the evaluator's passes run (try 1's map of an orthogonal search); false = not here (the
  // caller forms it on the host)
  virtual bool device_matrix_exp(const double* a, size_t n, double* out) {
    (void)a; (void)n; (void)out;
    return false;
  }
  // JADE sweeps (jade.rs:37-69) on the np = n(n+1)/2 cumulant matrices A, packed
  // position-major (A[pos(k,l)·np + m], k ≤ l, pos as in jade_warm_start). On
  // success v (n×n, row-major) holds the accumulated rotation V and *log the
  // sweeps run, whether the angle tolerance was met, and the max angle of
  // every 10th sweep (the verbose lines of jade.rs:57-66); false = not
  // supported here (the host runs them).
  virtual bool jade_sweeps(const double* A, size_t n, size_t max_iter, double tol, double* v, JadeSweepLog* log) {
    (void)A; (void)n; (void)max_iter; (void)tol; (void)v; (void)log;
    return false;
  }
  // The same sweeps on the cumulant matrices of the LAST moments4 call (Q_ij = M/t − δ-terms,
  // jade.rs:101-126, the values jade_warm_start builds on the host), formed where that call
  // left M; false = not available (the caller builds A and calls jade_sweeps).
  virtual bool jade_sweeps_moments(size_t n, double t, size_t max_iter, double tol, double* v, JadeSweepLog* log) {
    (void)n; (void)t; (void)max_iter; (void)tol; (void)v; (void)log;
    return false;
  }
  // eval_complete into a raw packed stats buffer (C ABI)
  virtual void eval_complete_into(pc_density d, bool need_h, double* stats) {
    (void)d; (void)need_h; (void)stats;
    throw computation_error("no kept evaluation to complete");
  }
};

}  // namespace pcamd
