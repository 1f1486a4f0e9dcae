// Host Picard driver: src/solver.rs:45-249 + src/core.rs:162-401 +
// src/lbfgs.rs:84-171 + src/jade.rs:22-197 restated over an Evaluator.
#pragma once
#include <cstdlib>
#include <deque>
#include <limits>
#include <memory>
#include <random>

#include "evaluator.hpp"
#include "host_linalg.hpp"

namespace pcamd {

std::string rust_e4(double v);  // Rust {:.4e}

// jade.rs:22-72 on Y = base·(X − μ) (n × T, base n × nf): the fourth-moment
// pass on the device, the cumulant matrices (jade.rs:78-131) and the Jacobi
// sweeps, then sym_decorrelation(V) (jade.rs:69). Sweep placement:
// AUTO = host; DEVICE = the cooperative device launch or an error; HOST; AUTO_DEVICE =
// the device launch where supported, the host otherwise. The solver uses AUTO_DEVICE,
// or AUTO when PICARD_HOST_JADE=1 is set.
enum JadeSweeps { JADE_SWEEPS_AUTO = 0, JADE_SWEEPS_DEVICE = 1, JADE_SWEEPS_HOST = 2, JADE_SWEEPS_AUTO_DEVICE = 3 };
struct JadeInfo { size_t sweeps = 0; bool converged = false; bool on_device = false; double moments_s = 0, sweeps_s = 0; };
size_t jade_max_pairs();  // PICARD_JADE_MAX_PAIRS test hook (SIZE_MAX when unset)
Mat jade_warm_start(Evaluator* ev, const Mat& base, size_t n, const double* mu, double T, size_t max_iter,
                    double tol, bool verbose, int where, JadeInfo* info);

// src/lbfgs.rs:6-71 (only the parts core::run uses)
struct LbfgsMemory {
  std::deque<Mat> s_list, y_list;
  std::deque<double> r_list;
  void clear() { s_list.clear(); y_list.clear(); r_list.clear(); }
  size_t len() const { return s_list.size(); }
};
Mat compute_direction(const Mat& g, const Mat& h, const std::vector<double>& h_off,
                      const LbfgsMemory& mem, bool ortho);          // lbfgs.rs:84-133
Mat solve_hessian_system(const Mat& h, const std::vector<double>& h_off, const Mat& g);  // 136-150
void regularize_hessian(Mat& h, const std::vector<double>& h_off, double lambda_min);   // 155-171

class TransformWorker;  // host_solver.cpp: line-search maps formed ahead on a helper thread

class Solver {
 public:
  Solver(Evaluator* ev, const pc_config& cfg);
  ~Solver();
  // one iteration of core.rs:211-391; returns true once finished
  bool step();
  void finish(pc_result* out);
  bool done() const { return done_; }
  double last_loss() const { return current_loss_; }
  double last_gnorm() const { return gradient_norm_; }
  uint64_t last_evals() const { return last_evals_; }
  // the last step(): [0] wall ms, [1] ms inside evaluator calls (device passes, their
  // all-reduces and waits), [2] host ms (the rest: N×N work), [3] ms waiting for the
  // line-search helper thread's maps
  void last_timing(double out[4]) const {
    for (int i = 0; i < 4; ++i) out[i] = last_timing_[i];
  }
  // setup phases, ms since the constructor started (cumulative): rowsum, Gram, eigh, w_init
  // and warm start, initial pass (0 for a phase that did not run)
  void setup_timing(double out[5]) const {
    for (int i = 0; i < 5; ++i) out[i] = setup_ms_[i];
  }
  uint64_t total_evals() const { return total_evals_; }
  uint64_t total_completions() const { return total_completions_; }
  uint64_t screen_passes() const { return screen_passes_; }
  uint64_t screen_rejects() const { return screen_rejects_; }

 private:
  std::unique_ptr<TransformWorker> ahead_;
  // sg / la: sign and log|det w| when the caller already has them (NaN: computed here)
  double loss_of(const EvalStats& s, const Mat& w, const std::vector<double>& signs, bool* singular,
                 double sg = std::numeric_limits<double>::quiet_NaN(), double la = 0.0);
  void evaluate(const Mat& w_core, EvalStats* out);
  bool evaluate_loss(const Mat& w_core, EvalStats* out);  // true: only Σℓ/Σy² filled, Y kept on device
  void complete(EvalStats* out);
  // screened_out: the last try was rejected by the screen alone (no exact stats for w)
  // det_sg / det_la: sign and log|det w| when the search already formed them (NaN: not formed)
  struct LsResult { bool success; Mat w; EvalStats stats; double loss; Mat step; bool partial; size_t tries; bool needs_full;
                    bool screened_out; double det_sg = std::numeric_limits<double>::quiet_NaN(), det_la = 0.0; };
  double device_share(double call_ms, double hook_ms) const;
  LsResult line_search(const Mat& direction, size_t tries, bool multi_first, bool first_loss_only,
                       bool full_first = false);
  void init_core();
  Mat ica_par(const Mat& w_init);
  Mat jade(size_t max_iter, double tol);

  Evaluator* ev_;
  pc_config cfg_;
  Mat wp_cache_, wp_cache_src_;  // W·P of the last full pass and its W (non-ortho)
  std::vector<double> w_init_user_;
  uint64_t nf_ = 0, T_ = 0;
  size_t nc_ = 0;
  bool extended_ = false;
  bool has_mu_ = false;
  std::vector<double> mu_;
  bool has_k_ = false;
  Mat K_;        // whitening (nc × nf)
  Mat w_init_;   // nc × nc
  Mat P_;        // w_init·K (nc × nf): maps X−μ to x1 (solver.rs:140)
  Mat gram_;     // Σ (x−μ)(x−μ)ᵀ when computed
  bool has_gram_ = false;
  // core::run state (core.rs:175-209)
  Mat W_;
  EvalStats S_;
  double current_loss_ = 0.0;
  std::vector<double> signs_, old_signs_;
  Mat C_;
  bool has_cov_ = false;
  LbfgsMemory mem_;
  bool has_g_old_ = false, has_prev_step_ = false;
  Mat g_old_, prev_step_;
  size_t iter_ = 0, n_iter_ = 0;
  double gradient_norm_ = 1.0;
  bool converged_ = false, done_ = false;
  uint64_t last_evals_ = 0, total_evals_ = 0;
  double last_timing_[4] = {0.0, 0.0, 0.0, 0.0};
  double setup_ms_[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  uint64_t total_completions_ = 0;
  uint64_t screen_passes_ = 0, screen_rejects_ = 0;  // line-search tries screened / rejected by the screen
  bool screen_ok_ = true;  // false once the evaluator declined a screen (then never asked again)
  bool screen_seen_ = false;  // a screen has run (the evaluator screens: tries need not all be exact)
  bool pairs_ok_ = true;      // false once the evaluator declined a paired screen
  uint64_t screen_pairs_ = 0;  // paired screens (two tries per pass)
  // Curvature rejection of orthogonal tries (Solver::set_curvature): C1 = P·Gram·Pᵀ/T, the
  // whitened covariance; per search a lower bound on L'(0), the floor −ls_curv_ of L'' along
  // expm(αD)·W, L''(0)'s lower bound ls_q_ with |L'''|-type slope ls_k3_, and the rounding
  // slack; ls_curv_ = 0 disables
  bool curv_ok_ = false;
  double gram_cond_ = 0.0;  // λmax/λmin of the Gram over the kept components (whitening)
  Mat C1_;
  double ls_slope_ = 0.0, ls_curv_ = 0.0, ls_q_ = 0.0, ls_k3_ = 0.0, ls_slack_ = 0.0;
  uint64_t curv_skips_ = 0;
  // Convexity rejection of non-orthogonal tanh tries (Solver::convexity_trim): the trailing
  // tries of a search whose lower bound exceeds the losses' rounding run no pass
  // (PICARD_CVX=0 turns it off); cvx_skips_ counts them
  bool cvx_on_ = true;
  uint64_t cvx_skips_ = 0;
  size_t convexity_trim(const Mat& d, size_t tries, double* b_first) const;
  // non-orthogonal searches: tries in the first multi-try pass (0: all; PICARD_MULTI_GROUP)
  // and how many searches needed a second pass for the rest
  size_t multi_group_ = 0;
  uint64_t multi_second_passes_ = 0;
  void set_curvature(const Mat& g, const Mat& gs, const Mat& d, double slope);
  double curvature_lower_bound(double alpha) const;
  // first-try policy: outcomes of descent-direction first tries
  // by cell: 2·(Picard's quadratic model predicts a decrease at α = 1) + (previous search accepted
  // at try 1); first_cell_ is this iteration's (set in step)
  double first_n_[4] = {0.0, 0.0, 0.0, 0.0}, first_acc_[4] = {0.0, 0.0, 0.0, 0.0};
  int first_cell_ = 0;
  // the model along this iteration's D (slope, qh) and the later-try cell's counts
  double pred_slope_ = 0.0, pred_qh_ = 0.0, later_n_ = 0.0, later_acc_ = 0.0;
  // pair the screens of an overshooting descent search (line_search; PICARD_DESCENT_PAIR=0: off)
  const bool descent_pair_ = [] {
    const char* e = std::getenv("PICARD_DESCENT_PAIR");
    return !(e && std::atoi(e) == 0);
  }();
  // the pair's second try lies at ≥ factor·|slope|/qh (PICARD_DESCENT_PAIR_FACTOR; 4 = 2·α₀:
  // C3 screens 20.6 → 20.3 ms per step against 8, profiles/r06_final/ab_descent_pair_factor.log)
  const double descent_pair_factor_ = [] {
    const char* e = std::getenv("PICARD_DESCENT_PAIR_FACTOR");
    const double f = e ? std::atof(e) : 4.0;
    return f >= 2.0 ? f : 4.0;
  }();
  // Evaluation schedule of a line search (results are bit-identical whatever
  // the schedule): try 1 is a full fused pass (accepted ≈ 80 % of the time on
  // the bench data, and then its G is the next gradient); tries ≥ 2 are
  // loss-only passes (about 0.6 of a fused pass) and only the accepted one is
  // completed, by recomputing it in full. Knobs for experiments:
  //   PICARD_KEEP_Y=1      loss-only tries keep Y in HBM (completion ≈ 0.5 pass,
  //                        each try pays the Y write ≈ 0.1 pass)
  //   PICARD_SPLIT_FIRST=1 try 1 is loss-only too unless the last line search
  //                        accepted at try 1
  bool first_full_ = true;
  bool keep_y_ = false, split_first_ = false;
  // Non-ortho searches evaluate tries >= 2 in one multi-α pass
  // (Evaluator::eval_loss_multi) unless PICARD_NO_MULTI=1.
  bool no_multi_ = false;
  // the bounded (fp32) multi-try pass is used until a search pays a full pass for a try the exact
  // pass then rejects (near convergence the tries differ by less than its bound): from then on
  // the exact multi-try pass. Decided from reduced statistics only: the same on every rank.
  bool multi_bound_on_ = true;
  // PICARD_TRACE timing: evaluator calls, try-1 map, waits for the helper's maps
  double eval_ms_ = 0.0, map1_ms_ = 0.0, ahead_wait_ms_ = 0.0;
  bool trace_ = false;  // PICARD_TRACE=1: one stderr line per iteration (line-search tries)
};

}  // namespace pcamd
