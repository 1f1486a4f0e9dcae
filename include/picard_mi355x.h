/*
 * picard_mi355x.h — C ABI of the MI355X-native Picard / Picard-O ICA solver.
 *
 * This is the drop-in boundary for the hot path of lmmx/picard-ica v0.1.6.
 * The reference is a Rust crate; its public API and the operator calls inside
 * core::run are what these entry points replace (file:line in the reference):
 *
 *   pc_fit / pc_fit_default   ← Picard::fit_with_config / Picard::fit   (src/solver.rs:45 / :33)
 *   pc_transform              ← Picard::transform                      (src/solver.rs:199)
 *   pc_full_unmixing          ← PicardResult::full_unmixing            (src/result.rs:39)
 *   pc_mixing                 ← PicardResult::mixing                   (src/result.rs:49)
 *   pc_amari_distance         ← utils::amari_distance                  (src/utils.rs:82)
 *   pc_permute                ← utils::permute                         (src/utils.rs:16)
 *   pc_config_default         ← impl Default for PicardConfig          (src/config.rs:64-85)
 *   pc_config_validate        ← PicardConfig::validate                 (src/config.rs:104-142)
 *   pc_result_free            ← Drop for PicardResult                  (src/result.rs:7)
 *   pc_error_name             ← PicardError variant names              (src/error.rs:9-42)
 *
 * The operator boundary inside core::run (src/core.rs:162-174), i.e. what
 * the HIP kernels replace (score_and_der core.rs:215, the .dot GEMMs
 * core.rs:124/218/274, compute_loss core.rs:39-85, center/whiten
 * whitening.rs:24-116):
 *
 *   pc_ctx_eval               one fused pass over X: Y = W·(X−μ) → ψ, ψ′, ℓ →
 *                             G_raw = ψ·Yᵀ [, H_raw = ψ′·(Y∘Y)ᵀ], Σψ′, Σℓ, Σy²
 *   pc_ctx_rowsum / pc_ctx_gram   centering and the whitening Gram X·Xᵀ
 *   pc_ctx_sources            Y = W·(X−μ) materialised (PicardResult.sources)
 *   pc_ctx_sources_device     the same Y kept in HBM (device pointer, one MFMA pass)
 *   pc_ctx_moments4 / pc_ctx_jade   the JADE warm start (src/jade.rs:22-197)
 *
 * Conventions: every matrix is row-major, contiguous, float64. Rows are
 * features/components, columns are samples (src/solver.rs:29,40). Inputs
 * are borrowed read-only; result buffers are owned by the library and
 * released by pc_result_free. Calls are synchronous. A context is driven by
 * one host thread. Errors are returned as pc_status codes with the message
 * text of src/error.rs:44-74 written into (err, errlen) when err != NULL.
 */
#ifndef PICARD_MI355X_H
#define PICARD_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI revision of this header. 2: pc_host_evaluator grew the eval_loss_multi and
 * eval_loss_screen slots (a caller built against revision 1 must be rebuilt), the
 * rank-group entry points (pc_group_*, pc_ctx_create_in_group, pc_ctx_comm_stats,
 * pc_ctx_abort) and pc_ctx_release_caches were added. 3: pc_ctx_eval_loss_multi_bound
 * was added (no layout change). 4: PC_ERR_UNSUPPORTED for capability misses of the
 * operator boundary (they no longer abort a rank group). 5: pc_ctx_comm_timing,
 * pc_solver_timing, pc_solver_setup_timing, pc_ctx_alloc_stats, pc_last_teardown,
 * pc_device_mem_info. 6: pc_ctx_eval_loss_screen2 (paired screen), pc_ctx_screen_tries.
 * 7: pc_ctx_matrix_exp, pc_matrix_exp (no layout change). 8: pc_ctx_screen_digit_gram,
 * pc_ctx_screen_products (no layout change).
 * pc_abi_version() returns the revision the library was built with. */
#define PC_ABI_VERSION 8

/* src/error.rs:9-42 (NotConverged is reserved: the reference never returns it) */
typedef enum {
  PC_OK = 0,
  PC_ERR_INVALID_DIMENSIONS = 1,
  PC_ERR_SINGULAR_MATRIX = 2,
  PC_ERR_COMPUTATION = 3,
  PC_ERR_INVALID_CONFIG = 4,
  PC_ERR_NOT_CONVERGED = 5,
  /* operator boundary only (never returned by pc_fit): the requested pass or placement is
   * not available for this context / shape / density. Nothing ran and a rank group is NOT
   * aborted — the documented fallback (pc_ctx_eval_loss_multi, an exact try, host JADE
   * sweeps) can be called next on every rank. */
  PC_ERR_UNSUPPORTED = 6
} pc_status;

/* src/density.rs:137-144 DensityType */
typedef enum { PC_DENSITY_TANH = 0, PC_DENSITY_EXP = 1, PC_DENSITY_CUBE = 2 } pc_density_kind;

typedef struct {
  int32_t kind;   /* pc_density_kind */
  double alpha;   /* Tanh/Exp alpha (density.rs:34,75); ignored for Cube */
} pc_density;

/* src/config.rs:11-62 — the 16 fields; Option<T> → has_* flag + value */
typedef struct {
  pc_density density;
  int32_t has_n_components; uint64_t n_components;
  int32_t ortho;
  int32_t has_extended; int32_t extended;
  int32_t whiten;
  int32_t centering;
  uint64_t max_iter;
  double tol;
  uint64_t m;
  uint64_t ls_tries;
  double lambda_min;
  const double* w_init; uint64_t w_init_rows; uint64_t w_init_cols; /* NULL = None */
  int32_t has_fastica_it; uint64_t fastica_it;
  int32_t has_jade_it; uint64_t jade_it;
  int32_t has_random_state; uint64_t random_state;
  int32_t verbose;
  /* MI355X additions (not in the reference): */
  int32_t device;          /* HIP device ordinal for pc_fit (default 0) */
  int32_t want_sources;    /* materialise PicardResult.sources (default 1) */
} pc_config;

/* src/result.rs:7-33 — buffers are library-owned, NULL for None */
typedef struct {
  double* whitening; uint64_t whitening_rows, whitening_cols; /* K: n_components × n_features */
  double* unmixing;  uint64_t unmixing_rows,  unmixing_cols;  /* W: n_components × n_components */
  double* sources;   uint64_t sources_rows,   sources_cols;   /* Y: n_components × n_samples */
  double* mean;      uint64_t mean_len;                       /* μ: n_features */
  uint64_t n_iterations;
  int32_t converged;
  double gradient_norm;
  double* signs;     uint64_t signs_len;                      /* extended only */
  /* MI355X additions: work counters for the iterations-to-tol metric */
  uint64_t n_evaluations;  /* fused passes over X issued by core::run */
} pc_result;

/* ---- public API (mirrors src/lib.rs:50-57) --------------------------- */
void pc_config_default(pc_config* cfg);
int pc_config_validate(const pc_config* cfg, char* err, size_t errlen);

int pc_fit(const double* x, uint64_t n_features, uint64_t n_samples, const pc_config* cfg,
           pc_result* out, char* err, size_t errlen);
int pc_fit_default(const double* x, uint64_t n_features, uint64_t n_samples, pc_result* out,
                   char* err, size_t errlen);
int pc_transform(const double* x, uint64_t n_features, uint64_t n_samples, const pc_result* res,
                 double* out /* n_components × n_samples */, int32_t device, char* err, size_t errlen);
int pc_full_unmixing(const pc_result* res, double* out /* n_components × n_features */);
int pc_mixing(const pc_result* res, double* out /* n_features × n_components */);
void pc_result_free(pc_result* res);
double pc_amari_distance(const double* w, const double* a, uint64_t n);
void pc_permute(const double* a, uint64_t n, int32_t scale, double* out);
const char* pc_error_name(int status);
const char* pc_version(void);
int pc_abi_version(void);

/* ---- device context: X resident in HBM, optionally T-sharded over ranks --- */
typedef struct pc_ctx pc_ctx;

/* RCCL bootstrap for one-process-per-GPU runs: rank 0 calls pc_rccl_unique_id,
 * the 128-byte id is broadcast by the caller (e.g. torch.distributed), every
 * rank then creates its context with it. world_size == 1 needs no id; given one,
 * the context is a one-rank RCCL communicator (the RCCL code path on one GPU). */
int pc_rccl_unique_id(char id_out[128]);

/* Each rank owns the samples [t0, t0 + n_local) of a global matrix with
 * n_total samples (contiguous T blocks). With world_size > 1 and
 * rccl_id == NULL the context is a DETACHED shard: no communicator is created,
 * every pc_ctx_* statistic is this shard's partial sum (per-sample constants
 * included, counted over its own n_local samples) and the caller adds the
 * shards up — e.g. one process driving several shards through
 * pc_fit_with_evaluator. pc_solver_create refuses a detached shard
 * (PC_ERR_INVALID_CONFIG). */
int pc_ctx_create(int32_t device, int32_t rank, int32_t world_size, const char* rccl_id /* or NULL */,
                  pc_ctx** out, char* err, size_t errlen);
void pc_ctx_destroy(pc_ctx* ctx);

/* In-process rank group: world_size contexts in ONE process, each driven by its own host
 * thread (they may share one GPU), exchange every pass's statistics through host memory —
 * a fixed rank-order sum, identical bits on every rank — instead of RCCL. It runs the
 * communicator code path of the one-process-per-GPU run (rank-replicated solvers, the
 * per-pass all-reduce, the capability agreements) on a single device. Every all-reduce
 * also checks that all ranks issued the same collective (call site and length) and
 * fails the group if they diverged. The group is reference-counted: destroying it while
 * contexts still use it is allowed. */
typedef struct pc_group pc_group;
int pc_group_create_local(int32_t world_size, pc_group** out, char* err, size_t errlen);
void pc_group_destroy(pc_group* g);
int pc_ctx_create_in_group(int32_t device, int32_t rank, pc_group* g, pc_ctx** out, char* err, size_t errlen);
/* Communicator state of a context: [0] all-reduces issued, [1] capability agreements
 * asked (int8 digit image / kept Y, DeviceCtx::agree_once), [2] the screen agreement,
 * [3] the kept-Y agreement (0 not asked, 1 every rank has it, -1 not every rank),
 * [4] 1 once the group was aborted, [5] world size, [6] 1 RCCL, 2 in-process group,
 * 0 none. */
void pc_ctx_comm_stats(const pc_ctx* ctx, int64_t out[7]);
/* Time inside the context's all-reduces since it was created: out[0] ms (RCCL: device time
 * between HIP events around each ncclAllReduce, which includes waiting for the slowest rank;
 * in-process group: host time of the exchange), out[1] the number of all-reduces timed. */
void pc_ctx_comm_timing(const pc_ctx* ctx, double out[2]);
/* HBM allocation calls of the context so far: out[0..2] ms spent in hipMalloc / hipFree /
 * hipMemGetInfo, out[3..5] their counts, out[6..8] the longest single call of each. */
void pc_ctx_alloc_stats(const pc_ctx* ctx, double out[9]);
/* The last context teardown in this process (pc_ctx_destroy): out[0] wall ms, [1] ms in its
 * hipFree calls, [2] the longest single hipFree of that context's life, [3] ms of the closing
 * hipDeviceSynchronize (deferred work of the frees is charged to the teardown). */
void pc_last_teardown(double out[4]);
/* Abort the context's rank group: every rank's pending and later collectives (RCCL:
 * through ncclCommAbort and a shared abort word the peers poll while they wait) end
 * with PC_ERR_COMPUTATION. Any pc_ctx_* / pc_solver_* call that fails with
 * PC_ERR_COMPUTATION on a rank of a group does this itself, so an error one rank alone
 * sees (HIP, HBM, a lost capability) ends every rank instead of leaving it waiting in a
 * collective. A peer process that exits, or a collective that does not complete within
 * PICARD_COMM_TIMEOUT_S seconds (default 600), aborts the group too. */
void pc_ctx_abort(pc_ctx* ctx, const char* why);
/* Free the context's HBM caches (the int8 digit image of X, the kept-Y buffer of split
 * evaluation, the second y-fragment buffer of the multi-try pass; the first y-fragment
 * slot, inside the tiled pass's buffer, is invalidated); later passes run without them
 * (the fp64 Y stage, completion and multi-try Y by recomputation). On a rank
 * whose group agreed to use the digit image this makes its next screened try fail —
 * and abort the group — rather than let the ranks diverge. */
int pc_ctx_release_caches(pc_ctx* ctx, char* err, size_t errlen);
/* copy a host shard (n_features × n_local, row-major) into HBM */
int pc_ctx_load(pc_ctx* ctx, const double* x_shard, uint64_t n_features, uint64_t n_local,
                uint64_t n_total, uint64_t t0, char* err, size_t errlen);
/* generate the benches/benchmarks.rs:8-35 mixture directly in HBM: this rank's
 * contiguous shard of the global (n_features × n_total) X for `seed`; the
 * mixing matrix A (n_features²) is written to a_out when not NULL */
int pc_ctx_generate(pc_ctx* ctx, uint64_t n_features, uint64_t n_total, uint64_t seed,
                    double* a_out, char* err, size_t errlen);
/* copy this rank's shard back to the host (n_features × n_local). The passes
 * centre X in place (the first call with a mean μ subtracts it from the
 * resident shard; a call with another μ, or download, adds it back), so after
 * a fit with centering the downloaded data equal the loaded data only up to
 * rounding: (x − μ) + μ may differ from x in the last bit. */
int pc_ctx_download(pc_ctx* ctx, double* x_shard_out);
uint64_t pc_ctx_n_local(const pc_ctx* ctx);
uint64_t pc_ctx_t0(const pc_ctx* ctx);

/* Operator boundary. All statistics are summed over every rank's shard
 * (one RCCL all-reduce per call when world_size > 1). */
enum { PC_EVAL_NEED_H = 1u, PC_EVAL_SKIP_Y2 = 2u };
/* stats = [G_raw (nc×nc) | H_raw (nc×nc, only with PC_EVAL_NEED_H) | Σψ′ (nc) | Σℓ (nc) | Σy² (nc)].
 * PC_EVAL_SKIP_Y2 (ignored with NEED_H): Σy² is not accumulated and reads 0 —
 * the orthogonal solver never uses it (core.rs:221 computes Y∘Y, read only at
 * :274 and by the extended non-orthogonal loss), saving one fp64 op per element. */
int pc_ctx_eval(pc_ctx* ctx, const double* w /* nc × n_features */, uint64_t nc,
                const double* mu /* n_features or NULL */, pc_density density, uint32_t flags,
                double* stats, char* err, size_t errlen);
/* Split form of pc_ctx_eval for line-search tries (core.rs:117-140 only needs
 * Σℓ and Σy² to accept or reject a try). pc_ctx_eval_loss fills the Σℓ, Σy²
 * entries of `stats` (same layout as pc_ctx_eval) from a pass that skips the
 * ψ·Yᵀ contraction and keeps Y in HBM; *kept = 1 then, and
 * pc_ctx_eval_complete fills the remaining entries (G_raw, H_raw, Σψ′) for the
 * same W from the kept Y. *kept = 0 means the pass was a full pc_ctx_eval
 * (shape not covered or HBM too short to keep Y). Sums are bit-identical to
 * pc_ctx_eval's. */
int pc_ctx_eval_loss(pc_ctx* ctx, const double* w, uint64_t nc, const double* mu, pc_density density,
                     uint32_t flags, double* stats, int32_t* kept, char* err, size_t errlen);
/* Non-orthogonal line search in one pass (core.rs:117-140 with the try
 * transform M = I + α·D, solver.rs's non-ortho branch): with w = W·P and
 * z = (D·W)·P (both nc × n_features), writes Σℓ and Σy² of
 * Y_j = (w + α_j·z)·(X − μ) for every α_j: ll_out[j·nc + i], y2_out[j·nc + i].
 * Equal to pc_ctx_eval_loss at w + α_j·z up to rounding (Y_j is formed as
 * Y + α_j·Z). Returns PC_ERR_UNSUPPORTED for a shape the pass does not cover
 * (nc > 256, or a negative tanh/exp α). */
int pc_ctx_eval_loss_multi(pc_ctx* ctx, const double* w, const double* z, uint64_t nc, const double* mu,
                           pc_density density, const double* alphas, uint64_t n_alpha, double* ll_out,
                           double* y2_out, char* err, size_t errlen);
/* The same tries with their row terms in fp32 and a rigorous bound instead of exact sums
 * (tanh, the int8 stage at n_features ≤ 256; the non-orthogonal line search of a
 * non-extended fit, whose loss needs no Σy²): |Σℓ_j,i − ll_out[j·nc + i]| ≤ bnd_out[j·nc + i]
 * where Σℓ_j,i is what pc_ctx_eval_loss gives at w + α_j·z. n_alpha ≤ 12. Opt-in:
 * PICARD_MULTI_F32=1 (the solver then uses it until a search pays a full pass for a try the exact
 * pass rejects). Returns PC_ERR_UNSUPPORTED where it does not apply or is not
 * enabled (the caller then uses pc_ctx_eval_loss_multi). */
int pc_ctx_eval_loss_multi_bound(pc_ctx* ctx, const double* w, const double* z, uint64_t nc, const double* mu,
                                 pc_density density, const double* alphas, uint64_t n_alpha, double* ll_out,
                                 double* bnd_out, char* err, size_t errlen);
int pc_ctx_eval_complete(pc_ctx* ctx, pc_density density, uint32_t flags, double* stats, char* err,
                         size_t errlen);
int pc_ctx_rowsum(pc_ctx* ctx, double* out /* n_features */, char* err, size_t errlen);
int pc_ctx_gram(pc_ctx* ctx, const double* mu /* or NULL */, double* out /* nf × nf */,
                char* err, size_t errlen);
/* this rank's shard of Y = W·(X−μ) → host (nc × n_local). When the context already holds
 * the int8 digit image of X at this μ (built by an earlier pass; PC_YSTAGE_F64 not set) and
 * 64 < nc ≤ 128, nf ≤ 128, Y comes from the exact int8 digit products (fp64-GEMM accuracy,
 * not the fp64 MFMA store's bits); pc_ctx_sources and pc_ctx_sources_device always agree
 * bit for bit. No image is built for a sources call alone. */
int pc_ctx_sources(pc_ctx* ctx, const double* w, uint64_t nc, const double* mu, double* out,
                   char* err, size_t errlen);
/* The same Y kept in HBM for device-side consumers (solver.rs:182,199-214
 * without the host round trip): the whole shard in one MFMA pass, nc rows of
 * *ld_out doubles (row-major; columns past n_local are zero). *dev_out is a
 * device pointer owned by the context, valid until the next
 * pc_ctx_sources_device or pc_ctx_destroy; *kernel_ms = the pass's device time.
 * Any out pointer may be NULL. */
int pc_ctx_sources_device(pc_ctx* ctx, const double* w, uint64_t nc, const double* mu, const double** dev_out,
                          uint64_t* ld_out, double* kernel_ms, char* err, size_t errlen);
/* Σ_t z_p z_q over the pair products z_(i,j) = y_i y_j (i ≤ j) of Y = W·(X−μ):
 * the fourth-moment matrix JADE's cumulants are built from (src/jade.rs:91-113).
 * out: P × P with P = nc(nc+1)/2, pairs in row-major (i ≤ j) order. */
int pc_ctx_moments4(pc_ctx* ctx, const double* w, uint64_t nc, const double* mu, double* out,
                    char* err, size_t errlen);

/* The JADE warm start (src/jade.rs:22-72, caller solver.rs:124-128) on
 * Y = W·(X−μ) (W: nc × n_features, normally the whitening K): the fourth-moment
 * pass on the device (pc_ctx_moments4), the nc(nc+1)/2 cumulant matrices
 * (jade.rs:78-131), up to max_iter Jacobi sweeps in the reference's cyclic
 * (p, q) order (jade.rs:37-69) with the angle tolerance tol, and
 * w_out = sym_decorrelation(V) (nc × nc, jade.rs:69). `where` places the
 * sweeps: PC_JADE_AUTO (host), PC_JADE_DEVICE (one device launch;
 * PC_ERR_UNSUPPORTED if the shape does not fit it) or PC_JADE_HOST.
 * sweeps_out (or NULL): [0] sweeps run, [1] 1 if the tolerance was met,
 * [2] 1 if the sweeps ran on the device. */
enum { PC_JADE_AUTO = 0, PC_JADE_DEVICE = 1, PC_JADE_HOST = 2 };
int pc_ctx_jade(pc_ctx* ctx, const double* w, uint64_t nc, const double* mu, uint64_t max_iter, double tol,
                int32_t where, double* w_out, uint64_t sweeps_out[3], char* err, size_t errlen);

/* Stepping solver over a context: pc_fit's pipeline (solver.rs:45-189) split
 * so that a caller can time individual Picard iterations (core.rs:211-391).
 * pc_solver_step runs ONE iteration; *done becomes 1 on convergence or when
 * max_iter iterations have run. pc_solver_finish fills the result (sources
 * only when cfg->want_sources, and then only this rank's shard). */
typedef struct pc_solver pc_solver;
int pc_solver_create(pc_ctx* ctx, const pc_config* cfg, pc_solver** out, char* err, size_t errlen);
int pc_solver_step(pc_solver* s, int32_t* done, char* err, size_t errlen);
int pc_solver_finish(pc_solver* s, pc_result* out, char* err, size_t errlen);
void pc_solver_destroy(pc_solver* s);
/* last iteration's: loss, gradient norm, passes issued in that iteration */
void pc_solver_last(const pc_solver* s, double* loss, double* gradient_norm, uint64_t* n_evals);
/* last iteration's timing: out[0] wall ms, [1] ms inside pass calls (device work, all-reduces,
 * waits), [2] host ms (the rest: the N×N work of core.rs), [3] ms waiting for the line-search
 * helper thread */
void pc_solver_timing(const pc_solver* s, double out[4]);
/* the solver's setup phases, ms since pc_solver_create started (cumulative): out[0] row sums,
 * [1] Gram, [2] eigh, [3] w_init + warm start, [4] the initial pass */
void pc_solver_setup_timing(const pc_solver* s, double out[5]);

/* Host-driver hook: run the same solver pipeline over caller-supplied
 * evaluation callbacks instead of the HIP context. Used by the CPU test suite
 * to check the host logic (core::run, L-BFGS, line search, whitening) without
 * a GPU; the product path never uses it. */
typedef struct {
  void* user;
  uint64_t n_features, n_samples;
  int (*rowsum)(void* user, double* out);
  int (*gram)(void* user, const double* mu, double* out);
  int (*eval)(void* user, const double* w, uint64_t nc, const double* mu, pc_density density,
              uint32_t flags, double* stats);
  int (*sources)(void* user, const double* w, uint64_t nc, const double* mu, double* out);
  int (*moments4)(void* user, const double* w, uint64_t nc, const double* mu, double* out);
  /* optional (NULL: every non-orthogonal line-search try is a full eval):
   * pc_ctx_eval_loss_multi's contract */
  int (*eval_loss_multi)(void* user, const double* w, const double* z, uint64_t nc, const double* mu,
                         pc_density density, const double* alphas, uint64_t n_alpha, double* ll_out,
                         double* y2_out);
  /* optional (NULL: no line-search screen): pc_ctx_eval_loss_screen's contract —
   * Σℓ of an approximation and per-row bounds on its distance to the exact Σℓ */
  int (*eval_loss_screen)(void* user, const double* w, uint64_t nc, const double* mu, pc_density density,
                          double* ll_out, double* bound_out);
} pc_host_evaluator;
int pc_fit_with_evaluator(const pc_host_evaluator* ev, const pc_config* cfg, pc_result* out,
                          char* err, size_t errlen);

/* Timing of the most recent pc_ctx_eval on the context's stream, measured
 * with HIP events around the fused-pass kernel and the whole call. */
void pc_ctx_last_timing(const pc_ctx* ctx, double* kernel_ms, double* call_ms);
/* Accumulated over every fused pass since the last reset: total kernel time,
 * total pc_ctx_eval wall time (upload + kernel + reduce + all-reduce + D2H)
 * and the number of fused-kernel launches. */
void pc_ctx_kernel_stats(pc_ctx* ctx, double* kernel_ms, double* call_ms, uint64_t* n_launches,
                         int32_t reset);
/* Per kernel kind since the last reset: [0] fused pass, [1] loss-only try,
 * [2] completion from kept Y — summed HIP-event kernel ms and launch counts. */
void pc_ctx_kernel_breakdown(pc_ctx* ctx, double ms[4], uint64_t n[4], int32_t reset);
/* Y-stage arithmetic of the passes (Y = W·(X−μ), core.rs:124). PC_YSTAGE_AUTO
 * (default): where the shape allows (64 < nc ≤ 128, n_features ≤ 128) the
 * loss-only line-search pass forms Y on the i8 matrix cores from exact int8
 * digits of X (7 radix-256 digits per value, one exponent per sample, built
 * once per resident mean) and of W (7 per value, one exponent per row): every
 * digit product is summed exactly in int32 and the 7 leading diagonals are
 * combined in fp64, so Y carries the accuracy of an fp64 GEMM (DESIGN.md §3,
 * the Ozaki scheme); the digit image costs another 7 bytes per element of HBM. PC_YSTAGE_F64: every pass on the
 * fp64 MFMA Y stage. Either way the statistics agree with the fp64 oracle to
 * 1e-12 relative; they are bit-identical only within one mode.
 * Under PC_YSTAGE_AUTO the orthogonal solver also SCREENS its loss-only
 * line-search tries: a pass on the 4 leading digit diagonals (10 digit products)
 * plus a rigorous bound on the exact Σℓ rejects a try when no exact value could
 * accept it (core.rs:127-140 decides the same way); every other try runs the
 * exact pass. PC_YSTAGE_INT8_EXACT: the int8 stage without the screen (every
 * try exact) — the fits are bit-identical to AUTO's. */
enum { PC_YSTAGE_AUTO = 0, PC_YSTAGE_F64 = 1, PC_YSTAGE_INT8_EXACT = 2 };
int pc_ctx_set_y_stage(pc_ctx* ctx, int32_t mode);
/* number of passes whose Y stage ran on the int8 slices since the context was created */
uint64_t pc_ctx_int8_passes(const pc_ctx* ctx);
/* G-stage arithmetic of the orthogonal fused pass (G = ψ(Y)·Yᵀ, core.rs:218). PC_GSTAGE_AUTO
 * (default):
 * where the fused pass runs on the int8 digit Y stage (64 < nc ≤ 128, nf ≤ 128, tanh or exp),
 * ψ and y are also split into 6 signed radix-256 digits each at one fixed scale per row and
 * pass, and G is summed exactly in int32 per 64-sample chunk on the i8 matrix cores (the 21
 * leading digit products for tanh, 26 for exp), then in fp64 (G within 1e-13 of the fp64 stage at
 * T ≥ 2^20, 1e-12 at T ≈ 5e3). PC_GSTAGE_F64: G on the fp64 MFMA. Row sums (Σψ′, Σℓ, Σy²)
 * are bit-identical in both modes. (PICARD_G8=0 in the environment selects PC_GSTAGE_F64 for
 * new contexts.) */
enum { PC_GSTAGE_AUTO = 0, PC_GSTAGE_F64 = 1 };
int pc_ctx_set_g_stage(pc_ctx* ctx, int32_t mode);
/* number of fused passes whose G stage ran on int8 digits since the context was created */
uint64_t pc_ctx_g8_passes(const pc_ctx* ctx);
/* number of non-ortho multi-try passes (pc_ctx_eval_loss_multi, core.rs:117-141) that read Y
 * from the tiled full pass at the same W instead of forming it (the same bits: both come from
 * the same int8 digit products; PICARD_MULTI_YBUF=0 in the environment turns this off for new
 * contexts) */
uint64_t pc_ctx_multi_ybuf_passes(const pc_ctx* ctx);
/* expm(a) of an n × n row-major a (math.rs:38-74 matrix_exp, the map W ← expm(α·D)·W of an
 * orthogonal line-search try, core.rs:118-125) as the solver forms try 1's map: on the device
 * (k_expm_ps) with the bits of pc_matrix_exp. Returns PC_ERR_UNSUPPORTED where the device leaves
 * it to the host (n not a multiple of 32 in [32, 128], a series the reference caps at 30 terms,
 * more than 48 squarings, PICARD_DEVICE_EXPM=0). pc_matrix_exp: the host's matrix_exp. */
int pc_ctx_matrix_exp(pc_ctx* ctx, const double* a, uint64_t n, double* out, char* err, size_t errlen);
void pc_matrix_exp(const double* a, uint64_t n, double* out);
/* The line-search screen itself: ll_out[i] = Σℓ of row i from the 4 leading digit
 * diagonals, bound_out[i] ≥ |Σℓ_exact − ll_out[i]| (rounding included), both summed
 * over ranks. Returns PC_ERR_UNSUPPORTED when the context has no screen for this
 * shape / density (int8 stage off, nc outside (32, 128], n_features above 64 for
 * nc ≤ 64 or above 128, cube, α ≤ 0). */
int pc_ctx_eval_loss_screen(pc_ctx* ctx, const double* w, uint64_t nc, const double* mu, pc_density density,
                            double* ll_out, double* bound_out, char* err, size_t errlen);
/* Two tries' screens in ONE pass (w1, w2: nc × n_features each): ll1/bound1 and ll2/bound2 are
 * what pc_ctx_eval_loss_screen returns for w1 and for w2 alone (the same arithmetic per W; the
 * solver pairs the screened tries of a non-descent search with it). tanh, the
 * fp32 screen at D ≤ 2 or 3 only; PC_ERR_UNSUPPORTED where it does not apply (or with
 * PICARD_SCREEN_PAIRS=0). With a communicator, collective like pc_ctx_eval. */
int pc_ctx_eval_loss_screen2(pc_ctx* ctx, const double* w1, const double* w2, uint64_t nc, const double* mu,
                             pc_density density, double* ll1, double* bound1, double* ll2, double* bound2,
                             char* err, size_t errlen);
/* line-search screen passes since the last reset: summed HIP-event kernel ms and count */
void pc_ctx_screen_stats(pc_ctx* ctx, double* kernel_ms, uint64_t* n_launches, int32_t reset);
/* tries those passes covered since the same reset (a paired pass covers 2) */
uint64_t pc_ctx_screen_tries(const pc_ctx* ctx);
/* digit products those tries kept since the same reset, summed per try: (D+1)(D+2)/2 for a
 * screen on diagonals D (6 for D ≤ 2, 10 for D ≤ 3, 15 for D ≤ 4) */
uint64_t pc_ctx_screen_products(const pc_ctx* ctx);
/* Inputs of the line-search screen's statistical bound for this context's shard (built on
 * first use, with the int8 digit image): lam[b] (b < 7) ≥ the largest eigenvalue of the digit
 * Gram D_b = Σ_t d_b,t·d_b,tᵀ (Gershgorin on the exact integer matrix), *s4 = Σ_t 4^(e_t) over
 * the sample exponents (padding included). The screen's per-row tail is then
 * 2^(f_i−12)·Σ_{dmax < a+b ≤ 6} 2^(−8(a+b))·√(s4·lam[b]·Σ_k w_a,ik²), or the worst-case tail
 * where that is smaller. PC_ERR_UNSUPPORTED without an int8 digit image. */
int pc_ctx_screen_digit_gram(pc_ctx* ctx, double* lam, double* s4, char* err, size_t errlen);
/* Exhaustive accuracy of the fp32 instructions the line-search screen evaluates its
 * log-likelihood with (v_exp_f32, v_log_f32), measured on `device` against fp64 libm
 * over every fp32 input of the ranges the screen uses: out[0] max relative error of 2^z
 * on [−126, 0], out[1] max absolute error of 2^z on [−150, −126), out[2] max absolute
 * error of log2 p on [2^-4, 1], out[3] 1 if 2^0 = 1 and log2 1 = 0 exactly. The screen's
 * bound is built from constants these must not exceed. */
int pc_device_check_fp32_transcendentals(int32_t device, double out[4]);
/* hipDeviceSynchronize on `device` (bench bracketing). */
int pc_device_synchronize(int32_t device);
/* hipMemGetInfo of `device`: free and total HBM bytes (either pointer may be NULL) */
int pc_device_mem_info(int32_t device, uint64_t* free_bytes, uint64_t* total_bytes);

#ifdef __cplusplus
}
#endif
#endif /* PICARD_MI355X_H */
