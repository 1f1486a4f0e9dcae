"""CPU ORACLE — test infrastructure only, never the product path.

A statement-for-statement numpy (float64) restatement of the Rust reference
lmmx/picard-ica v0.1.6 (mounted read-only at /root/reference during the
build; it is NOT present on the GPU box and nothing here reads it).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker / the
timed CPU baseline. The product (``picard-ica_amd/``) never calls it and fails
loudly when its HIP library is missing.

Parity pinning:
  * The reference is a Rust crate; no rustc/cargo exists in this image, so it
    cannot be compiled or run here. The reference ships no golden vectors.
  * PINNED against the reference's own known-answer unit tests, restated in
    ``tests/test_oracle_kats.py``: math.rs:101-152 (sym_decorrelation,
    matrix_exp(0), sln_det KATs, skew), whitening.rs:124-150 (center KAT,
    whiten shapes), utils.rs:147-208 (amari on A^-1 and a permuted A^-1,
    permute, score == d/dy log_lik by finite differences for Tanh(1),
    Exp(0.1), Cube), lbfgs.rs:178-202 (memory bookkeeping).
  * The end-to-end solver trajectory is "parity unpinned" beyond those KATs:
    no reference test pins a W, Y, loss or gradient value.
  * Third-party arithmetic the reference delegates (OpenBLAS dgemm via
    ndarray 0.17.1/cblas-sys 0.1.4; LAPACK eigh/svd/getrf via
    ndarray-linalg 0.18.0 / lax 0.18.0) is restated with numpy's bundled
    OpenBLAS/LAPACK (numpy 2.2), which implements the same LAPACK routines.
  * rand 0.9.2 StdRng (ChaCha12) + rand_distr 0.5.1 StandardNormal (the seeded
    random w_init) are restated in ``oracle/rust_rand.py`` from the crates'
    published algorithms (ChaCha pinned by RFC 8439; the composition itself is
    parity unpinned — no reference-held vector exists offline).

Every function cites the reference file:line it follows.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

try:
    from . import rust_rand
except ImportError:  # imported as a top-level module (tests put oracle/ on sys.path)
    import rust_rand

# ---------------------------------------------------------------------------
# error.rs:9-42 — PicardError variants (as Python exceptions)
# ---------------------------------------------------------------------------


class PicardError(Exception):
    """error.rs:9 PicardError."""


class InvalidDimensions(PicardError):
    """error.rs:19-22; Display error.rs:60 'Invalid dimensions: {message}'."""

    def __init__(self, message: str):
        super().__init__(f"Invalid dimensions: {message}")


class SingularMatrix(PicardError):
    """error.rs:25; Display error.rs:63."""

    def __init__(self):
        super().__init__("Singular matrix encountered during computation")


class ComputationError(PicardError):
    """error.rs:28-31; Display error.rs:66."""

    def __init__(self, message: str):
        super().__init__(f"Computation error: {message}")


class InvalidConfig(PicardError):
    """error.rs:34-40; Display error.rs:69 "Invalid configuration for '{p}': {m}"."""

    def __init__(self, parameter: str, message: str):
        super().__init__(f"Invalid configuration for '{parameter}': {message}")
        self.parameter = parameter


# ---------------------------------------------------------------------------
# density.rs — the elementwise operator API
# ---------------------------------------------------------------------------


@dataclass(frozen=True)
class Density:
    """density.rs:137-144 DensityType {Tanh(alpha), Exp(alpha), Cube}."""

    kind: str = "tanh"  # "tanh" | "exp" | "cube"
    alpha: float = 1.0

    def log_lik(self, y: np.ndarray) -> np.ndarray:
        """density.rs:179-185 → Tanh 50-56 / Exp 91-94 / Cube 122-124."""
        if self.kind == "tanh":
            a = self.alpha
            abs_y = np.abs(y)
            return abs_y + np.log(1.0 + np.exp(-2.0 * a * abs_y)) / a
        if self.kind == "exp":
            a = self.alpha
            return -np.exp(-a * y * y / 2.0) / a
        if self.kind == "cube":
            return (y * y) * (y * y) / 4.0
        raise ValueError(self.kind)

    def score_and_der(self, y: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """density.rs:188-194 → Tanh 58-63 / Exp 96-103 / Cube 126-130."""
        if self.kind == "tanh":
            a = self.alpha
            score = np.tanh(a * y)
            return score, a * (1.0 - score * score)
        if self.kind == "exp":
            a = self.alpha
            y_sq = y * y
            k = np.exp(-a / 2.0 * y_sq)
            return y * k, (1.0 - a * y_sq) * k
        if self.kind == "cube":
            return y * y * y, 3.0 * y * y
        raise ValueError(self.kind)


# ---------------------------------------------------------------------------
# config.rs — PicardConfig / defaults / validate
# ---------------------------------------------------------------------------


@dataclass
class PicardConfig:
    """config.rs:11-62 (16 fields), defaults config.rs:64-85."""

    density: Density = field(default_factory=Density)
    n_components: Optional[int] = None
    ortho: bool = True
    extended: Optional[bool] = None
    whiten: bool = True
    centering: bool = True
    max_iter: int = 500
    tol: float = 1e-7
    m: int = 7
    ls_tries: int = 10
    lambda_min: float = 0.01
    w_init: Optional[np.ndarray] = None
    fastica_it: Optional[int] = None
    jade_it: Optional[int] = None
    random_state: Optional[int] = None
    verbose: bool = False

    def effective_extended(self) -> bool:
        """config.rs:99-101."""
        return self.ortho if self.extended is None else self.extended

    def validate(self) -> None:
        """config.rs:104-142 (same order of checks)."""
        if self.max_iter == 0:
            raise InvalidConfig("max_iter", "must be greater than 0")
        if self.tol <= 0.0:
            raise InvalidConfig("tol", "must be positive")
        if self.lambda_min <= 0.0:
            raise InvalidConfig("lambda_min", "must be positive")
        if self.m == 0:
            raise InvalidConfig("m", "L-BFGS memory size must be at least 1")
        if self.fastica_it is not None and self.jade_it is not None:
            raise InvalidConfig(
                "jade_it",
                "cannot use both fastica_it and jade_it; choose one warm start method",
            )


# ---------------------------------------------------------------------------
# math.rs
# ---------------------------------------------------------------------------


def sym_decorrelation(w: np.ndarray) -> np.ndarray:
    """math.rs:12-33: W <- (W W^T)^{-1/2} W via eigh(UPLO::Lower)."""
    ww_t = w @ w.T
    eigenvalues, eigenvectors = np.linalg.eigh(ww_t, UPLO="L")
    if eigenvalues.min() < 1e-10:  # math.rs:21-24
        raise SingularMatrix()
    s_inv_sqrt = 1.0 / np.sqrt(eigenvalues)
    scaled = eigenvectors * s_inv_sqrt  # column scaling, math.rs:29
    return (scaled @ eigenvectors.T) @ w  # math.rs:30


def matrix_exp(a: np.ndarray) -> np.ndarray:
    """math.rs:38-74: Taylor series with 2^s scaling and s squarings."""
    n = a.shape[0]
    norm = float(np.max(np.abs(a))) if a.size else 0.0
    if norm < 1e-15:
        return np.eye(n)
    s = int(max(math.ceil(math.log2(norm)), 0.0))
    scale = 2.0 ** s
    a_scaled = a / scale
    result = np.eye(n)
    term = np.eye(n)
    for k in range(1, 31):  # max_terms = 30
        term = (term @ a_scaled) / float(k)
        result = result + term
        if float(np.max(np.abs(term))) < 1e-16:
            break
    for _ in range(s):
        result = result @ result
    return result


def sln_det(m: np.ndarray) -> Tuple[float, float]:
    """math.rs:84-88 (ndarray-linalg sln_det: LAPACK getrf; singular → (0,-inf))."""
    sign, logabs = np.linalg.slogdet(m)
    return float(sign), float(logabs)


def skew_symmetric(a: np.ndarray) -> np.ndarray:
    """math.rs:91-93."""
    return (a - a.T) / 2.0


# ---------------------------------------------------------------------------
# lbfgs.rs
# ---------------------------------------------------------------------------


class LbfgsMemory:
    """lbfgs.rs:6-71 (the dead ``update`` lbfgs.rs:42-59 is restated too)."""

    def __init__(self, max_size: int):
        self.s_list: List[np.ndarray] = []
        self.y_list: List[np.ndarray] = []
        self.r_list: List[float] = []
        self.max_size = max_size

    def clear(self) -> None:
        self.s_list.clear()
        self.y_list.clear()
        self.r_list.clear()

    def update(self, s: np.ndarray, y: np.ndarray) -> None:
        """lbfgs.rs:42-59 (unused by core::run, which pushes inline)."""
        sy = float(np.sum(s * y))
        if abs(sy) > 1e-15:
            r = 1.0 / sy
            if len(self.s_list) >= self.max_size:
                self.s_list.pop(0)
                self.y_list.pop(0)
                self.r_list.pop(0)
            self.s_list.append(s)
            self.y_list.append(y)
            self.r_list.append(r)

    def is_empty(self) -> bool:
        return not self.s_list

    def __len__(self) -> int:
        return len(self.s_list)


def compute_direction(g, h, h_off, memory: LbfgsMemory, ortho: bool) -> np.ndarray:
    """lbfgs.rs:84-133 two-loop recursion."""
    q = g.copy()
    alpha_list = []
    for s, y, r in reversed(list(zip(memory.s_list, memory.y_list, memory.r_list))):
        alpha = r * float(np.sum(s * q))
        alpha_list.append(alpha)
        q = q - alpha * y
    alpha_list.reverse()
    if ortho:
        z = q / h
        z = (z - z.T) / 2.0
    else:
        z = solve_hessian_system(h, h_off, q)
    for (s, y, r), alpha in zip(zip(memory.s_list, memory.y_list, memory.r_list), alpha_list):
        beta = r * float(np.sum(y * z))
        z = z + (alpha - beta) * s
    return -z


def solve_hessian_system(h, h_off, g) -> np.ndarray:
    """lbfgs.rs:136-150 (2x2 block solve per (i, j))."""
    n = h.shape[0]
    det = h * h.T - np.outer(h_off, h_off)
    num = h.T * g - h_off[:, None] * g.T
    out = np.zeros((n, n))
    mask = np.abs(det) > 1e-15
    out[mask] = num[mask] / det[mask]
    return out


def regularize_hessian(h: np.ndarray, h_off, lambda_min: float) -> None:
    """lbfgs.rs:155-171 — in place, row-major, so h[j,i] may already be updated."""
    n = h.shape[0]
    for i in range(n):
        for j in range(n):
            if i != j:
                diff = h[i, j] - h[j, i]
                discr = math.sqrt(diff * diff + 4.0 * h_off[i] * h_off[j])
                eigenvalue = 0.5 * (h[i, j] + h[j, i] - discr)
                if eigenvalue < lambda_min:
                    h[i, j] += lambda_min - eigenvalue


# ---------------------------------------------------------------------------
# core.rs
# ---------------------------------------------------------------------------

SINGULAR_PENALTY = 1e15  # core.rs:93-94


def compute_loss(y, w, density: Density, signs, ortho: bool, extended: bool):
    """core.rs:39-85 → float, or the string "singular" (LossResult::Singular)."""
    n = y.shape[0]
    t = float(y.shape[1])
    if not ortho:
        sign, log_abs_det = sln_det(w)
        if sign == 0.0:
            return "singular"
        loss = -log_abs_det
    else:
        loss = 0.0
    for i in range(n):
        row = y[i].copy()
        loss += signs[i] * float(density.log_lik(row).sum()) / t
        if extended and not ortho:
            loss += 0.5 * float(np.sum(row * row)) / t
    return loss


def loss_to_f64(res) -> float:
    """core.rs:90-96."""
    return SINGULAR_PENALTY if isinstance(res, str) else float(res)


@dataclass
class LineSearchResult:
    """core.rs:153-159."""

    success: bool
    y: np.ndarray
    w: np.ndarray
    loss: float
    step: np.ndarray
    n_evals: int = 0


def line_search(y, w, density, direction, signs, current_loss, ls_tries, ortho, extended):
    """core.rs:99-150 backtracking line search (Y_new = M·Y, core.rs:124)."""
    n = w.shape[0]
    alpha = 1.0
    y_new = y.copy()
    w_new = w.copy()
    new_loss = current_loss
    evals = 0
    for _ in range(ls_tries):
        transform = matrix_exp(direction * alpha) if ortho else np.eye(n) + alpha * direction
        y_new = transform @ y
        w_new = transform @ w
        new_loss = loss_to_f64(compute_loss(y_new, w_new, density, signs, ortho, extended))
        evals += 1
        if new_loss < current_loss:
            return LineSearchResult(True, y_new, w_new, new_loss, direction * alpha, evals)
        alpha /= 2.0
    return LineSearchResult(False, y_new, w_new, new_loss, direction * alpha, evals)


@dataclass
class CoreInfo:
    """core.rs:10-19 (+ oracle-only trace fields)."""

    converged: bool
    gradient_norm: float
    n_iterations: int
    signs: Optional[np.ndarray]
    trace_loss: List[float] = field(default_factory=list)
    trace_gnorm: List[float] = field(default_factory=list)
    n_evals: int = 0


def run(x, density: Density, ortho, extended, m, max_iter, tol, lambda_min, ls_tries,
        verbose=False, covariance=None):
    """core.rs:162-401 — the Picard / Picard-O iteration."""
    n, t = x.shape
    t_f = float(t)
    w = np.eye(n)
    y = x.copy()
    memory = LbfgsMemory(m)
    signs = np.ones(n)
    old_signs = signs.copy()
    init = compute_loss(y, w, density, signs, ortho, extended)  # core.rs:185
    if isinstance(init, str):
        raise SingularMatrix()
    current_loss = init
    gradient_norm = 1.0
    converged = False
    if extended:  # core.rs:199-205
        c = covariance.copy() if covariance is not None else (y @ y.T) / t_f
    else:
        c = np.eye(n)
    g_old = None
    prev_step = None
    n_iter = 0
    info = CoreInfo(False, 1.0, 0, None)
    info.n_evals = 1
    for it in range(max_iter):  # core.rs:211
        n_iter = it
        psi_y, psi_dy = density.score_and_der(y)  # 215
        g = (psi_y @ y.T) / t_f  # 218
        y_square = y * y  # 221
        sign_change = False
        if extended:  # 225-253
            psi_dy_mean = psi_dy.sum(axis=1) / t_f
            k = psi_dy_mean * np.diag(c) - np.diag(g)
            # f64::signum: +0 → +1, -0 → -1, NaN → NaN (core.rs:232)
            signs = np.where(np.isnan(k), np.nan, np.copysign(1.0, k))
            if it > 0:
                sign_change = bool(np.any(signs != old_signs))
            old_signs = signs.copy()
            g = g * signs[:, None]
            psi_dy = psi_dy * signs[:, None]
            if not ortho:
                g = g + c
                psi_dy = psi_dy + 1.0
        h_off = np.diag(g).copy() if ortho else np.ones(n)  # 256-260
        if ortho:  # 263-272
            psi_dy_mean = psi_dy.sum(axis=1) / t_f
            h = 0.5 * (psi_dy_mean[:, None] + psi_dy_mean[None, :] - h_off[:, None] - h_off[None, :])
            h = np.maximum(h, lambda_min)
        else:
            h = (psi_dy @ y_square.T) / t_f  # 274
            regularize_hessian(h, h_off, lambda_min)
        if ortho:  # 280-286
            g = skew_symmetric(g)
        else:
            g = g - np.eye(n)
        gradient_norm = float(np.max(np.abs(g)))  # 289
        info.trace_gnorm.append(gradient_norm)
        if gradient_norm < tol:
            converged = True
            break
        if it > 0 and prev_step is not None and g_old is not None:  # 296-313
            step = prev_step
            prev_step = None
            y_diff = g - g_old
            with np.errstate(divide="ignore", invalid="ignore"):
                r = 1.0 / float(np.sum(step * y_diff))
            if math.isfinite(r):
                memory.s_list.append(step)
                memory.y_list.append(y_diff)
                memory.r_list.append(r)
                if len(memory.s_list) > m:
                    memory.s_list.pop(0)
                    memory.y_list.pop(0)
                    memory.r_list.pop(0)
        g_old = g.copy()
        if extended and sign_change:  # 317-331
            res = compute_loss(y, w, density, signs, ortho, extended)
            current_loss = SINGULAR_PENALTY if isinstance(res, str) else res
            memory.clear()
        direction = compute_direction(g, h, h_off, memory, ortho)  # 334
        res = line_search(y, w, density, direction, signs, current_loss, ls_tries, ortho, extended)
        info.n_evals += res.n_evals
        if not res.success:  # 349-364
            memory.clear()
            res = line_search(y, w, density, -g, signs, current_loss, 10, ortho, extended)
            info.n_evals += res.n_evals
        prev_step = res.step  # 370
        y = res.y
        w = res.w
        if extended and covariance is not None:  # 375-379
            c = w @ covariance @ w.T
        current_loss = res.loss  # 381
        info.trace_loss.append(current_loss)
        if verbose:
            print(f"iteration {it + 1}, gradient norm = {rust_e4(gradient_norm)}, "
                  f"loss = {rust_e4(current_loss)}")
    info.converged = converged
    info.gradient_norm = gradient_norm
    info.n_iterations = n_iter + 1  # core.rs:396
    info.signs = signs if extended else None
    return y, w, info


def rust_e4(v: float) -> str:
    """Rust's ``{:.4e}`` (core.rs:385): mantissa .4f, exponent without padding."""
    if not math.isfinite(v):
        return "NaN" if math.isnan(v) else ("inf" if v > 0 else "-inf")
    s = f"{v:.4e}"
    mant, exp = s.split("e")
    return f"{mant}e{int(exp)}"


# ---------------------------------------------------------------------------
# whitening.rs
# ---------------------------------------------------------------------------


def center(x: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """whitening.rs:24-35."""
    mean = x.sum(axis=1) / x.shape[1]
    return x - mean[:, None], mean


def whiten_matrix_from_u_s(u: np.ndarray, s: np.ndarray, n_components: int, n_samples: int):
    """whitening.rs:72-107: min-sv check, K = (U/s)^T·sqrt(T), sign rule."""
    if float(np.min(s[:n_components])) < 1e-10:
        raise SingularMatrix()
    scale = math.sqrt(float(n_samples))
    k = (u[:, :n_components] / s[:n_components]).T * scale
    for i in range(k.shape[0]):
        # max_by over |·| keeps the LAST maximal element on ties (Iterator::max_by)
        absr = np.abs(k[i])
        idx = int(len(absr) - 1 - np.argmax(absr[::-1]))
        if k[i, idx] < 0.0:
            k[i] = -k[i]
    return k


def whiten(x: np.ndarray, n_components: int):
    """whitening.rs:48-116 (LAPACK SVD of the N×T data; U only)."""
    n_features, n_samples = x.shape
    if n_components > n_features:
        raise InvalidDimensions(
            f"n_components ({n_components}) cannot exceed n_features ({n_features})")
    u, s, _ = np.linalg.svd(x, full_matrices=False)
    k = whiten_matrix_from_u_s(u, s, n_components, n_samples)
    return k @ x, k


# ---------------------------------------------------------------------------
# jade.rs
# ---------------------------------------------------------------------------


def jade(x: np.ndarray, max_iter: int, tol: float = 1e-6, verbose: bool = False) -> np.ndarray:
    """jade.rs:22-72."""
    n = x.shape[0]
    if n < 2:
        return np.eye(n)
    cumulants = compute_cumulant_matrices(x)
    v = np.eye(n)
    for _ in range(max_iter):
        max_theta = 0.0
        for p in range(n):
            for q in range(p + 1, n):
                c, s, theta = compute_givens_rotation(cumulants, v, p, q)
                max_theta = max(max_theta, abs(theta))
                apply_givens_rotation(v, c, s, p, q)
        if max_theta < tol:
            break
    return sym_decorrelation(v)


def jade_sweeps_batched(mats: np.ndarray, max_iter: int, tol: float = 1e-6, max_pairs: Optional[int] = None):
    """jade.rs:37-69 with the matrix loop of compute_givens_rotation (jade.rs:137-167)
    vectorised over the stacked cumulant matrices ``mats`` [np, n, n]: the same
    cyclic (p, q) order, the same b = v_pᵀ M v_q forms recomputed from V for
    every pair, the same angle formula (jade.rs:172-182) and rotation of V
    (jade.rs:188-197). Only the order of the g-sums over matrices differs
    (numpy's). ``max_pairs`` stops after that many Givens pairs in all (a test
    hook: the sweeps amplify rounding, so parity is checked on prefixes).
    Returns (V, sweeps run, tolerance met) — before sym_decorrelation."""
    npm, n, _ = mats.shape
    flat = np.ascontiguousarray(mats).reshape(npm * n, n)
    v = np.eye(n)
    it = 0
    converged = False
    done = 0
    while it < max_iter and not converged:
        max_theta = 0.0
        for p in range(n):
            for q in range(p + 1, n):
                if max_pairs is not None and done >= max_pairs:
                    return v, it, False
                done += 1
                mv = (flat @ v[:, [p, q]]).reshape(npm, n, 2)  # M v_p, M v_q for every M
                b00 = mv[:, :, 0] @ v[:, p]
                b01 = mv[:, :, 1] @ v[:, p]   # v_pᵀ M v_q
                b10 = mv[:, :, 0] @ v[:, q]   # v_qᵀ M v_p
                b11 = mv[:, :, 1] @ v[:, q]
                h_pq = b01 + b10
                h_d = b00 - b11
                g00, g01, g11 = float(h_pq @ h_pq), float(h_pq @ h_d), float(h_d @ h_d)
                diff = g11 - g00
                angle = 0.0 if (abs(g01) < 1e-15 and abs(diff) < 1e-15) else 0.25 * math.atan2(2.0 * g01, diff)
                max_theta = max(max_theta, abs(angle))
                apply_givens_rotation(v, math.cos(angle), math.sin(angle), p, q)
        it += 1
        converged = max_theta < tol
    return v, it, converged


def cumulants_from_moments(m4: np.ndarray, n: int, t: float) -> np.ndarray:
    """jade.rs:101-126 from the pair-product moment matrix m4 = Σ_t z zᵀ, z = (y_i y_j)_{i≤j}
    (what pc_ctx_moments4 returns): Q_ij[k, l] = E[y_i y_j y_k y_l] − δ_ij δ_kl − δ_ik δ_jl
    − δ_il δ_jk, symmetrised; stacked [n(n+1)/2, n, n] in the reference's (i ≤ j) order."""
    pairs = [(i, j) for i in range(n) for j in range(i, n)]
    pidx = np.zeros((n, n), dtype=np.int64)
    for a, (i, j) in enumerate(pairs):
        pidx[i, j] = pidx[j, i] = a
    eye = np.eye(n)
    out = np.empty((len(pairs), n, n))
    for a, (i, j) in enumerate(pairs):
        q = m4[a][pidx] / t - eye[i, j] * eye - np.outer(eye[i], eye[j]) - np.outer(eye[j], eye[i])
        out[a] = (q + q.T) / 2.0
    return out


def compute_cumulant_matrices(x: np.ndarray) -> List[np.ndarray]:
    """jade.rs:78-131 (the n×n×T ``xx`` tensor is contracted without materialising it)."""
    n, t = x.shape
    e4 = np.einsum("it,jt,kt,lt->ijkl", x, x, x, x, optimize=True) / float(t)
    eye = np.eye(n)
    mats = []
    for i in range(n):
        for j in range(i, n):
            q = e4[i, j] - (eye[i, j] * eye) - np.outer(eye[i], eye[j]) - np.outer(eye[j], eye[i])
            mats.append((q + q.T) / 2.0)
    return mats


def compute_givens_rotation(matrices, v, p, q):
    """jade.rs:137-185."""
    g00 = g01 = g11 = 0.0
    vp, vq = v[:, p], v[:, q]
    for m in matrices:
        b00 = vp @ m @ vp
        b01 = vp @ m @ vq
        b10 = vq @ m @ vp
        b11 = vq @ m @ vq
        h_pq = b01 + b10
        h_pp_qq = b00 - b11
        g00 += h_pq * h_pq
        g01 += h_pq * h_pp_qq
        g11 += h_pp_qq * h_pp_qq
    diff = g11 - g00
    if abs(g01) < 1e-15 and abs(diff) < 1e-15:
        angle = 0.0
    else:
        angle = 0.25 * math.atan2(2.0 * g01, diff)
    return math.cos(angle), math.sin(angle), angle


def apply_givens_rotation(v, c, s, p, q):
    """jade.rs:188-197 (in place)."""
    v_p = v[:, p].copy()
    v_q = v[:, q].copy()
    v[:, p] = c * v_p - s * v_q
    v[:, q] = s * v_p + c * v_q


# ---------------------------------------------------------------------------
# solver.rs / result.rs
# ---------------------------------------------------------------------------


@dataclass
class PicardResult:
    """result.rs:7-33."""

    whitening: Optional[np.ndarray]
    unmixing: np.ndarray
    sources: np.ndarray
    mean: Optional[np.ndarray]
    n_iterations: int
    converged: bool
    gradient_norm: float
    signs: Optional[np.ndarray]
    info: Optional[CoreInfo] = None

    def full_unmixing(self) -> np.ndarray:
        """result.rs:39-44."""
        return self.unmixing @ self.whitening if self.whitening is not None else self.unmixing.copy()

    def mixing(self) -> np.ndarray:
        """result.rs:49-64 (pinv via Gauss-Jordan, fallback W^T)."""
        full_w = self.full_unmixing()
        wt = full_w.T
        wtw = wt @ full_w
        inv = invert_matrix(wtw)
        if inv is not None:
            return inv @ wt
        return wt.copy()


def invert_matrix(m: np.ndarray) -> Optional[np.ndarray]:
    """result.rs:68-129 Gauss-Jordan with partial pivoting."""
    n = m.shape[0]
    aug = np.zeros((n, 2 * n))
    aug[:, :n] = m
    aug[:, n:] = np.eye(n)
    for i in range(n):
        max_row = i
        for k in range(i + 1, n):
            if abs(aug[k, i]) > abs(aug[max_row, i]):
                max_row = k
        aug[[i, max_row]] = aug[[max_row, i]]
        if abs(aug[i, i]) < 1e-15:
            return None
        aug[i] = aug[i] / aug[i, i]
        for k in range(n):
            if k != i:
                aug[k] = aug[k] - aug[k, i] * aug[i]
    return aug[:, n:].copy()


def ica_par(x, density: Density, max_iter: int, w_init, verbose=False):
    """solver.rs:218-249 FastICA parallel iterations."""
    w = sym_decorrelation(w_init)
    p = float(x.shape[1])
    for _ in range(max_iter):
        wx = w @ x
        gwtx, g_wtx = density.score_and_der(wx)
        g_wtx_mean = g_wtx.sum(axis=1) / p
        c = (gwtx @ x.T) / p
        c = c - g_wtx_mean[:, None] * w
        w = sym_decorrelation(c)
    return w


def fit_with_config(x: np.ndarray, config: PicardConfig, w_init_random=None) -> PicardResult:
    """solver.rs:45-189. ``w_init_random`` replaces the StdRng draw (solver.rs:112-118)."""
    config.validate()
    n, p = x.shape
    if n == 0 or p == 0:
        raise InvalidDimensions("Input matrix cannot be empty")
    n_components = min(config.n_components if config.n_components is not None else min(n, p), min(n, p))
    extended = config.effective_extended()
    if config.centering:
        x1, x_mean = center(x)
    else:
        x1, x_mean = x.copy(), None
    if config.whiten:
        x1, k = whiten(x1, n_components)
    else:
        k = None
    actual = x1.shape[0]
    if config.w_init is not None:
        w_init = np.asarray(config.w_init, dtype=np.float64)
        if w_init.shape != (actual, actual):
            raise InvalidDimensions(
                f"w_init shape {list(w_init.shape)} doesn't match expected ({actual}, {actual})")
        w_init = w_init.copy()
    else:
        if w_init_random is None:
            if config.random_state is not None:  # solver.rs:56-58, :112-118 (oracle/rust_rand.py)
                w_init_random = np.array(rust_rand.random_w_init(config.random_state, actual))
            else:  # solver.rs:59: an OS-entropy stream (not reproducible by design)
                w_init_random = np.random.default_rng().standard_normal((actual, actual))
        w_init = sym_decorrelation(np.asarray(w_init_random, dtype=np.float64))
    if config.jade_it is not None:
        w_init = jade(x1, config.jade_it, 1e-6, config.verbose)
    elif config.fastica_it is not None:
        w_init = ica_par(x1, config.density, config.fastica_it, w_init, config.verbose)
    x1 = w_init @ x1
    covariance = np.eye(actual) if (extended and config.whiten) else None
    y, w, info = run(x1, config.density, config.ortho, extended, config.m, config.max_iter,
                     config.tol, config.lambda_min, config.ls_tries, config.verbose, covariance)
    w = w @ w_init
    return PicardResult(k, w, y, x_mean, info.n_iterations, info.converged, info.gradient_norm,
                        info.signs, info)


def fit(x: np.ndarray) -> PicardResult:
    """solver.rs:33-35."""
    return fit_with_config(x, PicardConfig())


def transform(x: np.ndarray, result: PicardResult) -> np.ndarray:
    """solver.rs:199-214."""
    x = x.copy()
    if result.mean is not None:
        x = x - result.mean[:, None]
    return result.full_unmixing() @ x


# ---------------------------------------------------------------------------
# utils.rs
# ---------------------------------------------------------------------------


def amari_distance(w: np.ndarray, a: np.ndarray) -> float:
    """utils.rs:82-103."""
    p = w @ a
    n = float(p.shape[0])

    def s(r):
        total = 0.0
        for i in range(r.shape[0]):
            row_sq = r[i] * r[i]
            row_sum = float(row_sq.sum())
            row_max = float(row_sq.max()) if row_sq.size else 0.0
            row_max = max(row_max, 0.0)
            if row_max > 1e-15:
                total += row_sum / row_max - 1.0
        return total

    pa = np.abs(p)
    return (s(pa) + s(pa.T.copy())) / (2.0 * n)


def permute(a: np.ndarray, scale: bool = True) -> np.ndarray:
    """utils.rs:16-69."""
    n = a.shape[0]
    a = a.copy()
    done = False
    while not done:
        done = True
        for i in range(n):
            for j in range(i):
                diag_sq = a[i, i] ** 2 + a[j, j] ** 2
                off_sq = a[i, j] ** 2 + a[j, i] ** 2
                if diag_sq < off_sq:
                    a[[i, j]] = a[[j, i]]
                    done = False
    if scale:
        for i in range(n):
            d = a[i, i]
            if abs(d) > 1e-10:
                a[i] = a[i] / d
    col_sums = np.abs(a).sum(axis=0)
    order = sorted(range(n), key=lambda j: col_sums[j])
    return a[np.ix_(order, order)]


def check_density(density: Density, tol: float) -> bool:
    """utils.rs:110-137 finite-difference score check (test-only in the reference)."""
    eps = 1e-7
    for y in [-2.0, -1.0, -0.5, 0.0, 0.5, 1.0, 2.0]:
        lp = density.log_lik(np.array([y + eps]))[0]
        lm = density.log_lik(np.array([y - eps]))[0]
        numerical = (lp - lm) / (2.0 * eps)
        score, _ = density.score_and_der(np.array([[y]]))
        if abs(numerical - score[0, 0]) > tol:
            return False
    return True


# ---------------------------------------------------------------------------
# Pass-P statistics: the per-evaluation sums the HIP kernel produces
# (core.rs:215-274 and core.rs:73-82 re-expressed as raw sums over t)
# ---------------------------------------------------------------------------


def pass_stats(w_total: np.ndarray, mu: Optional[np.ndarray], x: np.ndarray, density: Density,
               need_h: bool):
    """Raw sums for Y = W_total·(X − μ):
    G_raw = ψ(Y)·Yᵀ (core.rs:218), H_raw = ψ'(Y)·(Y∘Y)ᵀ (core.rs:274),
    Σ_t ψ'(y_it) (core.rs:226,264), Σ_t ℓ(y_it) (core.rs:76), Σ_t y_it² (core.rs:79).
    """
    xc = x - mu[:, None] if mu is not None else x
    y = w_total @ xc
    psi, dpsi = density.score_and_der(y)
    out = {
        "G": psi @ y.T,
        "dpsi": dpsi.sum(axis=1),
        "ll": density.log_lik(y).sum(axis=1),
        "y2": (y * y).sum(axis=1),
    }
    if need_h:
        out["H"] = dpsi @ (y * y).T
    return out
