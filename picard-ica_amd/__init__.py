"""picard_ica_amd — MI355X-native Picard / Picard-O ICA (Python host mirror).

Thin ctypes layer over the C ABI in ``include/picard_mi355x.h``
(``libpicard_mi355x.so``, built in-tree by ``make -C picard-ica_amd``).
Names, argument meaning, defaults and errors mirror the Rust reference
lmmx/picard-ica v0.1.6 (src/lib.rs:50-57):

    Picard.fit(x)                       ← Picard::fit              (src/solver.rs:33)
    Picard.fit_with_config(x, config)   ← Picard::fit_with_config  (src/solver.rs:45)
    Picard.transform(x, result)         ← Picard::transform        (src/solver.rs:199)
    PicardConfig / PicardConfig.builder() ← config.rs:11-62, :147-273
    PicardResult.full_unmixing()/mixing() ← result.rs:39, :49
    DensityType.tanh()/exp()/cube()     ← density.rs:137-195
    utils.amari_distance / utils.permute ← utils.rs:82, :16
    PicardError subclasses              ← error.rs:9-42

There is no CPU fallback: every compute call goes through the HIP library,
and importing this package raises if the library is missing.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

__all__ = [
    "Picard", "PicardConfig", "ConfigBuilder", "PicardResult", "DensityType", "PicardError",
    "InvalidDimensions", "SingularMatrix", "ComputationError", "InvalidConfig", "NotConverged",
    "Unsupported", "DeviceContext", "LocalGroup", "Solver", "utils", "lib", "LIB_PATH",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpicard_mi355x.so")

# ------------------------------------------------------------------ errors


class PicardError(Exception):
    """error.rs:9 PicardError."""

    code = -1


class InvalidDimensions(PicardError):
    code = 1


class SingularMatrix(PicardError):
    code = 2


class ComputationError(PicardError):
    code = 3


class InvalidConfig(PicardError):
    code = 4


class NotConverged(PicardError):
    code = 5


class Unsupported(ComputationError):
    """PC_ERR_UNSUPPORTED (operator boundary only): the pass is not available for this
    context / shape; nothing ran and a rank group is not aborted, so the documented fallback
    can be called next. A ComputationError, so callers that catch those still do."""

    code = 6


_ERRORS = {c.code: c for c in (InvalidDimensions, SingularMatrix, ComputationError, InvalidConfig, NotConverged,
                               Unsupported)}

# ------------------------------------------------------------------ C types


class _Density(C.Structure):
    _fields_ = [("kind", C.c_int32), ("alpha", C.c_double)]


class _Config(C.Structure):
    _fields_ = [
        ("density", _Density),
        ("has_n_components", C.c_int32), ("n_components", C.c_uint64),
        ("ortho", C.c_int32),
        ("has_extended", C.c_int32), ("extended", C.c_int32),
        ("whiten", C.c_int32),
        ("centering", C.c_int32),
        ("max_iter", C.c_uint64),
        ("tol", C.c_double),
        ("m", C.c_uint64),
        ("ls_tries", C.c_uint64),
        ("lambda_min", C.c_double),
        ("w_init", C.POINTER(C.c_double)), ("w_init_rows", C.c_uint64), ("w_init_cols", C.c_uint64),
        ("has_fastica_it", C.c_int32), ("fastica_it", C.c_uint64),
        ("has_jade_it", C.c_int32), ("jade_it", C.c_uint64),
        ("has_random_state", C.c_int32), ("random_state", C.c_uint64),
        ("verbose", C.c_int32),
        ("device", C.c_int32),
        ("want_sources", C.c_int32),
    ]


class _Result(C.Structure):
    _fields_ = [
        ("whitening", C.POINTER(C.c_double)), ("whitening_rows", C.c_uint64), ("whitening_cols", C.c_uint64),
        ("unmixing", C.POINTER(C.c_double)), ("unmixing_rows", C.c_uint64), ("unmixing_cols", C.c_uint64),
        ("sources", C.POINTER(C.c_double)), ("sources_rows", C.c_uint64), ("sources_cols", C.c_uint64),
        ("mean", C.POINTER(C.c_double)), ("mean_len", C.c_uint64),
        ("n_iterations", C.c_uint64),
        ("converged", C.c_int32),
        ("gradient_norm", C.c_double),
        ("signs", C.POINTER(C.c_double)), ("signs_len", C.c_uint64),
        ("n_evaluations", C.c_uint64),
    ]


RowsumFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double))
GramFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double))
EvalFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_uint64, C.POINTER(C.c_double), _Density,
                     C.c_uint32, C.POINTER(C.c_double))
SourcesFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_uint64, C.POINTER(C.c_double),
                        C.POINTER(C.c_double))
Moments4Fn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_uint64, C.POINTER(C.c_double),
                         C.POINTER(C.c_double))
MultiFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_uint64,
                      C.POINTER(C.c_double), _Density, C.POINTER(C.c_double), C.c_uint64, C.POINTER(C.c_double),
                      C.POINTER(C.c_double))


ScreenFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_uint64, C.POINTER(C.c_double), _Density,
                       C.POINTER(C.c_double), C.POINTER(C.c_double))


class _HostEvaluator(C.Structure):
    _fields_ = [
        ("user", C.c_void_p), ("n_features", C.c_uint64), ("n_samples", C.c_uint64),
        ("rowsum", RowsumFn), ("gram", GramFn), ("eval", EvalFn), ("sources", SourcesFn),
        ("moments4", Moments4Fn), ("eval_loss_multi", MultiFn), ("eval_loss_screen", ScreenFn),
    ]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C picard-ica_amd` (hipcc, gfx950). "
            "There is no CPU fallback.")
    lib = C.CDLL(LIB_PATH)
    P = C.POINTER
    d, u64, i32, vp, cp, sz = P(C.c_double), C.c_uint64, C.c_int32, C.c_void_p, C.c_char_p, C.c_size_t
    sigs = {
        "pc_config_default": (None, [P(_Config)]),
        "pc_config_validate": (C.c_int, [P(_Config), cp, sz]),
        "pc_fit": (C.c_int, [d, u64, u64, P(_Config), P(_Result), cp, sz]),
        "pc_fit_default": (C.c_int, [d, u64, u64, P(_Result), cp, sz]),
        "pc_transform": (C.c_int, [d, u64, u64, P(_Result), d, i32, cp, sz]),
        "pc_full_unmixing": (C.c_int, [P(_Result), d]),
        "pc_mixing": (C.c_int, [P(_Result), d]),
        "pc_result_free": (None, [P(_Result)]),
        "pc_amari_distance": (C.c_double, [d, d, u64]),
        "pc_permute": (None, [d, u64, i32, d]),
        "pc_error_name": (C.c_char_p, [C.c_int]),
        "pc_version": (C.c_char_p, []),
        "pc_abi_version": (C.c_int, []),
        "pc_group_create_local": (C.c_int, [i32, P(vp), cp, sz]),
        "pc_group_destroy": (None, [vp]),
        "pc_ctx_create_in_group": (C.c_int, [i32, i32, vp, P(vp), cp, sz]),
        "pc_ctx_comm_stats": (None, [vp, P(C.c_int64)]),
        "pc_ctx_comm_timing": (None, [vp, d]),
        "pc_ctx_alloc_stats": (None, [vp, d]),
        "pc_last_teardown": (None, [d]),
        "pc_ctx_abort": (None, [vp, cp]),
        "pc_ctx_release_caches": (C.c_int, [vp, cp, sz]),
        "pc_rccl_unique_id": (C.c_int, [cp]),
        "pc_ctx_create": (C.c_int, [i32, i32, i32, cp, P(vp), cp, sz]),
        "pc_ctx_destroy": (None, [vp]),
        "pc_ctx_load": (C.c_int, [vp, d, u64, u64, u64, u64, cp, sz]),
        "pc_ctx_generate": (C.c_int, [vp, u64, u64, u64, d, cp, sz]),
        "pc_ctx_download": (C.c_int, [vp, d]),
        "pc_ctx_n_local": (u64, [vp]),
        "pc_ctx_t0": (u64, [vp]),
        "pc_ctx_eval": (C.c_int, [vp, d, u64, d, _Density, C.c_uint32, d, cp, sz]),
        "pc_ctx_eval_loss": (C.c_int, [vp, d, u64, d, _Density, C.c_uint32, d, P(i32), cp, sz]),
        "pc_ctx_eval_loss_multi": (C.c_int, [vp, d, d, u64, d, _Density, d, u64, d, d, cp, sz]),
        "pc_ctx_eval_loss_multi_bound": (C.c_int, [vp, d, d, u64, d, _Density, d, u64, d, d, cp, sz]),
        "pc_ctx_eval_complete": (C.c_int, [vp, _Density, C.c_uint32, d, cp, sz]),
        "pc_ctx_rowsum": (C.c_int, [vp, d, cp, sz]),
        "pc_ctx_gram": (C.c_int, [vp, d, d, cp, sz]),
        "pc_ctx_sources": (C.c_int, [vp, d, u64, d, d, cp, sz]),
        "pc_ctx_moments4": (C.c_int, [vp, d, u64, d, d, cp, sz]),
        "pc_ctx_sources_device": (C.c_int, [vp, d, u64, d, P(C.c_void_p), P(u64), d, cp, sz]),
        "pc_ctx_jade": (C.c_int, [vp, d, u64, d, u64, C.c_double, i32, d, P(u64), cp, sz]),
        "pc_ctx_last_timing": (None, [vp, d, d]),
        "pc_ctx_kernel_stats": (None, [vp, d, d, P(u64), i32]),
        "pc_device_synchronize": (C.c_int, [i32]),
        "pc_device_mem_info": (C.c_int, [i32, P(u64), P(u64)]),
        "pc_device_check_fp32_transcendentals": (C.c_int, [i32, P(C.c_double)]),
        "pc_ctx_kernel_breakdown": (None, [vp, d, P(u64), i32]),
        "pc_ctx_set_y_stage": (C.c_int, [vp, i32]),
        "pc_ctx_int8_passes": (u64, [vp]),
        "pc_ctx_set_g_stage": (C.c_int, [vp, i32]),
        "pc_ctx_g8_passes": (u64, [vp]),
        "pc_ctx_multi_ybuf_passes": (u64, [vp]),
        "pc_ctx_matrix_exp": (i32, [vp, d, u64, d, cp, sz]),
        "pc_matrix_exp": (None, [d, u64, d]),
        "pc_ctx_screen_stats": (None, [vp, d, P(u64), i32]),
        "pc_ctx_eval_loss_screen": (C.c_int, [vp, d, u64, d, _Density, d, d, cp, sz]),
        "pc_ctx_eval_loss_screen2": (C.c_int, [vp, d, d, u64, d, _Density, d, d, d, d, cp, sz]),
        "pc_ctx_screen_tries": (u64, [vp]),
        "pc_ctx_screen_digit_gram": (C.c_int, [vp, d, d, cp, sz]),
        "pc_ctx_screen_products": (u64, [vp]),
        "pc_solver_create": (C.c_int, [vp, P(_Config), P(vp), cp, sz]),
        "pc_solver_step": (C.c_int, [vp, P(i32), cp, sz]),
        "pc_solver_finish": (C.c_int, [vp, P(_Result), cp, sz]),
        "pc_solver_destroy": (None, [vp]),
        "pc_solver_last": (None, [vp, d, d, P(u64)]),
        "pc_solver_timing": (None, [vp, d]),
        "pc_solver_setup_timing": (None, [vp, d]),
        "pc_fit_with_evaluator": (C.c_int, [P(_HostEvaluator), P(_Config), P(_Result), cp, sz]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()

# public list of exported symbols (checked against include/*.h by the tests)
EXPORTED = [
    "pc_config_default", "pc_config_validate", "pc_fit", "pc_fit_default", "pc_transform",
    "pc_full_unmixing", "pc_mixing", "pc_result_free", "pc_amari_distance", "pc_permute",
    "pc_error_name", "pc_version", "pc_abi_version", "pc_rccl_unique_id", "pc_ctx_create", "pc_ctx_destroy",
    "pc_group_create_local", "pc_group_destroy", "pc_ctx_create_in_group", "pc_ctx_comm_stats", "pc_ctx_comm_timing", "pc_ctx_alloc_stats", "pc_last_teardown", "pc_ctx_abort",
    "pc_ctx_release_caches",
    "pc_ctx_load", "pc_ctx_generate", "pc_ctx_download", "pc_ctx_n_local", "pc_ctx_t0",
    "pc_ctx_eval", "pc_ctx_eval_loss", "pc_ctx_eval_loss_multi", "pc_ctx_eval_loss_multi_bound", "pc_ctx_eval_complete", "pc_ctx_rowsum", "pc_ctx_gram", "pc_ctx_sources", "pc_ctx_sources_device", "pc_ctx_moments4",
    "pc_ctx_jade", "pc_ctx_last_timing", "pc_ctx_kernel_stats", "pc_ctx_kernel_breakdown", "pc_ctx_set_y_stage", "pc_ctx_int8_passes", "pc_ctx_set_g_stage", "pc_ctx_g8_passes", "pc_ctx_multi_ybuf_passes", "pc_ctx_matrix_exp", "pc_matrix_exp", "pc_ctx_screen_stats", "pc_ctx_eval_loss_screen", "pc_ctx_eval_loss_screen2", "pc_ctx_screen_tries", "pc_ctx_screen_digit_gram", "pc_ctx_screen_products", "pc_device_synchronize", "pc_device_mem_info", "pc_device_check_fp32_transcendentals", "pc_solver_create", "pc_solver_step", "pc_solver_finish",
    "pc_solver_destroy", "pc_solver_last", "pc_solver_timing", "pc_solver_setup_timing", "pc_fit_with_evaluator",
]


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _c64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def _raise(rc: int, buf) -> None:
    if rc != 0:
        msg = buf.value.decode(errors="replace") if hasattr(buf, "value") else str(buf)
        raise _ERRORS.get(rc, PicardError)(msg)


def _errbuf():
    return C.create_string_buffer(1024)

# ------------------------------------------------------------------ API mirror


@dataclass(frozen=True)
class DensityType:
    """density.rs:137-195 (Tanh(alpha) | Exp(alpha) | Cube)."""

    kind: int = 0
    alpha: float = 1.0

    @staticmethod
    def tanh(alpha: float = 1.0) -> "DensityType":
        return DensityType(0, alpha)

    tanh_with_alpha = tanh

    @staticmethod
    def exp(alpha: float = 1.0) -> "DensityType":
        return DensityType(1, alpha)

    exp_with_alpha = exp

    @staticmethod
    def cube() -> "DensityType":
        return DensityType(2, 1.0)

    def _c(self) -> _Density:
        return _Density(self.kind, self.alpha)


@dataclass
class PicardConfig:
    """config.rs:11-62 with the defaults of config.rs:64-85."""

    density: DensityType = field(default_factory=DensityType)
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
    # MI355X additions
    device: int = 0
    want_sources: bool = True

    @staticmethod
    def builder() -> "ConfigBuilder":
        return ConfigBuilder()

    def effective_extended(self) -> bool:
        """config.rs:99-101."""
        return self.ortho if self.extended is None else bool(self.extended)

    def validate(self) -> None:
        """config.rs:104-142 (through the C ABI)."""
        c, _keep = self._c()
        err = _errbuf()
        _raise(lib.pc_config_validate(C.byref(c), err, len(err)), err)

    def _c(self):
        c = _Config()
        lib.pc_config_default(C.byref(c))
        c.density = self.density._c()
        if self.n_components is not None:
            c.has_n_components, c.n_components = 1, int(self.n_components)
        c.ortho = int(bool(self.ortho))
        if self.extended is not None:
            c.has_extended, c.extended = 1, int(bool(self.extended))
        c.whiten = int(bool(self.whiten))
        c.centering = int(bool(self.centering))
        c.max_iter, c.tol, c.m, c.ls_tries = int(self.max_iter), float(self.tol), int(self.m), int(self.ls_tries)
        c.lambda_min = float(self.lambda_min)
        keep = None
        if self.w_init is not None:
            keep = _c64(self.w_init)
            if keep.ndim != 2:
                keep = keep.reshape(keep.shape[0], -1)
            c.w_init, c.w_init_rows, c.w_init_cols = _ptr(keep), keep.shape[0], keep.shape[1]
        if self.fastica_it is not None:
            c.has_fastica_it, c.fastica_it = 1, int(self.fastica_it)
        if self.jade_it is not None:
            c.has_jade_it, c.jade_it = 1, int(self.jade_it)
        if self.random_state is not None:
            c.has_random_state, c.random_state = 1, int(self.random_state)
        c.verbose = int(bool(self.verbose))
        c.device = int(self.device)
        c.want_sources = int(bool(self.want_sources))
        return c, keep


class ConfigBuilder:
    """config.rs:147-273 fluent builder."""

    def __init__(self):
        self.config = PicardConfig()

    def __getattr__(self, name):
        if name in PicardConfig.__dataclass_fields__:
            def setter(value):
                setattr(self.config, name, value)
                return self
            return setter
        raise AttributeError(name)

    def build(self) -> PicardConfig:
        return self.config

    def build_validated(self) -> PicardConfig:
        self.config.validate()
        return self.config


def _arr(p, *shape) -> Optional[np.ndarray]:
    if not p:
        return None
    n = int(np.prod(shape))
    return np.ctypeslib.as_array(p, shape=(n,)).reshape(shape).copy()


@dataclass
class PicardResult:
    """result.rs:7-33 (+ n_evaluations: fused passes issued by core::run)."""

    whitening: Optional[np.ndarray]
    unmixing: np.ndarray
    sources: Optional[np.ndarray]
    mean: Optional[np.ndarray]
    n_iterations: int
    converged: bool
    gradient_norm: float
    signs: Optional[np.ndarray]
    n_evaluations: int = 0

    @staticmethod
    def _from_c(r: _Result) -> "PicardResult":
        return PicardResult(
            whitening=_arr(r.whitening, r.whitening_rows, r.whitening_cols),
            unmixing=_arr(r.unmixing, r.unmixing_rows, r.unmixing_cols),
            sources=_arr(r.sources, r.sources_rows, r.sources_cols),
            mean=_arr(r.mean, r.mean_len),
            n_iterations=int(r.n_iterations),
            converged=bool(r.converged),
            gradient_norm=float(r.gradient_norm),
            signs=_arr(r.signs, r.signs_len),
            n_evaluations=int(r.n_evaluations),
        )

    def _c(self):
        r = _Result()
        keep = []

        def put(name, a):
            if a is not None:
                a = _c64(a)
                keep.append(a)
                setattr(r, name, _ptr(a))
                return a.shape
            return None
        if (s := put("whitening", self.whitening)) is not None:
            r.whitening_rows, r.whitening_cols = s
        s = put("unmixing", self.unmixing)
        r.unmixing_rows, r.unmixing_cols = s
        if (s := put("mean", self.mean)) is not None:
            r.mean_len = s[0]
        return r, keep

    def full_unmixing(self) -> np.ndarray:
        """result.rs:39-44."""
        r, _k = self._c()
        nf = self.whitening.shape[1] if self.whitening is not None else self.unmixing.shape[1]
        out = np.empty((self.unmixing.shape[0], nf))
        lib.pc_full_unmixing(C.byref(r), _ptr(out))
        return out

    def mixing(self) -> np.ndarray:
        """result.rs:49-64."""
        r, _k = self._c()
        nf = self.whitening.shape[1] if self.whitening is not None else self.unmixing.shape[1]
        out = np.empty((nf, self.unmixing.shape[0]))
        lib.pc_mixing(C.byref(r), _ptr(out))
        return out


class Picard:
    """solver.rs:23-215."""

    @staticmethod
    def fit(x) -> PicardResult:
        return Picard.fit_with_config(x, PicardConfig())

    @staticmethod
    def fit_with_config(x, config: PicardConfig) -> PicardResult:
        x = _c64(x)
        if x.ndim != 2:
            raise InvalidDimensions("Invalid dimensions: X must be 2-D (n_features × n_samples)")
        c, _keep = config._c()
        r = _Result()
        err = _errbuf()
        rc = lib.pc_fit(_ptr(x), x.shape[0], x.shape[1], C.byref(c), C.byref(r), err, len(err))
        try:
            _raise(rc, err)
            return PicardResult._from_c(r)
        finally:
            lib.pc_result_free(C.byref(r))

    @staticmethod
    def transform(x, result: PicardResult, device: int = 0) -> np.ndarray:
        x = _c64(x)
        r, _k = result._c()
        out = np.empty((result.unmixing.shape[0], x.shape[1]))
        err = _errbuf()
        _raise(lib.pc_transform(_ptr(x), x.shape[0], x.shape[1], C.byref(r), _ptr(out), device, err, len(err)), err)
        return out


class utils:
    """utils.rs."""

    @staticmethod
    def amari_distance(w, a) -> float:
        w, a = _c64(w), _c64(a)
        return float(lib.pc_amari_distance(_ptr(w), _ptr(a), w.shape[0]))

    @staticmethod
    def permute(a, scale: bool = True) -> np.ndarray:
        a = _c64(a)
        out = np.empty_like(a)
        lib.pc_permute(_ptr(a), a.shape[0], int(scale), _ptr(out))
        return out

# ------------------------------------------------------------------ device level


def device_synchronize(device: int = 0) -> None:
    rc = lib.pc_device_synchronize(device)
    if rc:
        raise ComputationError("hipDeviceSynchronize failed")


def device_mem_info(device: int = 0) -> tuple:
    """pc_device_mem_info: (free, total) HBM bytes of `device`."""
    f, t = C.c_uint64(), C.c_uint64()
    rc = lib.pc_device_mem_info(device, C.byref(f), C.byref(t))
    if rc:
        raise ComputationError("hipMemGetInfo failed")
    return f.value, t.value


def last_teardown() -> dict:
    """pc_last_teardown: the last pc_ctx_destroy's wall ms, ms in hipFree, longest hipFree,
    ms of the closing device synchronisation."""
    o = (C.c_double * 4)()
    lib.pc_last_teardown(o)
    return {"wall_ms": o[0], "free_ms": o[1], "max_free_ms": o[2], "sync_ms": o[3]}


def rccl_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    if lib.pc_rccl_unique_id(buf) != 0:
        raise ComputationError("ncclGetUniqueId failed")
    return buf.raw


class LocalGroup:
    """pc_group: an in-process rank group — `world_size` DeviceContexts in this process,
    one host thread per rank (they may share one GPU), that exchange every pass's
    statistics through host memory (fixed rank-order sum) instead of RCCL. Runs the
    communicator path of bench.py --gpus N (rank-replicated Solver, per-pass
    all-reduce, capability agreements, group abort) on one device."""

    def __init__(self, world_size: int):
        h = C.c_void_p()
        err = _errbuf()
        _raise(lib.pc_group_create_local(world_size, C.byref(h), err, len(err)), err)
        self.h = h
        self.world_size = world_size

    def close(self):
        if self.h:
            lib.pc_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceContext:
    """pc_ctx: one GPU, one contiguous T shard of X resident in HBM. With `group`
    (a LocalGroup) the context is rank `rank` of that in-process group; with
    an `rccl_id` it is one rank of an RCCL communicator (world_size 1 included: a
    one-rank communicator); with world_size > 1 and neither, a detached shard
    (partial sums)."""

    def __init__(self, device: int = 0, rank: int = 0, world_size: int = 1, rccl_id: Optional[bytes] = None,
                 group: Optional[LocalGroup] = None):
        h = C.c_void_p()
        err = _errbuf()
        if group is not None:
            _raise(lib.pc_ctx_create_in_group(device, rank, group.h, C.byref(h), err, len(err)), err)
        else:
            _raise(lib.pc_ctx_create(device, rank, world_size, rccl_id, C.byref(h), err, len(err)), err)
        self.h = h
        self.n_features = 0

    def comm_stats(self) -> dict:
        """pc_ctx_comm_stats: all-reduces issued, capability agreements asked and their outcome."""
        o = (C.c_int64 * 7)()
        lib.pc_ctx_comm_stats(self.h, o)
        return {"allreduces": o[0], "agreements": o[1], "screen_agreed": o[2], "keep_y_agreed": o[3],
                "aborted": bool(o[4]), "world_size": o[5], "kind": {0: None, 1: "rccl", 2: "local"}[o[6]]}

    def comm_timing(self) -> dict:
        """pc_ctx_comm_timing: ms inside all-reduces (RCCL: device time between events around
        each ncclAllReduce, which includes waiting for the slowest rank) and how many."""
        o = (C.c_double * 2)()
        lib.pc_ctx_comm_timing(self.h, o)
        return {"allreduce_ms": o[0], "allreduces_timed": int(o[1])}

    def alloc_stats(self) -> dict:
        """pc_ctx_alloc_stats: ms / count / longest call of hipMalloc, hipFree, hipMemGetInfo."""
        o = (C.c_double * 9)()
        lib.pc_ctx_alloc_stats(self.h, o)
        return {k: {"ms": o[i], "calls": int(o[3 + i]), "max_ms": o[6 + i]}
                for i, k in enumerate(("malloc", "free", "meminfo"))}

    def abort(self, why: str = "aborted by the caller"):
        """pc_ctx_abort: end every rank's pending and later collectives with an error."""
        lib.pc_ctx_abort(self.h, why.encode())

    def release_caches(self):
        """pc_ctx_release_caches: free the int8 digit image and the kept-Y buffer."""
        err = _errbuf()
        _raise(lib.pc_ctx_release_caches(self.h, err, len(err)), err)

    def close(self):
        if self.h:
            lib.pc_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, x_shard, n_total: Optional[int] = None, t0: int = 0):
        x = _c64(x_shard)
        err = _errbuf()
        n_total = x.shape[1] if n_total is None else n_total
        _raise(lib.pc_ctx_load(self.h, _ptr(x), x.shape[0], x.shape[1], n_total, t0, err, len(err)), err)
        self.n_features = x.shape[0]

    def generate(self, n_features: int, n_total: int, seed: int = 42) -> np.ndarray:
        a = np.empty((n_features, n_features))
        err = _errbuf()
        _raise(lib.pc_ctx_generate(self.h, n_features, n_total, seed, _ptr(a), err, len(err)), err)
        self.n_features = n_features
        return a

    @property
    def n_local(self) -> int:
        return int(lib.pc_ctx_n_local(self.h))

    @property
    def t0(self) -> int:
        return int(lib.pc_ctx_t0(self.h))

    def download(self) -> np.ndarray:
        out = np.empty((self.n_features, self.n_local))
        lib.pc_ctx_download(self.h, _ptr(out))
        return out

    def eval(self, w, mu=None, density: DensityType = DensityType(), need_h: bool = False,
             need_y2: bool = True) -> dict:
        """pc_ctx_eval: one fused pass. need_y2=False (PC_EVAL_SKIP_Y2) leaves Σy² at 0
        unless need_h (the orthogonal solver never reads it)."""
        w = _c64(w)
        nc = w.shape[0]
        mu_a = _c64(mu) if mu is not None else None
        n = (2 if need_h else 1) * nc * nc + 3 * nc
        st = np.empty(n)
        err = _errbuf()
        flags = (1 if need_h else 0) | (0 if need_y2 else 2)
        _raise(lib.pc_ctx_eval(self.h, _ptr(w), nc, _ptr(mu_a) if mu_a is not None else None, density._c(),
                               flags, _ptr(st), err, len(err)), err)
        o = nc * nc
        out = {"G": st[:o].reshape(nc, nc)}
        if need_h:
            out["H"] = st[o:2 * o].reshape(nc, nc)
            o *= 2
        out["dpsi"], out["ll"], out["y2"] = st[o:o + nc], st[o + nc:o + 2 * nc], st[o + 2 * nc:o + 3 * nc]
        return out

    @staticmethod
    def _unpack(st, nc, need_h):
        o = nc * nc
        out = {"G": st[:o].reshape(nc, nc)}
        if need_h:
            out["H"] = st[o:2 * o].reshape(nc, nc)
            o *= 2
        out["dpsi"], out["ll"], out["y2"] = st[o:o + nc], st[o + nc:o + 2 * nc], st[o + 2 * nc:o + 3 * nc]
        return out

    def eval_split(self, w, mu=None, density: DensityType = DensityType(), need_h: bool = False,
                   need_y2: bool = True):
        """pc_ctx_eval_loss then pc_ctx_eval_complete; returns (loss-only stats, kept, completed stats)."""
        w = _c64(w)
        nc = w.shape[0]
        mu_a = _c64(mu) if mu is not None else None
        n = (2 if need_h else 1) * nc * nc + 3 * nc
        st = np.full(n, np.nan)
        kept = C.c_int32()
        err = _errbuf()
        flags = (1 if need_h else 0) | (0 if need_y2 else 2)
        _raise(lib.pc_ctx_eval_loss(self.h, _ptr(w), nc, _ptr(mu_a) if mu_a is not None else None, density._c(),
                                    flags, _ptr(st), C.byref(kept), err, len(err)), err)
        loss_only = st.copy()
        if kept.value:
            _raise(lib.pc_ctx_eval_complete(self.h, density._c(), 1 if need_h else 0, _ptr(st), err, len(err)), err)
        return self._unpack(loss_only, nc, need_h), bool(kept.value), self._unpack(st, nc, need_h)

    def eval_loss_multi(self, w, z, alphas, mu=None, density: DensityType = DensityType()):
        """pc_ctx_eval_loss_multi: (Σℓ, Σy²) of (w + α_j·z)(X − μ) for every α_j, each [n_alpha, nc]."""
        w, z = _c64(w), _c64(z)
        nc = w.shape[0]
        al = _c64(np.asarray(alphas, dtype=np.float64).ravel())
        mu_a = _c64(mu) if mu is not None else None
        ll = np.empty((len(al), nc))
        y2 = np.empty((len(al), nc))
        err = _errbuf()
        _raise(lib.pc_ctx_eval_loss_multi(self.h, _ptr(w), _ptr(z), nc, _ptr(mu_a) if mu_a is not None else None,
                                          density._c(), _ptr(al), len(al), _ptr(ll), _ptr(y2), err, len(err)), err)
        return ll, y2

    def eval_loss_multi_bound(self, w, z, alphas, mu=None, density: DensityType = DensityType()):
        """pc_ctx_eval_loss_multi_bound: (Σℓ estimate, bound on its distance to the exact pass)
        of (w + α_j·z)(X − μ) for every α_j, each [n_alpha, nc]."""
        w, z = _c64(w), _c64(z)
        nc = w.shape[0]
        al = _c64(np.asarray(alphas, dtype=np.float64).ravel())
        mu_a = _c64(mu) if mu is not None else None
        ll = np.empty((len(al), nc))
        bnd = np.empty((len(al), nc))
        err = _errbuf()
        _raise(lib.pc_ctx_eval_loss_multi_bound(self.h, _ptr(w), _ptr(z), nc,
                                                _ptr(mu_a) if mu_a is not None else None, density._c(), _ptr(al),
                                                len(al), _ptr(ll), _ptr(bnd), err, len(err)), err)
        return ll, bnd

    def last_timing(self):
        k, c = C.c_double(), C.c_double()
        lib.pc_ctx_last_timing(self.h, C.byref(k), C.byref(c))
        return k.value, c.value

    def kernel_stats(self, reset: bool = False):
        """(Σ fused-kernel ms, Σ eval-call ms, launches) since the last reset (HIP events)."""
        k, c, n = C.c_double(), C.c_double(), C.c_uint64()
        lib.pc_ctx_kernel_stats(self.h, C.byref(k), C.byref(c), C.byref(n), int(reset))
        return k.value, c.value, n.value

    def kernel_breakdown(self, reset: bool = False) -> dict:
        """{kind: (Σ kernel ms, launches)} for kind in fused / loss / fromy / multi (HIP events)."""
        ms = (C.c_double * 4)()
        n = (C.c_uint64 * 4)()
        lib.pc_ctx_kernel_breakdown(self.h, ms, n, int(reset))
        return {k: (ms[i], n[i]) for i, k in enumerate(("fused", "loss", "fromy", "multi"))}

    def set_y_stage(self, mode: str = "auto"):
        """pc_ctx_set_y_stage: "auto" (int8-digit Y stage where the shape allows, line-search
        screen on), "f64", or "int8-exact" (int8 stage, every try evaluated exactly)."""
        _raise(lib.pc_ctx_set_y_stage(self.h, {"auto": 0, "f64": 1, "int8-exact": 2}[mode]), _errbuf())

    def set_g_stage(self, mode: str = "auto"):
        """pc_ctx_set_g_stage: "auto" (G = ψ·Yᵀ on int8 digits where the fused pass runs on the
        int8 Y stage, tanh / exp) or "f64" (G on the fp64 MFMA)."""
        _raise(lib.pc_ctx_set_g_stage(self.h, {"auto": 0, "f64": 1}[mode]), _errbuf())

    @property
    def g8_passes(self) -> int:
        """fused passes whose G stage ran on int8 digits (pc_ctx_g8_passes)."""
        return int(lib.pc_ctx_g8_passes(self.h))

    def matrix_exp(self, a) -> np.ndarray:
        """pc_ctx_matrix_exp: expm(a) on the device with the host matrix_exp's bits (try 1's
        map of an orthogonal line search); raises Unsupported where the device leaves it to the
        host."""
        a = np.ascontiguousarray(a, dtype=np.float64)
        n = a.shape[0]
        out = np.empty((n, n))
        err = _errbuf()
        _raise(lib.pc_ctx_matrix_exp(self.h, _ptr(a), n, _ptr(out), err, len(err)), err)
        return out

    @property
    def multi_ybuf_passes(self) -> int:
        """multi-try passes that read Y from the full pass at the same W (pc_ctx_multi_ybuf_passes)."""
        return int(lib.pc_ctx_multi_ybuf_passes(self.h))

    def eval_loss_screen(self, w, mu=None, density: DensityType = DensityType()):
        """pc_ctx_eval_loss_screen: (Σℓ from the screen, bound on |Σℓ_exact − Σℓ_screen|), each [nc]."""
        w = _c64(w)
        nc = w.shape[0]
        mu_a = _c64(mu) if mu is not None else None
        ll, bnd = np.empty(nc), np.empty(nc)
        err = _errbuf()
        _raise(lib.pc_ctx_eval_loss_screen(self.h, _ptr(w), nc, _ptr(mu_a) if mu_a is not None else None,
                                           density._c(), _ptr(ll), _ptr(bnd), err, len(err)), err)
        return ll, bnd

    def eval_loss_screen2(self, w1, w2, mu=None, density: DensityType = DensityType()):
        """pc_ctx_eval_loss_screen2: two tries in one pass → ((Σℓ, bound) of w1, (Σℓ, bound) of w2),
        each as eval_loss_screen gives it for that W alone."""
        w1, w2 = _c64(w1), _c64(w2)
        nc = w1.shape[0]
        if w2.shape != w1.shape:
            raise InvalidDimensions("eval_loss_screen2: w1 and w2 differ in shape")
        mu_a = _c64(mu) if mu is not None else None
        out = [np.empty(nc) for _ in range(4)]
        err = _errbuf()
        _raise(lib.pc_ctx_eval_loss_screen2(self.h, _ptr(w1), _ptr(w2), nc, _ptr(mu_a) if mu_a is not None else None,
                                            density._c(), *[_ptr(o) for o in out], err, len(err)), err)
        return (out[0], out[1]), (out[2], out[3])

    def screen_tries(self) -> int:
        """pc_ctx_screen_tries: tries the screen passes covered since the last screen_stats reset
        (a paired pass covers 2)."""
        return int(lib.pc_ctx_screen_tries(self.h))

    def screen_products(self) -> int:
        """pc_ctx_screen_products: digit products per try summed over the screened tries since the
        last screen_stats reset (6 for a D ≤ 2 try, 10 for D ≤ 3, 15 for D ≤ 4)."""
        return int(lib.pc_ctx_screen_products(self.h))

    def screen_digit_gram(self):
        """pc_ctx_screen_digit_gram: (lam[7], s4) — the largest-eigenvalue bounds of this shard's
        digit Grams and Σ_t 4^e_t, the inputs of the screen's statistical bound."""
        lam, s4 = np.zeros(7), C.c_double()
        err = _errbuf()
        _raise(lib.pc_ctx_screen_digit_gram(self.h, _ptr(lam), C.byref(s4), err, len(err)), err)
        return lam, s4.value

    def screen_stats(self, reset: bool = False):
        """pc_ctx_screen_stats: (Σ screen-pass kernel ms, screen passes) since the last reset."""
        ms, n = C.c_double(), C.c_uint64()
        lib.pc_ctx_screen_stats(self.h, C.byref(ms), C.byref(n), int(reset))
        return ms.value, n.value

    @property
    def int8_passes(self) -> int:
        """pc_ctx_int8_passes: passes whose Y stage ran on the int8 slices so far."""
        return int(lib.pc_ctx_int8_passes(self.h))

    def rowsum(self) -> np.ndarray:
        out = np.empty(self.n_features)
        err = _errbuf()
        _raise(lib.pc_ctx_rowsum(self.h, _ptr(out), err, len(err)), err)
        return out

    def gram(self, mu=None) -> np.ndarray:
        out = np.empty((self.n_features, self.n_features))
        mu_a = _c64(mu) if mu is not None else None
        err = _errbuf()
        _raise(lib.pc_ctx_gram(self.h, _ptr(mu_a) if mu_a is not None else None, _ptr(out), err, len(err)), err)
        return out

    def sources(self, w, mu=None) -> np.ndarray:
        w = _c64(w)
        out = np.empty((w.shape[0], self.n_local))
        mu_a = _c64(mu) if mu is not None else None
        err = _errbuf()
        _raise(lib.pc_ctx_sources(self.h, _ptr(w), w.shape[0], _ptr(mu_a) if mu_a is not None else None,
                                  _ptr(out), err, len(err)), err)
        return out

    def sources_device(self, w, mu=None):
        """pc_ctx_sources_device: Y = w·(X − μ) kept in HBM. Returns (device pointer,
        leading dimension in doubles, kernel ms); the buffer belongs to the context."""
        w = _c64(w)
        mu_a = _c64(mu) if mu is not None else None
        p, ld, ms = C.c_void_p(), C.c_uint64(), C.c_double()
        err = _errbuf()
        _raise(lib.pc_ctx_sources_device(self.h, _ptr(w), w.shape[0], _ptr(mu_a) if mu_a is not None else None,
                                         C.byref(p), C.byref(ld), C.byref(ms), err, len(err)), err)
        return p.value, ld.value, ms.value

    def jade(self, w, mu=None, max_iter: int = 50, tol: float = 1e-6, where: str = "auto"):
        """pc_ctx_jade: the JADE warm start (jade.rs:22-72) on Y = w·(X − μ).
        Returns (sym_decorrelation(V), sweeps run, tolerance met, sweeps ran on the device)."""
        w = _c64(w)
        nc = w.shape[0]
        mu_a = _c64(mu) if mu is not None else None
        out = np.empty((nc, nc))
        info = (C.c_uint64 * 3)()
        err = _errbuf()
        _raise(lib.pc_ctx_jade(self.h, _ptr(w), nc, _ptr(mu_a) if mu_a is not None else None, max_iter, tol,
                               {"auto": 0, "device": 1, "host": 2}[where], _ptr(out), info, err, len(err)), err)
        return out, int(info[0]), bool(info[1]), bool(info[2])

    def moments4(self, w, mu=None) -> np.ndarray:
        w = _c64(w)
        nc = w.shape[0]
        npair = nc * (nc + 1) // 2
        out = np.empty((npair, npair))
        mu_a = _c64(mu) if mu is not None else None
        err = _errbuf()
        _raise(lib.pc_ctx_moments4(self.h, _ptr(w), nc, _ptr(mu_a) if mu_a is not None else None,
                                   _ptr(out), err, len(err)), err)
        return out


class Solver:
    """pc_solver: fit_with_config split into create / step (one core.rs iteration) / finish."""

    def __init__(self, ctx: DeviceContext, config: PicardConfig):
        c, keep = config._c()
        self._keep = keep
        h = C.c_void_p()
        err = _errbuf()
        _raise(lib.pc_solver_create(ctx.h, C.byref(c), C.byref(h), err, len(err)), err)
        self.h = h
        self.ctx = ctx

    def step(self) -> bool:
        done = C.c_int32()
        err = _errbuf()
        _raise(lib.pc_solver_step(self.h, C.byref(done), err, len(err)), err)
        return bool(done.value)

    def last(self):
        loss, gn, ne = C.c_double(), C.c_double(), C.c_uint64()
        lib.pc_solver_last(self.h, C.byref(loss), C.byref(gn), C.byref(ne))
        return loss.value, gn.value, ne.value

    def setup_timing(self) -> dict:
        """pc_solver_setup_timing: cumulative ms of the setup phases."""
        o = (C.c_double * 5)()
        lib.pc_solver_setup_timing(self.h, o)
        return dict(zip(("rowsum_ms", "gram_ms", "eigh_ms", "w_init_ms", "initial_pass_ms"), list(o)))

    def timing(self) -> dict:
        """pc_solver_timing: the last step's wall / in-pass / host / helper-wait ms."""
        o = (C.c_double * 4)()
        lib.pc_solver_timing(self.h, o)
        return {"step_ms": o[0], "eval_ms": o[1], "host_ms": o[2], "map_wait_ms": o[3]}

    def finish(self) -> PicardResult:
        r = _Result()
        err = _errbuf()
        rc = lib.pc_solver_finish(self.h, C.byref(r), err, len(err))
        try:
            _raise(rc, err)
            return PicardResult._from_c(r)
        finally:
            lib.pc_result_free(C.byref(r))

    def close(self):
        if self.h:
            lib.pc_solver_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fit_with_host_evaluator(n_features: int, n_samples: int, config: PicardConfig, *, rowsum, gram, eval,
                            sources, moments4=None, eval_loss_multi=None, eval_loss_screen=None) -> PicardResult:
    """Run the host driver over Python callbacks (pc_fit_with_evaluator).

    Test hook for the host logic on machines without a GPU, or over detached
    shard contexts on one GPU; the callbacks get numpy arrays and return them
    (see pc_host_evaluator). ``eval_loss_multi(w, z, alphas, mu, density)``
    returns (Σℓ, Σy²), each [n_alpha, nc]; ``eval_loss_screen(w, mu, density)`` returns
    (Σℓ of an approximation, per-row bound on its distance to the exact Σℓ), each [nc]."""
    def _rs(user, out):
        o = np.ctypeslib.as_array(out, shape=(n_features,))
        o[:] = rowsum()
        return 0

    def _gram(user, mu, out):
        m = np.ctypeslib.as_array(mu, shape=(n_features,)).copy() if mu else None
        o = np.ctypeslib.as_array(out, shape=(n_features * n_features,))
        o[:] = np.asarray(gram(m)).reshape(-1)
        return 0

    def _eval(user, w, nc, mu, dens, flags, out):
        W = np.ctypeslib.as_array(w, shape=(nc * n_features,)).reshape(nc, n_features).copy()
        m = np.ctypeslib.as_array(mu, shape=(n_features,)).copy() if mu else None
        need_h = bool(flags & 1)
        st = eval(W, m, DensityType(dens.kind, dens.alpha), need_h)
        parts = [st["G"].reshape(-1)]
        if need_h:
            parts.append(st["H"].reshape(-1))
        parts += [st["dpsi"], st["ll"], st["y2"]]
        flat = np.concatenate(parts)
        o = np.ctypeslib.as_array(out, shape=(flat.size,))
        o[:] = flat
        return 0

    def _src(user, w, nc, mu, out):
        W = np.ctypeslib.as_array(w, shape=(nc * n_features,)).reshape(nc, n_features).copy()
        m = np.ctypeslib.as_array(mu, shape=(n_features,)).copy() if mu else None
        o = np.ctypeslib.as_array(out, shape=(nc * n_samples,))
        o[:] = np.asarray(sources(W, m)).reshape(-1)
        return 0

    def _m4(user, w, nc, mu, out):
        W = np.ctypeslib.as_array(w, shape=(nc * n_features,)).reshape(nc, n_features).copy()
        m = np.ctypeslib.as_array(mu, shape=(n_features,)).copy() if mu else None
        npair = nc * (nc + 1) // 2
        o = np.ctypeslib.as_array(out, shape=(npair * npair,))
        o[:] = np.asarray(moments4(W, m)).reshape(-1)
        return 0

    def _multi(user, w, z, nc, mu, dens, al, na, ll_out, y2_out):
        W = np.ctypeslib.as_array(w, shape=(nc * n_features,)).reshape(nc, n_features).copy()
        Z = np.ctypeslib.as_array(z, shape=(nc * n_features,)).reshape(nc, n_features).copy()
        m = np.ctypeslib.as_array(mu, shape=(n_features,)).copy() if mu else None
        a = np.ctypeslib.as_array(al, shape=(na,)).copy()
        ll, y2 = eval_loss_multi(W, Z, a, m, DensityType(dens.kind, dens.alpha))
        np.ctypeslib.as_array(ll_out, shape=(na * nc,))[:] = np.asarray(ll).reshape(-1)
        np.ctypeslib.as_array(y2_out, shape=(na * nc,))[:] = np.asarray(y2).reshape(-1)
        return 0

    def _screen(user, w, nc, mu, dens, ll_out, bound_out):
        W = np.ctypeslib.as_array(w, shape=(nc * n_features,)).reshape(nc, n_features).copy()
        m = np.ctypeslib.as_array(mu, shape=(n_features,)).copy() if mu else None
        ll, bnd = eval_loss_screen(W, m, DensityType(dens.kind, dens.alpha))
        np.ctypeslib.as_array(ll_out, shape=(nc,))[:] = np.asarray(ll).reshape(-1)
        np.ctypeslib.as_array(bound_out, shape=(nc,))[:] = np.asarray(bnd).reshape(-1)
        return 0

    cbs = (RowsumFn(_rs), GramFn(_gram), EvalFn(_eval), SourcesFn(_src),
           Moments4Fn(_m4) if moments4 is not None else Moments4Fn(),
           MultiFn(_multi) if eval_loss_multi is not None else MultiFn(),
           ScreenFn(_screen) if eval_loss_screen is not None else ScreenFn())
    ev = _HostEvaluator(None, n_features, n_samples, *cbs)
    c, _keep = config._c()
    r = _Result()
    err = _errbuf()
    rc = lib.pc_fit_with_evaluator(C.byref(ev), C.byref(c), C.byref(r), err, len(err))
    try:
        _raise(rc, err)
        return PicardResult._from_c(r)
    finally:
        lib.pc_result_free(C.byref(r))
