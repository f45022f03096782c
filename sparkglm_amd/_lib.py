"""ctypes binding of libsglm_hip.so (the C ABI declared in include/sglm.h).

The library is built in-tree (sparkglm_amd/lib/) by ``make -C sparkglm_amd/csrc`` or
``__graft_entry__.build()``.  There is no fallback: if the HIP library is missing the
import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# SGLM_LIB selects another in-tree build of the same library (A/B kernel comparisons in tools/)
LIB_PATH = os.environ.get("SGLM_LIB") or os.path.join(HERE, "lib", "libsglm_hip.so")

SGLM_OK, SGLM_EINVAL, SGLM_ESINGULAR, SGLM_EHIP, SGLM_ECOMM, SGLM_ENOMEM = range(6)
FAMILIES = {"binomial": 0, "gaussian": 1, "poisson": 2, "gamma": 3}
LINKS = {"logit": 0, "probit": 1, "cloglog": 2, "identity": 3, "log": 4, "inverse": 5}
CANONICAL_LINK = {"gaussian": "identity", "poisson": "log", "gamma": "inverse"}
INIT_SINGLE, INIT_MULTIPLE = 0, 1
NS = 8
S_DEV, S_PEARSON, S_LL, S_BAD, S_AUX0, S_AUX1, S_AUX2, S_SUMW = range(8)

# Symbols include/sglm.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "sglm_abi_version", "sglm_last_error", "sglm_device_count", "sglm_create", "sglm_destroy",
    "sglm_set_data", "sglm_set_data_device", "sglm_synth", "sglm_synth_procedural", "sglm_get_data", "sglm_set_comm",
    "sglm_rccl_unique_id", "sglm_set_comm_rccl", "sglm_fit_glm", "sglm_fit_lm", "sglm_irls_pass", "sglm_irls_step",
    "sglm_irls_iterations", "sglm_predict", "sglm_get_stats", "sglm_reset_stats",
    "sglm_fit_glm_external", "sglm_fit_lm_external", "sglm_glm_create_obj", "sglm_glm_summary",
    "sglm_lm_summary", "sglm_sig_digits", "sglm_round_digits", "sglm_java_double_string",
    "sglm_pval_normal", "sglm_pval_t", "sglm_create_device", "sglm_create_multi", "sglm_handle_devices", "sglm_reserve", "sglm_set_rows",
    "sglm_predict_glm", "sglm_predict_new", "sglm_local_comm_create", "sglm_local_comm_destroy",
    "sglm_local_comm_rank", "sglm_local_allreduce", "sglm_set_comm_rank", "sglm_pass_kernel_for",
]
PREDICT_LINK, PREDICT_RESPONSE = 0, 1

dp = C.POINTER(C.c_double)


class GlmOpts(C.Structure):
    _fields_ = [("family", C.c_int), ("link", C.c_int), ("tol", C.c_double), ("verbose", C.c_int),
                ("max_iter", C.c_int), ("init_mode", C.c_int), ("npart", C.c_int)]


class PreGLM(C.Structure):
    _fields_ = [("coefs", dp), ("std_err", dp), ("deviance", C.c_double), ("null_deviance", C.c_double),
                ("pearson", C.c_double), ("loglik", C.c_double), ("iter", C.c_int), ("nrow", C.c_double),
                ("npart", C.c_int), ("dev_trace", dp), ("max_trace", C.c_int)]


class PreLM(C.Structure):
    _fields_ = [("coefs", dp), ("xtxi", dp), ("std_err", dp), ("sse", C.c_double), ("r2", C.c_double),
                ("fstat", C.c_double), ("sigma", C.c_double), ("nrow", C.c_double), ("npart", C.c_int)]


class Stats(C.Structure):
    _fields_ = [("passes", C.c_int64), ("pass_kernel_ms", C.c_double), ("reduce_kernel_ms", C.c_double),
                ("last_pass_ms", C.c_double), ("comm_ms", C.c_double), ("solve_ms", C.c_double),
                ("n_local", C.c_int64), ("p", C.c_int64), ("workgroups", C.c_int), ("kernel_variant", C.c_int),
                ("path", C.c_int), ("wide_panels", C.c_int), ("row_kernel_ms", C.c_double),
                ("gram_kernel_ms", C.c_double), ("load_ms", C.c_double), ("load_bytes", C.c_int64),
                ("ndev", C.c_int), ("rccl_group", C.c_int), ("dev_passes", C.c_int64),
                ("overlap_chunks", C.c_int), ("comm_path", C.c_int), ("rank_blocks", C.c_int),
                ("pass_kernel_ms_min", C.c_double), ("proc_chunks", C.c_int), ("proc_chunk_rows", C.c_int64),
                ("solve_path", C.c_int), ("pass_kernel", C.c_int), ("pass_kernel_name", C.c_char * 64),
                ("lm_device_fits", C.c_int64), ("lm_device_reruns", C.c_int64),
                ("lm_onepass_fits", C.c_int64)]


COMM_PATHS = {0: "none", 1: "caller-host", 2: "caller-device", 3: "rccl", 4: "group-rccl", 5: "group-host"}
SOLVE_PATHS = {-1: "none", 0: "host-cholesky", 1: "host-lu", 2: "device-cholesky", 3: "device-lu"}
PASS_KERNELS = {0: "none", 1: "fused", 2: "fused-split", 3: "narrow", 4: "wide", 5: "wide-procedural"}


class GlmDerived(C.Structure):
    _fields_ = [("df_residual", C.c_double), ("df_null", C.c_double), ("p_dispersion", C.c_double),
                ("aic", C.c_double)]


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, dp, C.c_int64, C.c_void_p, C.c_int)
LOCAL_SUMS_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, dp)
PASS_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, dp, C.c_double, C.c_double, dp)


class Backend(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("p", C.c_int64), ("local_sums", LOCAL_SUMS_FN), ("pass_", PASS_FN)]


class SGLMError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[sglm status {code}] {msg}")
        self.code = code


class CommError(SGLMError):
    """SGLM_ECOMM: the all-reduce failed -- RCCL or caller error, or no completion within
    SGLM_COMM_TIMEOUT_S (a peer rank died or stalled); the message names the rank."""


class IllegalArgumentException(ValueError):
    """The reference's require(...) failures (java.lang.IllegalArgumentException)."""


class MatrixSingularException(ArithmeticError):
    """breeze.linalg.MatrixSingularException raised by inv()."""


_lib = None


def load():
    """Load the in-tree HIP library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"sparkglm_amd: HIP engine library missing at {LIB_PATH}; "
                          f"build it with `make -C sparkglm_amd/csrc` (or __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    E = C.POINTER(C.c_void_p)
    h = C.c_void_p
    sig = {
        "sglm_abi_version": ([], C.c_int),
        "sglm_last_error": ([], C.c_char_p),
        "sglm_device_count": ([C.POINTER(C.c_int)], C.c_int),
        "sglm_create": ([C.POINTER(C.c_int), C.c_int, E], C.c_int),
        "sglm_create_device": ([C.c_int, E], C.c_int),
        "sglm_create_multi": ([C.POINTER(C.c_int), C.c_int, E], C.c_int),
        "sglm_destroy": ([h], None),
        "sglm_set_data": ([h, dp, C.c_int64, C.c_int64, C.c_int64, dp, dp, dp, dp], C.c_int),
        "sglm_set_data_device": ([h, C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_void_p], C.c_int),
        "sglm_synth": ([h, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_uint64], C.c_int),
        "sglm_synth_procedural": ([h, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_uint64], C.c_int),
        "sglm_get_data": ([h, dp, dp, dp, dp, dp], C.c_int),
        "sglm_set_comm": ([h, ALLREDUCE_FN, C.c_void_p, C.c_int], C.c_int),
        "sglm_set_comm_rank": ([h, C.c_int], C.c_int),
        "sglm_rccl_unique_id": ([C.c_void_p], C.c_int),
        "sglm_set_comm_rccl": ([h, C.c_int, C.c_int, C.c_void_p], C.c_int),
        "sglm_fit_glm": ([h, C.POINTER(GlmOpts), C.POINTER(PreGLM)], C.c_int),
        "sglm_fit_lm": ([h, C.POINTER(PreLM)], C.c_int),
        "sglm_irls_pass": ([h, C.POINTER(GlmOpts), dp, C.c_double, dp, dp, dp], C.c_int),
        "sglm_irls_step": ([h, C.POINTER(GlmOpts), dp, dp, dp, dp], C.c_int),
        "sglm_irls_iterations": ([h, C.POINTER(GlmOpts), dp, C.c_int, dp], C.c_int),
        "sglm_predict": ([h, dp, C.c_int, dp], C.c_int),
        "sglm_get_stats": ([h, C.POINTER(Stats)], C.c_int),
        "sglm_reset_stats": ([h], C.c_int),
        "sglm_fit_glm_external": ([C.POINTER(Backend), ALLREDUCE_FN, C.c_void_p, C.POINTER(GlmOpts),
                                   C.POINTER(PreGLM)], C.c_int),
        "sglm_fit_lm_external": ([C.POINTER(Backend), ALLREDUCE_FN, C.c_void_p, C.POINTER(PreLM)], C.c_int),
        "sglm_glm_create_obj": ([C.POINTER(PreGLM), C.c_int64, C.POINTER(GlmDerived)], C.c_int),
        "sglm_glm_summary": ([C.POINTER(PreGLM), C.c_int64, C.POINTER(C.c_char_p), C.c_char_p, C.c_char_p,
                              C.c_char_p, C.c_char_p, C.c_int64], C.c_int64),
        "sglm_lm_summary": ([C.POINTER(PreLM), C.c_int64, C.POINTER(C.c_char_p), C.c_char_p, C.c_char_p,
                             C.c_int64], C.c_int64),
        "sglm_sig_digits": ([C.c_double, C.c_int], C.c_double),
        "sglm_round_digits": ([C.c_double, C.c_int], C.c_double),
        "sglm_java_double_string": ([C.c_double, C.c_char_p, C.c_int64], C.c_int64),
        "sglm_pval_normal": ([C.c_double], C.c_double),
        "sglm_pval_t": ([C.c_double, C.c_double], C.c_double),
        "sglm_handle_devices": ([h, C.POINTER(C.c_int)], C.c_int),
        "sglm_reserve": ([h, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int], C.c_int),
        "sglm_set_rows": ([h, C.c_int64, C.c_int64, dp, C.c_int64, dp, dp, dp, dp], C.c_int),
        "sglm_predict_glm": ([h, dp, C.c_int, C.c_int, C.c_int, C.c_int, dp], C.c_int),
        "sglm_predict_new": ([h, dp, C.c_int64, C.c_int64, C.c_int64, dp, dp, dp, C.c_int, C.c_int, C.c_int, dp],
                             C.c_int),
        "sglm_local_comm_create": ([C.c_int, C.POINTER(C.c_void_p)], C.c_int),
        "sglm_local_comm_destroy": ([C.c_void_p], None),
        "sglm_local_comm_rank": ([C.c_void_p, C.c_int], C.c_void_p),
        "sglm_local_allreduce": ([C.c_void_p, dp, C.c_int64, C.c_void_p, C.c_int], C.c_int),
        "sglm_pass_kernel_for": ([C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_int64],
                                 C.c_int),
    }
    for name, (args, res) in sig.items():
        if os.environ.get("SGLM_LIB") and not hasattr(lib, name):
            continue  # an older build under A/B comparison (tools/ab.py)
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    _lib = lib
    return lib


def pass_kernel_for(n: int, p: int, family: str = "binomial", link: str = "logit", fused_split: int = 1,
                    procedural: bool = False, force_wide: bool = False):
    """(kind, name) of the kernel an engine runs an n x p pass with (sglm_pass_kernel_for; no GPU)."""
    buf = C.create_string_buffer(64)
    flags = (1 if procedural else 0) | (2 if force_wide else 0)
    k = load().sglm_pass_kernel_for(int(n), int(p), int(fused_split), flags, FAMILIES[family], LINKS[link], buf, 64)
    if k < 0:
        raise IllegalArgumentException(last_error())
    return PASS_KERNELS[k], buf.value.decode()


def last_error() -> str:
    return (load().sglm_last_error() or b"").decode()


def check(rc: int, what: str = "") -> None:
    if rc == SGLM_OK:
        return
    msg = last_error()
    if rc == SGLM_EINVAL:
        raise IllegalArgumentException(msg)
    if rc == SGLM_ESINGULAR:
        raise MatrixSingularException(msg)
    if rc == SGLM_ECOMM:
        raise CommError(rc, f"{what}: {msg}" if what else msg)
    raise SGLMError(rc, f"{what}: {msg}" if what else msg)


def ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(dp)


def java_double_str(x: float) -> str:
    buf = C.create_string_buffer(64)
    load().sglm_java_double_string(float(x), buf, 64)
    return buf.value.decode()
