"""ctypes binding of libmlffpcg.so (include/mlffpcg.h).

The library is the only compute path: if it is missing or fails to load this
module raises, there is no NumPy fallback.  Error codes are mapped back onto the
exception types the reference raises at the same places:

  MLFF_ERR_NOT_PSD  -> AssertionError      (incomplete_cholesky.py:62 `assert pivot_element > 0`)
  MLFF_ERR_LINALG   -> numpy.linalg.LinAlgError   (scipy cho_factor / cholesky)
  MLFF_ERR_ARG      -> ValueError
  others            -> RuntimeError
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

PKG_ROOT = Path(__file__).resolve().parent.parent
LIB_PATH = Path(os.environ.get("MLFF_PCG_LIB", PKG_ROOT / "lib" / "libmlffpcg.so"))

MLFF_OK = 0
MLFF_ERR_ARG = -1
MLFF_ERR_HIP = -2
MLFF_ERR_NOT_PSD = -3
MLFF_ERR_LINALG = -4
MLFF_ERR_STATE = -5
MLFF_ERR_COMM = -6
MLFF_ERR_NOMEM = -7

PRECON_NONE, PRECON_PIVCHOL, PRECON_NYSTROM, PRECON_NYSTROM_SB, PRECON_LOWRANK, PRECON_EIG = range(6)
PCG_RUNNING, PCG_CONVERGED, PCG_MAXITER = 0, 2, 3
STORAGE_DENSE, STORAGE_SYMTILE, STORAGE_AUTO, STORAGE_MATFREE = 0, 1, 2, 3

# every symbol declared in include/mlffpcg.h with its ctypes signature
_c_ctx = ctypes.c_void_p
_p_dbl = ctypes.POINTER(ctypes.c_double)
_p_i64 = ctypes.POINTER(ctypes.c_int64)
_p_i32 = ctypes.POINTER(ctypes.c_int32)
_p_int = ctypes.POINTER(ctypes.c_int)
_i64 = ctypes.c_int64
_int = ctypes.c_int
_dbl = ctypes.c_double

SIGNATURES = {
    "mlff_version": (_int, []),
    "mlff_build_hash": (ctypes.c_char_p, []),
    "mlff_device_count": (_int, [_p_int]),
    "mlff_comm_unique_id": (_int, [ctypes.c_char_p]),
    "mlff_comm_selftest": (_int, [_int, _i64, ctypes.POINTER(ctypes.c_double)]),
    "mlff_ctx_create": (_int, [_int, _int, _int, ctypes.c_char_p, _i64, ctypes.POINTER(_c_ctx)]),
    "mlff_ctx_destroy": (_int, [_c_ctx]),
    "mlff_last_error": (ctypes.c_char_p, [_c_ctx]),
    "mlff_shard_range": (_int, [_c_ctx, _p_i64, _p_i64]),
    "mlff_comm_abort": (_int, [_c_ctx]),
    "mlff_matrix_ld": (_int, [_c_ctx, _p_i64]),
    "mlff_synchronize": (_int, [_c_ctx]),
    "mlff_stream": (_int, [_c_ctx, ctypes.POINTER(ctypes.c_void_p)]),
    "mlff_set_matrix_host": (_int, [_c_ctx, _p_dbl, _i64]),
    "mlff_get_matrix_rows": (_int, [_c_ctx, _i64, _i64, _p_dbl, _i64]),
    "mlff_gen_rbf": (_int, [_c_ctx, _p_dbl, _int, _dbl, _dbl]),
    "mlff_assemble_sgdml": (_int, [_c_ctx, _p_dbl, _p_dbl, _i64, _int, _p_i32, _int, _dbl]),
    "mlff_sgdml_operator": (_int, [_c_ctx, _p_dbl, _p_dbl, _i64, _int, _p_i32, _int, _dbl]),
    "mlff_set_energy_constraints": (_int, [_c_ctx, _int]),
    "mlff_spectrum": (_int, [_c_ctx, _int, _p_dbl]),
    "mlff_test_gemm": (_int, [_c_ctx, _int, _int, _i64, _i64, _i64, _dbl, _p_dbl, _i64, _p_dbl,
                              _i64, _dbl, _p_dbl, _i64, _int]),
    "mlff_test_gram": (_int, [_c_ctx, _p_dbl, _i64, _i64, _int, _p_dbl]),
    "mlff_sgdml_energies": (_int, [_c_ctx, _p_dbl, _p_dbl, _p_i64, _p_i64]),
    "mlff_sgdml_descriptors": (_int, [_p_dbl, _i64, _int, _p_dbl, _p_dbl]),
    "mlff_set_operator": (_int, [_c_ctx, _dbl, _dbl]),
    "mlff_matvec": (_int, [_c_ctx, _p_dbl, _p_dbl]),
    "mlff_get_diag": (_int, [_c_ctx, _p_dbl]),
    "mlff_set_storage": (_int, [_c_ctx, _int]),
    "mlff_storage_info": (_int, [_c_ctx, _p_int, _p_dbl]),
    "mlff_operator_form": (_int, [_c_ctx, _p_int]),
    "mlff_precon_none": (_int, [_c_ctx]),
    "mlff_precon_pivchol": (_int, [_c_ctx, _i64, _int, _p_i64, _p_dbl]),
    "mlff_precon_nystrom": (_int, [_c_ctx, _p_i64, _i64, _int, _p_dbl]),
    "mlff_pivchol_times": (_int, [_c_ctx, _p_dbl, _i64, _p_dbl]),
    "mlff_precon_lowrank": (_int, [_c_ctx, _p_dbl, _i64]),
    "mlff_precon_eig": (_int, [_c_ctx, _i64, _int, _i64, _int, _p_dbl, _p_dbl]),
    "mlff_precon_info": (_int, [_c_ctx, _p_int, _p_i64]),
    "mlff_precon_apply_traffic": (_int, [_c_ctx, _p_int, _p_dbl]),
    "mlff_precon_apply": (_int, [_c_ctx, _p_dbl, _p_dbl]),
    "mlff_precon_get_panel": (_int, [_c_ctx, _p_dbl, _i64]),
    "mlff_lev_scores": (_int, [_c_ctx, _p_i64, _i64, _dbl, _p_dbl]),
    "mlff_eig_info": (_int, [_c_ctx, _p_int, _p_dbl]),
    "mlff_cho_factor_stable": (_int, [_c_ctx, _p_dbl, _i64, _p_dbl, _p_dbl]),
    "mlff_sym_min_eig": (_int, [_c_ctx, _p_dbl, _i64, _p_dbl, _p_dbl, _p_dbl]),
    "mlff_pcg_start": (_int, [_c_ctx, _p_dbl, _p_dbl, _dbl, _i64, _p_int]),
    "mlff_pcg_run": (_int, [_c_ctx, _i64, _i64, _p_int]),
    "mlff_pcg_result": (_int, [_c_ctx, _p_i64, _p_int, _p_dbl, _p_int]),
    "mlff_pcg_get_x": (_int, [_c_ctx, _p_dbl]),
    "mlff_pcg_get_trace": (_int, [_c_ctx, _p_dbl, _i64]),
    "mlff_timing_enable": (_int, [_c_ctx, _int]),
    "mlff_timing_read": (_int, [_c_ctx, _p_dbl, _p_i64, _p_dbl, _p_i64]),
    "mlff_timing_reset": (_int, [_c_ctx]),
    "mlff_timing_read_precon": (_int, [_c_ctx, _p_dbl, _p_i64]),
    "mlff_timing_read_comm": (_int, [_c_ctx, _p_dbl, _p_i64]),
    "mlff_device_memory": (_int, [_c_ctx, _p_i64, _p_i64]),
}

_lib = None


def load_library(path: str | os.PathLike | None = None):
    """Load libmlffpcg.so once.  torch (if importable) is imported first so that
    its bundled HIP runtime and ours resolve to the same loaded libamdhip64."""
    global _lib
    if _lib is not None:
        return _lib
    try:  # pragma: no cover - depends on the environment
        import torch  # noqa: F401
    except Exception:
        pass
    # MLFF_LIB: an alternative build of the same library (kernel A/B experiments)
    p = Path(path) if path is not None else Path(os.environ.get("MLFF_LIB") or LIB_PATH)
    if not p.exists():
        raise ImportError(
            f"libmlffpcg.so not found at {p}: build it with "
            "`python mlff-preconditioner_amd/build_native.py` (no CPU fallback exists)")
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error(ctx=None) -> str:
    lib = load_library()
    msg = lib.mlff_last_error(ctx)
    return msg.decode() if msg else ""


def check(rc: int, ctx=None, what: str = ""):
    if rc == MLFF_OK:
        return
    msg = f"{what}: {last_error(ctx)}" if what else last_error(ctx)
    if rc == MLFF_ERR_NOT_PSD:
        raise AssertionError(msg)
    if rc == MLFF_ERR_LINALG:
        raise np.linalg.LinAlgError(msg)
    if rc == MLFF_ERR_ARG:
        raise ValueError(msg)
    raise RuntimeError(f"libmlffpcg error {rc}: {msg}")


def dptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_p_dbl)


def i64ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.int64 and a.flags.c_contiguous
    return a.ctypes.data_as(_p_i64)


def i32ptr(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_p_i32)


def build_hash() -> str:
    """The source hash compiled into the loaded library (build_native.src_hash at build time)."""
    return load_library().mlff_build_hash().decode()


def device_count() -> int:
    lib = load_library()
    n = ctypes.c_int(0)
    rc = lib.mlff_device_count(ctypes.byref(n))
    return n.value if rc == MLFF_OK else 0


def comm_unique_id() -> bytes:
    lib = load_library()
    buf = ctypes.create_string_buffer(128)
    check(lib.mlff_comm_unique_id(buf), None, "mlff_comm_unique_id")
    return buf.raw


def comm_selftest(device: int = 0, count: int = 1 << 20) -> float:
    """RCCL transport self-test on a one-rank communicator (include/mlffpcg.h)."""
    lib = load_library()
    err = ctypes.c_double(-1.0)
    check(lib.mlff_comm_selftest(int(device), int(count), ctypes.byref(err)), None, "mlff_comm_selftest")
    return err.value
