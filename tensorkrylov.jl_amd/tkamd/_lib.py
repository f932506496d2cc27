"""ctypes binding of libtkhip.so (include/tk.h).

The product path has exactly one implementation of the hot path: the HIP kernels in
libtkhip.so.  There is no CPU fallback -- if the library is missing or no gfx950
device is visible, every entry point raises TKError.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TKHIP_LIB", os.path.join(_HERE, "libtkhip.so"))

TK_ARNOLDI, TK_LANCZOS, TK_LANCZOS_REORTH = 0, 1, 2

# timing classes (tk_abi.cpp TCLS_*)
T_STEP, T_PASS1, T_PASS2, T_FIN, T_RED, T_VY, T_XCH, T_SWEEP, T_GRAM = 0, 1, 2, 3, 4, 5, 6, 7, 8


class TKError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libtkhip.so once; raise loudly if it is absent (no fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise TKError("libtkhip.so not found at %s -- run __graft_entry__.build() "
                      "(the HIP extension is required; there is no CPU fallback)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    P = ctypes.c_void_p
    I = ctypes.c_int
    I64 = ctypes.c_int64
    DP = ctypes.POINTER(ctypes.c_double)
    sigs = {
        "tk_last_error": (ctypes.c_char_p, []),
        "tk_version": (I, []),
        "tk_reduce_handoff": (I, []),
        "tk_reduce_check_ms": (ctypes.c_double, []),
        "tk_ctx_create": (I, [I, ctypes.POINTER(P)]),
        "tk_ctx_destroy": (I, [P]),
        "tk_ctx_sync": (I, [P]),
        "tk_comm_unique_id": (I, [ctypes.c_char_p]),
        "tk_comm_init": (I, [P, ctypes.c_char_p, I, I]),
        "tk_comm_allreduce_host": (I, [P, DP, ctypes.c_size_t]),
        "tk_comm_count": (I, [P, ctypes.POINTER(I)]),
        "tk_matrix_from_csc": (I, [P, I64, ctypes.POINTER(I64), ctypes.POINTER(I64), DP, I, ctypes.POINTER(P)]),
        "tk_matrix_from_csr": (I, [P, I64, ctypes.POINTER(I64), ctypes.POINTER(I64), DP, I, ctypes.POINTER(P)]),
        "tk_matrix_destroy": (I, [P]),
        "tk_matvec": (I, [P, DP, DP]),
        "tk_matrix_format": (I, [P]),
        "tk_record_len": (I, [I]),
        "tk_decomp_create": (I, [P, I, I, I, I, ctypes.POINTER(P), ctypes.POINTER(DP), I64, I, I, ctypes.POINTER(P)]),
        "tk_decomp_destroy": (I, [P]),
        "tk_decomp_arnoldi_sweeps": (I, [P]),
        "tk_decomp_exchange_signalled": (I, [P]),
        "tk_decomp_set_replica": (I, [P, I]),
        "tk_decomp_agree": (I, [P, ctypes.POINTER(I), I]),
        "tk_decomp_next_step": (I, [P]),
        "tk_decomp_matrix_reads": (I, [P]),
        "tk_decomp_gram_deferred": (I, [P]),
        "tk_decomp_factor_groups": (I, [P]),
        "tk_decomp_single_columns": (I, [P]),
        "tk_decomp_gram": (I, [P, I, I, DP]),
        "tk_decomp_gram_ahead": (I, [P, ctypes.POINTER(I)]),
        "tk_decomp_init": (I, [P, DP]),
        "tk_decomp_step": (I, [P, I, DP]),
        "tk_decomp_sweep": (I, [P, I, I]),
        "tk_decomp_flush": (I, [P, DP]),
        "tk_decomp_records": (I, [P, I, I, DP]),
        "tk_decomp_get_basis": (I, [P, I, I, I, DP]),
        "tk_decomp_basis_mul": (I, [P, I, I, DP, DP]),
        "tk_timing_enable": (I, [P, I]),
        "tk_timing_read": (I, [P, I, DP, ctypes.POINTER(ctypes.c_long)]),
        "tk_compressed_solve": (I, [I, I, DP, I, DP, I, DP, DP, ctypes.c_double, DP, DP]),
        "tk_residualnorm": (I, [I, I, I, DP, DP, DP, DP, DP, ctypes.c_double, DP, DP]),
        "tk_solver_create": (I, [I, I, I, I, ctypes.c_double, DP, ctypes.POINTER(I), DP, DP, ctypes.POINTER(P)]),
        "tk_solver_destroy": (I, [P]),
        "tk_solver_overlay": (I, [P, I, I, DP]),
        "tk_solver_apply": (I, [P, I, DP]),
        "tk_solver_evaluate": (I, [P, I, DP]),
        "tk_solver_rank": (I, [P, I]),
        "tk_solver_solution": (I, [P, I, DP, DP]),
        "tk_solver_state": (I, [P, DP, DP, DP]),
        "tk_solver_run": (I, [P, P, ctypes.c_double, I, I, I, DP, DP, DP, ctypes.POINTER(I), ctypes.POINTER(I)]),
        "tk_solver_prepare": (I, [P, I]),
        "tk_solver_share": (I, [P, ctypes.c_char_p, I, I]),
        "tk_solver_share_emulated": (I, [P, I, I, DP]),
        "tk_solver_results": (I, [P, DP]),
        "tk_solver_evaluate_shared": (I, [P, I, DP]),
        "tk_orthogonality_losses": (I, [I, DP, DP]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


# every symbol include/tk.h declares (tests check the .so exports all of them)
EXPORTS = ("tk_last_error", "tk_version", "tk_reduce_handoff", "tk_reduce_check_ms", "tk_ctx_create", "tk_ctx_destroy", "tk_ctx_sync",
           "tk_comm_unique_id", "tk_comm_init", "tk_comm_allreduce_host", "tk_comm_count",
           "tk_matrix_from_csc", "tk_matrix_from_csr", "tk_matrix_destroy", "tk_matrix_format", "tk_matvec",
           "tk_record_len", "tk_decomp_create", "tk_decomp_destroy", "tk_decomp_arnoldi_sweeps",
           "tk_decomp_exchange_signalled", "tk_decomp_set_replica", "tk_decomp_agree", "tk_decomp_next_step",
           "tk_decomp_matrix_reads", "tk_decomp_gram_deferred", "tk_decomp_factor_groups", "tk_decomp_single_columns", "tk_decomp_gram", "tk_decomp_gram_ahead",
           "tk_decomp_init",
           "tk_decomp_step", "tk_decomp_sweep", "tk_decomp_flush", "tk_decomp_records",
           "tk_decomp_get_basis", "tk_decomp_basis_mul", "tk_timing_enable", "tk_timing_read",
           "tk_compressed_solve", "tk_residualnorm", "tk_solver_create", "tk_solver_destroy", "tk_solver_overlay",
           "tk_solver_apply", "tk_solver_evaluate", "tk_solver_rank", "tk_solver_solution", "tk_solver_state",
           "tk_solver_run", "tk_solver_prepare", "tk_solver_share", "tk_solver_share_emulated", "tk_solver_results",
           "tk_solver_evaluate_shared", "tk_orthogonality_losses")

TK_BREAKDOWN = 7


def check(status):
    if status != 0:
        msg = lib().tk_last_error().decode(errors="replace")
        raise TKError("libtkhip error %d: %s" % (status, msg))


def dptr(a):
    """ctypes double* of a C-contiguous float64 array (or None)."""
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def i64ptr(a):
    assert a.dtype == np.int64 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


def record_len(kmax):
    return 2 * kmax + 10


class RecordLayout:
    """Field offsets of one factor's record (include/tk.h)."""

    def __init__(self, kmax):
        self.kmax = kmax
        self.m = record_len(kmax)
        self.H = 0
        self.gram = kmax + 2
        self.bt = 2 * kmax + 4
        self.col = 2 * kmax + 5
        self.beta = 2 * kmax + 6
        self.loss = 2 * kmax + 7
        self.flag = 2 * kmax + 8
        self.tracked = 2 * kmax + 9
