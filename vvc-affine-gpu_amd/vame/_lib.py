"""ctypes binding of libvame.so (include/vame.h).  Fails loudly when the
library is missing -- there is no fallback implementation."""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("VAME_LIB", os.path.join(PKG_DIR, "lib", "libvame.so"))

# every symbol include/vame.h declares
EXPORTS = (
    "vame_create", "vame_destroy", "vame_affine_me", "vame_affine_me_poc", "vame_num_ctus",
    "vame_cus_per_ctu", "vame_num_groups", "vame_group_geometry", "vame_lambda", "vame_poc_qp",
    "vame_ref_list", "vame_strerror", "vame_last_hip_error", "vame_version", "vame_set_timing",
    "vame_get_timing", "vame_read_frames", "vame_log_remove_old", "vame_log_write_headers",
    "vame_log_append", "vame_log_file_count", "vame_set_prof", "vame_affine_me_batch",
    "vame_log_writer_create", "vame_log_writer_poc", "vame_log_writer_destroy", "vame_pred_mask",
    "vame_log_writer_refs", "vame_read_frames_range", "vame_count_lines", "vame_read_frames_span",
    "vame_log_writer_set_deferred", "vame_log_writer_num_files", "vame_log_writer_file_name",
    "vame_log_writer_sizes", "vame_log_writer_flush_at", "vame_template_coverage", "vame_pack_records",
    "vame_count_lines_ranges", "vame_set_max_pairs", "vame_get_max_pairs",
)


class VameError(RuntimeError):
    pass


class PocResult(ctypes.Structure):
    _fields_ = [("cost", (ctypes.c_void_p * 4) * 4), ("cpmvs", (ctypes.c_void_p * 4) * 4)]


class PocJob(ctypes.Structure):
    """vame_poc_job (include/vame.h)."""
    _fields_ = [("cur", ctypes.c_void_p), ("refs", ctypes.c_void_p), ("nrefs", ctypes.c_int),
                ("lam", ctypes.c_float), ("out", ctypes.c_void_p)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise VameError(f"libvame.so not built ({LIB_PATH}); run `make` at the repo root")
        L = ctypes.CDLL(LIB_PATH)
        P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.vame_create.argtypes = [ctypes.POINTER(P), I, I, I]
        L.vame_destroy.argtypes = [P]
        L.vame_destroy.restype = None
        L.vame_affine_me.argtypes = [P, P, P, F, I, I, I, P, P, P, P]
        L.vame_affine_me_poc.argtypes = [P, P, P, I, F, I, I, ctypes.POINTER(PocResult), P]
        L.vame_affine_me_batch.argtypes = [P, ctypes.POINTER(PocJob), I, I, I, P]
        L.vame_pack_records.argtypes = [P, ctypes.POINTER(PocJob), I, I, P, ctypes.c_longlong, P, P]
        L.vame_num_ctus.argtypes = [I, I]
        L.vame_cus_per_ctu.argtypes = [I]
        L.vame_num_groups.argtypes = [I]
        L.vame_group_geometry.argtypes = [I, I, P, P, P, P, P, P]
        L.vame_lambda.argtypes = [I, I]
        L.vame_lambda.restype = F
        L.vame_poc_qp.argtypes = [I, I]
        L.vame_ref_list.argtypes = [I, P]
        L.vame_strerror.argtypes = [I]
        L.vame_strerror.restype = ctypes.c_char_p
        L.vame_last_hip_error.restype = ctypes.c_char_p
        L.vame_version.restype = ctypes.c_char_p
        L.vame_set_timing.argtypes = [P, I]
        L.vame_set_prof.argtypes = [P, I]
        L.vame_set_max_pairs.argtypes = [P, I]
        L.vame_get_max_pairs.argtypes = [P]
        L.vame_get_timing.argtypes = [P, I, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_int), I]
        C = ctypes.c_char_p
        L.vame_read_frames.argtypes = [C, I, I, I, P, I]
        L.vame_read_frames_range.argtypes = [C, I, I, I, I, P, I]
        LL = ctypes.c_longlong
        L.vame_count_lines.argtypes = [C, LL, LL, I]
        L.vame_count_lines.restype = LL
        L.vame_count_lines_ranges.argtypes = [C, P, P, I, P, I]
        L.vame_read_frames_span.argtypes = [C, I, I, I, I, LL, LL, LL, P, I]
        L.vame_log_remove_old.argtypes = [C]
        L.vame_log_write_headers.argtypes = [C, I]
        L.vame_log_append.argtypes = [C, I, I, I, I, I, P, P, I]
        L.vame_log_append.restype = ctypes.c_longlong
        L.vame_log_file_count.argtypes = [I]
        L.vame_log_writer_create.argtypes = [C, I, I, I]
        L.vame_log_writer_create.restype = P
        L.vame_log_writer_poc.argtypes = [P, I, I, I, P, P]
        L.vame_log_writer_poc.restype = ctypes.c_longlong
        L.vame_log_writer_refs.argtypes = [P, I, I, I, I, P, P]
        L.vame_log_writer_refs.restype = ctypes.c_longlong
        L.vame_log_writer_destroy.argtypes = [P]
        L.vame_log_writer_set_deferred.argtypes = [P, I]
        L.vame_log_writer_num_files.argtypes = [P]
        L.vame_log_writer_file_name.argtypes = [P, I, ctypes.c_char_p, I]
        L.vame_log_writer_sizes.argtypes = [P, P]
        L.vame_log_writer_flush_at.argtypes = [P, P]
        L.vame_log_writer_flush_at.restype = ctypes.c_longlong
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != 0:
        L = lib()
        raise VameError(f"vame error {rc}: {L.vame_strerror(rc).decode()} "
                        f"{L.vame_last_hip_error().decode()}")
