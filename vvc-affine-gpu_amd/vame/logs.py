"""Host I/O contracts of the reference's ./main, through libvame.so:
frame ingest (main.cpp:293-330) and the per-CU decision log
(main_aux_functions.h:387-525, 1547-1585).  Native and multi-threaded
(csrc/vame_io.cpp); these are thin numpy wrappers."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import VameError, lib

PREDS = ("FULL_2CP", "FULL_3CP", "HALF_2CP", "HALF_3CP")  # constants.h:15-21 PRED_TYPES
CPMVS_DTYPE = np.dtype([("nCPs", "<i4"), ("LTx", "<i4"), ("LTy", "<i4"), ("RTx", "<i4"),
                        ("RTy", "<i4"), ("LBx", "<i4"), ("LBy", "<i4")])


def read_frames(path: str, width: int, height: int, n_frames: int, nthreads: int = 0) -> np.ndarray:
    """(n_frames, H, W) uint16 from a reference-layout CSV (or raw .u16/.yuv)."""
    out = np.empty((n_frames, height, width), np.uint16)
    rc = lib().vame_read_frames(path.encode(), width, height, n_frames,
                                out.ctypes.data_as(ctypes.c_void_p), nthreads)
    if rc != 0:
        raise VameError(f"cannot read {n_frames} frames of {width}x{height} from {path} (rc={rc})")
    return out


def remove_old(prefix: str) -> None:
    lib().vame_log_remove_old(prefix.encode())


def write_headers(prefix: str, pred: int) -> None:
    if lib().vame_log_write_headers(prefix.encode(), pred) != 0:
        raise VameError(f"cannot create log files {prefix}_*")


def append(prefix: str, pred: int, width: int, height: int, poc: int, ref: int,
           cost: np.ndarray, cpmvs: np.ndarray, nthreads: int = 0) -> int:
    """Rows of one (POC, refIdx, pred); cost int64[n], cpmvs = [n, 7] int32 or CPMVS_DTYPE[n]."""
    cost = np.ascontiguousarray(cost, np.int64)
    cpmvs = np.ascontiguousarray(cpmvs)
    if cpmvs.dtype != CPMVS_DTYPE:
        cpmvs = np.ascontiguousarray(cpmvs, np.int32)
        assert cpmvs.ndim == 2 and cpmvs.shape[1] == 7
    n = lib().vame_num_ctus(width, height) * (284 if pred >> 1 else 201)
    if cost.shape[0] != n or cpmvs.shape[0] != n:
        raise ValueError(f"results must hold {n} entries")
    nb = lib().vame_log_append(prefix.encode(), pred, width, height, poc, ref,
                               cost.ctypes.data_as(ctypes.c_void_p),
                               cpmvs.ctypes.data_as(ctypes.c_void_p), nthreads)
    if nb < 0:
        raise VameError(f"writing log files {prefix}_* failed")
    return nb


def write_poc(prefix: str, width: int, height: int, poc: int, results, nthreads: int = 0) -> int:
    """Log one POC like main.cpp:942-958: for each refIdx the four PREDs in
    order (headers first at POC 1 / refIdx 0).  results: {(ref, PRED name):
    (cost, cpmvs)} as host arrays."""
    nb = 0
    refs = sorted({r for r, _ in results})
    for r in refs:
        for m, name in enumerate(PREDS):
            if (r, name) not in results:
                continue
            if poc == 1 and r == 0:
                write_headers(prefix, m)
            cost, cp = results[(r, name)]
            nb += append(prefix, m, width, height, poc, r, cost, cp, nthreads)
    return nb
