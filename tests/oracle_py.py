"""ctypes view of oracle/libvame_oracle.so (the CPU restatement).  Test
infrastructure: imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "libvame_oracle.so")

CPMVS_DTYPE = np.dtype([("nCPs", "<i4"), ("LTx", "<i4"), ("LTy", "<i4"), ("RTx", "<i4"),
                        ("RTy", "<i4"), ("LBx", "<i4"), ("LBy", "<i4")])
assert CPMVS_DTYPE.itemsize == 28

_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ORACLE_DIR, "vame_oracle.c")
        if (not os.path.exists(ORACLE_SO)) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "libvame_oracle.so"])
        L = ctypes.CDLL(ORACLE_SO)
        P = ctypes.c_void_p
        L.vame_oracle_affine_me.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P,
                                            ctypes.c_int]
        L.vame_oracle_affine_me.restype = ctypes.c_int
        L.vame_oracle_affine_me_ex.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, P, P, P, ctypes.c_int]
        L.vame_oracle_affine_me_ex.restype = ctypes.c_int
        L.vame_oracle_prof_deltas.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P]
        L.vame_oracle_predict_4x4_prof.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                   P, P, P]
        L.vame_oracle_num_ctus.argtypes = [ctypes.c_int, ctypes.c_int]
        L.vame_oracle_satd4x4.argtypes = [P, P]
        L.vame_oracle_eg_bits.argtypes = [ctypes.c_int]
        L.vame_oracle_to_quarter.argtypes = [ctypes.c_int]
        L.vame_oracle_affine_bits.argtypes = [P, ctypes.c_int]
        L.vame_oracle_rate_cost.argtypes = [ctypes.c_int, ctypes.c_float]
        L.vame_oracle_rate_cost.restype = ctypes.c_int64
        L.vame_oracle_scale_delta.argtypes = [ctypes.c_double]
        L.vame_oracle_spread.argtypes = [ctypes.c_int] * 4
        L.vame_oracle_predict_4x4.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
        L.vame_oracle_seed_3cp.argtypes = [P] + [ctypes.c_int] * 6 + [P]
        L.vame_oracle_solve.argtypes = [P, ctypes.c_int, P]
        L.vame_oracle_group_geometry.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P, P, P]
        _lib = L
    return _lib


def ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def affine_me(ref: np.ndarray, cur: np.ndarray, lam: float, align: int, ncp: int,
              extra: int = 0, prev: np.ndarray | None = None, nthreads: int = 0,
              prof: bool = False):
    """One reference launch (affine.cl:11 / :960 with -DnCP=ncp) on the CPU;
    prof=True turns on the reference's (hard-disabled) PROF branch."""
    H, W = ref.shape
    ref = np.ascontiguousarray(ref, dtype=np.uint16)
    cur = np.ascontiguousarray(cur, dtype=np.uint16)
    n = lib().vame_oracle_num_ctus(W, H) * (284 if align else 201)
    cost = np.zeros(n, np.int64)
    cp = np.zeros(n, CPMVS_DTYPE)
    pv = None if prev is None else np.ascontiguousarray(prev)
    rc = lib().vame_oracle_affine_me_ex(ptr(ref), ptr(cur), W, H, lam, align, ncp, extra,
                                        int(prof), None if pv is None else ptr(pv),
                                        ptr(cost), ptr(cp), nthreads)
    if rc != 0:
        raise RuntimeError(f"oracle rc={rc}")
    return cost, cp


def affine_me_pair(ref, cur, lam, extra=0, modes=(2, 3), nthreads=0, prof=False):
    """All four reference launches of one (POC, ref) pair, chained like
    main.cpp:759-966.  Returns {(align, ncp): (cost, cpmvs)}."""
    out = {}
    for align in (0, 1):
        c2, p2 = affine_me(ref, cur, lam, align, 2, extra, nthreads=nthreads, prof=prof)
        out[(align, 2)] = (c2, p2)
        if 3 in modes:
            out[(align, 3)] = affine_me(ref, cur, lam, align, 3, extra, prev=p2,
                                        nthreads=nthreads, prof=prof)
    return out


def prof_deltas(cp: np.ndarray, ncp: int, w: int, h: int):
    """aux_functions.cl:218-404: (dH[16], dV[16]) of a CU's sub-blocks."""
    cp = np.ascontiguousarray(cp, CPMVS_DTYPE)
    dh, dv = np.zeros(16, np.int32), np.zeros(16, np.int32)
    lib().vame_oracle_prof_deltas(ptr(cp), ncp, w, h, ptr(dh), ptr(dv))
    return dh, dv


def predict_4x4_prof(ref: np.ndarray, x0: int, y0: int, mvx: int, mvy: int, dh, dv):
    """horizontal_vertical_filter_new with enablePROF=1, isSpread=0."""
    H, W = ref.shape
    ref = np.ascontiguousarray(ref, dtype=np.uint16)
    dh = np.ascontiguousarray(dh, np.int32)
    dv = np.ascontiguousarray(dv, np.int32)
    out = np.zeros(16, np.int32)
    lib().vame_oracle_predict_4x4_prof(ptr(ref), W, H, x0, y0, mvx, mvy, ptr(dh), ptr(dv),
                                       ptr(out))
    return out


def group_geometry(align):
    """[(w, h, xs, ys, stride)] per CU group of an alignment, from the oracle's tables."""
    out = []
    for g in range(24 if align else 12):
        w, h, n, s = (np.zeros(1, np.int32) for _ in range(4))
        xs, ys = np.zeros(64, np.int32), np.zeros(64, np.int32)
        assert lib().vame_oracle_group_geometry(align, g, ptr(w), ptr(h), ptr(n),
                                                ptr(s), ptr(xs), ptr(ys)) == 0
        out.append((int(w[0]), int(h[0]), xs[:n[0]].copy(), ys[:n[0]].copy(), int(s[0])))
    return out
