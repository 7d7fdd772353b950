"""Host-side per-POC logic, served by libvame.so (native C++:
csrc/vame_hostlogic.cpp).  No device work."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import lib


def poc_qp(qp: int, poc: int) -> int:
    """main_aux_functions.h:1482-1497 computeDeltaQp."""
    return int(lib().vame_poc_qp(qp, poc))


def lambda_for_poc(qp: int, poc: int) -> float:
    """main.cpp:585: fullLambdas[computeDeltaQp(QP, POC)] (a float32 value)."""
    return float(np.float32(lib().vame_lambda(qp, poc)))


def ref_list(poc: int) -> list[int]:
    """POCs held by refIdx 0..min(4,poc)-1 at `poc` (main.cpp:591-707)."""
    out = (ctypes.c_int * 4)()
    n = lib().vame_ref_list(poc, out)
    if n < 0:
        raise ValueError(f"bad poc {poc}")
    return [out[i] for i in range(n)]


def geometry(align: int):
    """[(w, h, xs, ys, stride)] per CU group of an alignment (product tables)."""
    L = lib()
    out = []
    for g in range(L.vame_num_groups(align)):
        w, h, n, s = (np.zeros(1, np.int32) for _ in range(4))
        xs, ys = np.zeros(64, np.int32), np.zeros(64, np.int32)
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        rc = L.vame_group_geometry(align, g, P(w), P(h), P(n), P(s), P(xs), P(ys))
        assert rc == 0
        out.append((int(w[0]), int(h[0]), xs[:n[0]].copy(), ys[:n[0]].copy(), int(s[0])))
    return out
