#!/usr/bin/env python3
"""Golden vectors for the host-side per-POC logic (run here, where the
reference checkout exists; the output JSON is what the tests read).

* lambda / QP per POC: main.cpp:585 `fullLambdas[computeDeltaQp(QP, POC)]`,
  computeDeltaQp restated from main_aux_functions.h:1481-1496, the 60-entry
  table parsed as data from constants.h:94.
* reference list per POC: the reference's own debug replay of the ring
  (testReferences, main_aux_functions.h:1499-1545), restated.
* decision-log tables: the host-side arrays the log writer indexes
  (reportAffineResultsMaster_new, main_aux_functions.h:387-525) parsed as data
  from constants.h -- WIDTH/HEIGHT_LIST, RETURN_STRIDE_LIST, HA_WIDTH/HEIGHT_LIST,
  HA_RETURN_STRIDE_LIST, HA_ALL_X_POS / HA_ALL_Y_POS -- with the per-group CU
  count rule of main_aux_functions.h:447-450.
"""
import json
import math
import os
import re
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def full_lambdas():
    src = open(os.path.join(REF, "constants.h")).read()
    body = src[src.index("fullLambdas[60]"):]
    body = body[body.index("{") + 1:body.index("}")]
    body = re.sub(r"/\*.*?\*/|//[^\n]*", "", body, flags=re.S)  # drop the index comments
    vals = [float(v) for v in re.findall(r"\d+\.\d+", body)]
    assert len(vals) == 60, len(vals)
    return [float(np.float32(v)) for v in vals]


def compute_delta_qp(qp_in, poc):
    off = [1, 5, 4, 5, 4, 5, 4, 5]
    scale = 0.0 if poc % 8 == 0 else 0.259
    offset = 0.0 if poc % 8 == 0 else -6.5
    qp = qp_in + off[poc % 8]
    d = qp * scale + offset + 0.5
    qp += int(math.floor(min(max(d, 0.0), 3.0)))  # clip3 returns floor (main_aux_functions.h:1478)
    return qp


def ref_lists(n):
    L, LT, out = [-1] * 4, [0] * 4, {}
    for f in range(1, n + 1):
        if f < 5:
            tA = L[0]; L[0] = f - 1; tB = L[1]; L[1] = tA; tA = L[2]; L[2] = tB; L[3] = tA
            LT[3] = 1 if L[3] % 8 == 0 else 0
        else:
            tA = L[0]; L[0] = f - 1; tB = L[1]
            L[1] = tA if LT[1] == 0 else (tA if (tA % 8 == 0 and tA != L[0]) else L[1])
            tA = L[2]
            L[2] = tB if LT[2] == 0 else (tB if (tB % 8 == 0 and tB != L[1]) else L[2])
            L[3] = tA if LT[3] == 0 else (tA if (tA % 8 == 0 and tA != L[2]) else L[3])
            LT[3] = 1 if L[3] % 8 == 0 else 0
            LT[2] = 1 if (L[2] % 8 == 0 and LT[3]) else 0
            LT[1] = 1 if (L[1] % 8 == 0 and LT[2]) else 0
        out[f] = L[:min(4, f)]
    return out


def _c_array(src, name):
    """Integer initialiser of `name[...] = {...}` in constants.h (1-D or 2-D)."""
    i = re.search(r"\b" + name + r"\[", src).start()
    i = src.index("=", i)
    j = src.index("{", i)
    depth, k = 0, j
    while True:
        if src[k] == "{":
            depth += 1
        elif src[k] == "}":
            depth -= 1
            if depth == 0:
                break
        k += 1
    body = re.sub(r"/\*.*?\*/|//[^\n]*", "", src[j:k + 1], flags=re.S)
    if body.count("{") > 1:
        rows = re.findall(r"\{([^{}]*)\}", body)
        return [[int(eval(v.strip())) for v in r.split(",") if v.strip()] for r in rows]
    return [int(eval(v.strip())) for v in body.strip().strip("{}").split(",") if v.strip()]


def log_tables():
    src = open(os.path.join(REF, "constants.h")).read()
    t = {n: _c_array(src, n) for n in ("WIDTH_LIST", "HEIGHT_LIST", "RETURN_STRIDE_LIST",
                                       "HA_WIDTH_LIST", "HA_HEIGHT_LIST", "HA_RETURN_STRIDE_LIST",
                                       "HA_ALL_X_POS", "HA_ALL_Y_POS")}
    # main_aux_functions.h:447-450: the last group of each list has a fixed count
    full_n = [64 if g == 11 else t["RETURN_STRIDE_LIST"][g + 1] - t["RETURN_STRIDE_LIST"][g]
              for g in range(12)]
    half_n = [32 if g == 23 else t["HA_RETURN_STRIDE_LIST"][g + 1] - t["HA_RETURN_STRIDE_LIST"][g]
              for g in range(24)]
    full = [{"w": t["WIDTH_LIST"][g], "h": t["HEIGHT_LIST"][g], "n": full_n[g],
             "stride": t["RETURN_STRIDE_LIST"][g]} for g in range(12)]
    half = [{"w": t["HA_WIDTH_LIST"][g], "h": t["HA_HEIGHT_LIST"][g], "n": half_n[g],
             "stride": t["HA_RETURN_STRIDE_LIST"][g],
             "x": t["HA_ALL_X_POS"][g][:half_n[g]], "y": t["HA_ALL_Y_POS"][g][:half_n[g]]}
            for g in range(24)]
    for g in half:
        assert len(g["x"]) == g["n"] and len(g["y"]) == g["n"], g
    return {"full": full, "half": half}


def main():
    lam = full_lambdas()
    rows = []
    for qp in range(22, 38):
        for poc in range(1, 17):
            q = compute_delta_qp(qp, poc)
            rows.append({"qp": qp, "poc": poc, "poc_qp": q, "lambda": lam[q]})
    refs = ref_lists(64)
    out = {"lambda": rows, "ref_lists": {str(k): v for k, v in refs.items()},
           "log_tables": log_tables()}
    json.dump(out, open(os.path.join(HERE, "hostlogic.json"), "w"), indent=0)
    print(f"{len(rows)} lambda rows, {len(refs)} ref lists")


if __name__ == "__main__":
    sys.exit(main())
