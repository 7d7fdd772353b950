"""Restatement of the reference's decision-log writer and frame reader, for
checking the native ones (test infrastructure only).

* write: reportAffineResultsMaster_new (main_aux_functions.h:387-525) -- file
  names (:392-425), header (:418/:430), CU positions (:460-479) and the fprintf
  row format (:491), driven by the host tables parsed from constants.h into
  tests/golden/hostlogic.json ("log_tables") by make_hostlogic_golden.py.
* remove: removeOldTraces (main_aux_functions.h:1547-1585).
* read: main.cpp:313-328 (getline per line, getline(',') + stoi per value).
"""
from __future__ import annotations

import json
import math
import os

import re

import numpy as np

_STOI = re.compile(r"\s*([+-]?\d+)")

HERE = os.path.dirname(os.path.abspath(__file__))
TABLES = json.load(open(os.path.join(HERE, "golden", "hostlogic.json")))["log_tables"]
HEADER = "POC,List,Ref,CTU,idx,X,Y,Cost,LT_X,LT_Y,RT_X,RT_Y,LB_X,LB_Y\n"
TYPES = ("_FULL_2CPs_", "_FULL_3CPs_", "_HALF_2CPs_", "_HALF_3CPs_")
NUM_CTUS = {(3840, 2160): 510, (1920, 1080): 135, (1280, 720): 60, (832, 480): 28, (416, 240): 8}


def groups(pred):
    return TABLES["half"] if pred >= 2 else TABLES["full"]


def file_names(prefix, pred):
    return [f"{prefix}{TYPES[pred]}{g['w']}x{g['h']}.csv" for g in groups(pred)]


def write_headers(prefix, pred):
    for fn in file_names(prefix, pred):
        with open(fn, "w") as f:
            f.write(HEADER)


def rows(pred, W, H, poc, ref, cost, cp):
    """{file name suffix: text} of one (POC, refIdx, pred) in group order."""
    n_ctus = NUM_CTUS[(W, H)]
    total = 284 if pred >= 2 else 201
    cols = math.ceil(W / 128)
    out = []
    for gi, g in enumerate(groups(pred)):
        lines = []
        for ctu in range(n_ctus):
            for cu in range(g["n"]):
                if pred < 2:
                    y = (cu * g["w"]) // 128 * g["h"]
                    x = (cu * g["w"]) % 128
                else:
                    x, y = g["x"][cu], g["y"][cu]
                y += (ctu // cols) * 128
                x += (ctu % cols) * 128
                i = ctu * total + g["stride"] + cu
                c = cp[i]
                lines.append("%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d\n" % (
                    poc, 0, ref, ctu, cu, x, y, cost[i], c[1], c[2], c[3], c[4], c[5], c[6]))
        out.append((gi, "".join(lines)))
    return out


def append(prefix, pred, W, H, poc, ref, cost, cp):
    names = file_names(prefix, pred)
    for gi, text in rows(pred, W, H, poc, ref, cost, cp):
        with open(names[gi], "a") as f:
            f.write(text)


def remove_old(prefix):
    for t in ("FULL_2CPs", "FULL_3CPs", "HALF_2CPs", "HALF_3CPs"):
        for g in TABLES["full"]:
            fn = f"{prefix}_{t}_{g['w']}x{g['h']}.csv"
            if os.path.exists(fn):
                os.remove(fn)


def read_frames(path, W, H, n):
    out = np.zeros((n, H, W), np.uint16)
    with open(path) as f:
        for k in range(n):
            for h in range(H):
                vals = f.readline().rstrip("\n").split(",")
                for w in range(W):
                    # stoi: leading blanks, sign, digits; the rest is ignored
                    out[k, h, w] = int(_STOI.match(vals[w]).group(1)) & 0xFFFF
    return out
