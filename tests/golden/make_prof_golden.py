#!/usr/bin/env python3
"""PROF known-answer vectors from the reference's own PROF functions.

    python tests/golden/make_prof_golden.py prepare <dir>   # inputs -> <dir>/in.bin
    oracle/_ref/prof_kat_hip oracle/_ref/prof_kat.co <dir>/in.bin <dir>/out.bin   (MI355X)
    python tests/golden/make_prof_golden.py pack <dir>      # -> tests/golden/prof_kat.npz

oracle/prof_kat.cl calls aux_functions.cl's get{Horizontal,Vertical}DeltasPROF{2,3}Cps
and horizontal_vertical_filter_new(..., enablePROF=1) (compiled from
/root/reference where they lie) on these cases; the npz holds inputs and the
reference's outputs.  Seeded, so `prepare` is reproducible.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
N = 4096
SIZES = [8, 16, 32, 64, 128]


def cases():
    rng = np.random.default_rng(0x9E0F)
    win = np.zeros((N, 121), np.int32)
    prm = np.zeros((N, 12), np.int32)
    yy, xx = np.mgrid[0:11, 0:11]
    for g in range(N):
        kind = g % 4
        if kind == 0:    # noise
            w = rng.integers(0, 1024, (11, 11))
        elif kind == 1:  # smooth ramp + texture
            a, b, c = rng.uniform(-80, 80, 3)
            w = np.clip(512 + a * xx + b * yy + c * np.sin(xx * 0.9 + yy * 0.4), 0, 1023)
        elif kind == 2:  # hard edge
            t = rng.integers(1, 10)
            w = np.where(xx + (yy if rng.random() < 0.5 else 0) < t, rng.integers(0, 200),
                         rng.integers(800, 1024)) + 0 * xx
        else:            # extremes
            w = rng.choice([0, 1023], (11, 11))
        win[g] = np.asarray(w, np.int64).reshape(-1)
        ncp = 2 + (g // 4) % 2
        mag = [16, 256, 4096, 1 << 17][(g // 8) % 4]
        cp = rng.integers(-mag, mag, 6)
        if ncp == 2:
            cp[4:] = 0
        pw, ph = SIZES[rng.integers(0, 5)], SIZES[rng.integers(0, 5)]
        fx, fy = rng.integers(0, 16, 2)
        spread = 1 if g % 16 == 15 else 0  # a few cases take the non-PROF branch
        prm[g] = [ncp, *cp, pw, ph, fx, fy, spread]
    return win, prm


def main():
    mode, d = sys.argv[1], sys.argv[2]
    os.makedirs(d, exist_ok=True)
    win, prm = cases()
    if mode == "prepare":
        with open(os.path.join(d, "in.bin"), "wb") as f:
            np.array([N], np.int32).tofile(f)
            win.tofile(f)
            prm.tofile(f)
    elif mode == "pack":
        out = np.fromfile(os.path.join(d, "out.bin"), np.int32).reshape(N, 48)
        np.savez_compressed(os.path.join(HERE, "prof_kat.npz"), win=win.astype(np.int16),
                            prm=prm, dH=out[:, :16].astype(np.int8), dV=out[:, 16:32].astype(np.int8),
                            pred=out[:, 32:].astype(np.int16))
    else:
        raise SystemExit(__doc__)


if __name__ == "__main__":
    main()
