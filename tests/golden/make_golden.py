#!/usr/bin/env python3
"""Golden-vector pipeline: outputs of the REFERENCE kernels on fixed inputs.

    python tests/golden/make_golden.py prepare DIR     # inputs (.u16) + DIR/jobs.txt
    oracle/_ref/ref_harness oracle/_ref/affine_2cp.co oracle/_ref/affine_3cp.co DIR/jobs.txt
                                                       # on an MI355X (OpenCL runtime)
    python tests/golden/make_golden.py pack DIR        # -> tests/golden/*.npz

The reference kernels are compiled from /root/reference/affine.cl by
`make -C oracle ref` (see oracle/Makefile).  Each fixture holds the input
frames, lambda, ExtraGradientIter and the reference's cost/CPMV arrays for the
four launches of one (POC, ref) pair; tests/test_oracle_golden.py checks the
CPU oracle against them bit for bit.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "vvc-affine-gpu_amd"))

from vame import synth  # noqa: E402

CPMVS_DTYPE = np.dtype([("nCPs", "<i4"), ("LTx", "<i4"), ("LTy", "<i4"), ("RTx", "<i4"),
                        ("RTy", "<i4"), ("LBx", "<i4"), ("LBy", "<i4")])
TAGS = ("FULL_2CP", "FULL_3CP", "HALF_2CP", "HALF_3CP")
LAMBDA = {(32, 1): 78.949063, (32, 2): 70.335619, (22, 1): 11.077166, (37, 1): 177.234655}


def cases():
    """name -> (W, H, lambda, extra, ref frame, cur frame)."""
    out = {}
    o, r = synth.synth_sequence(416, 240, 2, 32)
    out["s416_qp32_poc1_ref0"] = (416, 240, LAMBDA[(32, 1)], 0, r[0], o[0])
    out["s416_qp32_poc2_ref0"] = (416, 240, LAMBDA[(32, 2)], 0, r[1], o[1])
    out["s416_qp32_poc2_ref1"] = (416, 240, LAMBDA[(32, 2)], 0, r[0], o[1])
    o22, r22 = synth.synth_sequence(416, 240, 1, 22, seed=0x1234)
    out["s416_qp22_poc1_extra1"] = (416, 240, LAMBDA[(22, 1)], 1, r22[0], o22[0])
    out["s416_identical"] = (416, 240, LAMBDA[(32, 1)], 0, o[0], o[0].copy())
    flat = np.full((240, 416), 512, np.uint16)
    out["s416_flat"] = (416, 240, LAMBDA[(32, 1)], 0, flat, flat.copy())
    rng = np.random.Generator(np.random.PCG64(77))
    out["s416_noise"] = (416, 240, LAMBDA[(32, 1)], 0,
                         rng.integers(0, 1024, (240, 416)).astype(np.uint16),
                         rng.integers(0, 1024, (240, 416)).astype(np.uint16))
    yy, xx = np.mgrid[0:240, 0:416]
    chk = np.where((xx + yy) % 2 == 0, 1023, 0).astype(np.uint16)
    out["s416_checker"] = (416, 240, LAMBDA[(32, 1)], 0, chk, np.roll(chk, 1, axis=1))
    big = synth.synth_frame(416 + 128, 240 + 128, 3, seed=0xBEEF)
    out["s416_bigmotion"] = (416, 240, LAMBDA[(32, 1)], 0, big[64:304, 64:480].copy(),
                             big[64 + 23:304 + 23, 64 - 37:480 - 37].copy())
    o8, r8 = synth.synth_sequence(832, 480, 1, 37, seed=0x832)
    out["s832_qp37_poc1"] = (832, 480, LAMBDA[(37, 1)], 0, r8[0], o8[0])
    return out


def prepare(d):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "jobs.txt"), "w") as jf:
        for name, (W, H, lam, extra, ref, cur) in cases().items():
            rp, cp = os.path.join(d, name + "_ref.u16"), os.path.join(d, name + "_cur.u16")
            np.ascontiguousarray(ref, np.uint16).tofile(rp)
            np.ascontiguousarray(cur, np.uint16).tofile(cp)
            jf.write(f"{W} {H} {lam!r} {extra} {rp} {cp} {os.path.join(d, name)}\n")


def prepare1080(d):
    """One 1080p QP32 pair (POC 1, ref 0) for live reference-vs-HIP checks and the
    reference's own GPU kernel time (not committed: ~4 MB of outputs)."""
    os.makedirs(d, exist_ok=True)
    o, r = synth.synth_sequence(1920, 1080, 1, 32)
    rp, cp = os.path.join(d, "p1080_ref.u16"), os.path.join(d, "p1080_cur.u16")
    r[0].tofile(rp)
    o[0].tofile(cp)
    with open(os.path.join(d, "jobs.txt"), "w") as jf:
        jf.write(f"1920 1080 {LAMBDA[(32, 1)]!r} 0 {rp} {cp} {os.path.join(d, 'p1080')}\n")


def load_result(prefix, tag, n):
    raw = np.fromfile(f"{prefix}_{tag}.bin", np.uint8)
    assert raw.size == n * 36, (prefix, tag, raw.size, n)
    cost = raw[: n * 8].view(np.int64).copy()
    cp = raw[n * 8:].view(CPMVS_DTYPE).copy()
    return cost, cp


def pack(d):
    for name, (W, H, lam, extra, ref, cur) in cases().items():
        nctu = {416: 8, 832: 28}[W]
        for tag in TAGS:  # runs A and B of the (racy) reference must agree
            n = nctu * (201 if tag.startswith("FULL") else 284)
            a = open(os.path.join(d, f"{name}_A_{tag}.bin"), "rb").read()
            b = open(os.path.join(d, f"{name}_B_{tag}.bin"), "rb").read()
            ca, pa = load_result(os.path.join(d, name + "_A"), tag, n)
            cb, pb = load_result(os.path.join(d, name + "_B"), tag, n)
            assert (ca == cb).all() and all((pa[f] == pb[f]).all() for f in CPMVS_DTYPE.names[1:]), \
                f"reference runs disagree: {name} {tag}"
            del a, b
        arrays = dict(W=W, H=H, lam=np.float32(lam), extra=extra,
                      ref=np.ascontiguousarray(ref, np.uint16),
                      cur=np.ascontiguousarray(cur, np.uint16))
        for tag in TAGS:
            n = nctu * (201 if tag.startswith("FULL") else 284)
            cost, cp = load_result(os.path.join(d, name + "_A"), tag, n)
            arrays[tag + "_cost"] = cost
            # nCPs is never written by the reference kernel (uninitialised LDS): drop it
            arrays[tag + "_cpmv"] = np.stack([cp[f] for f in CPMVS_DTYPE.names[1:]], 1)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
        print("packed", name)


if __name__ == "__main__":
    {"prepare": prepare, "prepare1080": prepare1080, "pack": pack}[sys.argv[1]](sys.argv[2])
