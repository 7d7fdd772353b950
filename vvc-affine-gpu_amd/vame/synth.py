"""Deterministic synthetic 10-bit luma sequences (the reference's data/*.csv are
absent from its repository).

Every value is built from integer hashing and +,-,*,/ on float64 only -- no
transcendental numpy ufuncs -- so the same seed yields the same bytes on any
x86 host (numpy's SIMD sin/cos dispatch differs between CPUs; these do not).

This numpy code is the specification.  `synth_frame` / `synth_sequence` run
the native generator (csrc/vame_synth.c, lib/libvame_synth.so: the same
arithmetic in the same order, OpenMP over rows) when it is built -- a 240-frame
3840x2160 sequence (BASELINE configs[4]) would take hours here -- and
tests/test_synth.py checks both produce identical bytes.

Layout matches the reference inputs (main.cpp:313-328): `orig[k]` is POC k+1
(the frame being coded), `recon[k]` is the reconstructed POC k (the reference
picture pool), each H x W uint16 in [0, 1023].

Content per frame: multi-octave value noise + three oriented triangle-wave
gratings (texture for the gradient solver), a 96x96 flat patch (singular
normal equations), a hard-edged 64x64 block touching the
bottom-right border (clamp-to-edge padding and MV clipping).  POC k is the
canvas seen through a cumulative affine camera motion (zoom, rotation,
translation) so the affine search has something to find.
"""
from __future__ import annotations

import ctypes
import math
import os
import sys

import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix(z: np.ndarray) -> np.ndarray:
    """SplitMix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    z = z ^ (z >> np.uint64(30))
    z = z * _M1
    z = z ^ (z >> np.uint64(27))
    z = z * _M2
    return z ^ (z >> np.uint64(31))


def _lattice(ix: np.ndarray, iy: np.ndarray, salt: int) -> np.ndarray:
    """Uniform [0,1) value per integer lattice point."""
    with np.errstate(over="ignore"):
        h = (ix.astype(np.int64).view(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
             + iy.astype(np.int64).view(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F)
             + np.uint64(salt & 0xFFFFFFFFFFFFFFFF))
        h = _mix(h)
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def _value_noise(x: np.ndarray, y: np.ndarray, scale: float, salt: int) -> np.ndarray:
    u = x / scale
    v = y / scale
    iu = np.floor(u)
    iv = np.floor(v)
    fu = u - iu
    fv = v - iv
    iu = iu.astype(np.int64)
    iv = iv.astype(np.int64)
    a = _lattice(iu, iv, salt)
    b = _lattice(iu + 1, iv, salt)
    c = _lattice(iu, iv + 1, salt)
    d = _lattice(iu + 1, iv + 1, salt)
    top = a + (b - a) * fu
    bot = c + (d - c) * fu
    return top + (bot - top) * fv - 0.5


def _tri(t: np.ndarray) -> np.ndarray:
    return np.abs(t - np.floor(t) - 0.5) - 0.25


def canvas(x: np.ndarray, y: np.ndarray, W: int, H: int, seed: int) -> np.ndarray:
    """Continuous test pattern at canvas coordinates (x, y)."""
    f = np.full(x.shape, 512.0)
    for k, (scale, amp) in enumerate(((61.0, 420.0), (29.0, 230.0), (13.0, 120.0),
                                      (6.5, 60.0), (3.1, 28.0))):
        f += amp * _value_noise(x, y, scale, seed * 131 + k)
    for (dx, dy, period, amp) in ((0.8, 0.6, 37.0, 240.0), (-0.28, 0.96, 17.0, 160.0),
                                  (0.96, -0.28, 91.0, 200.0)):
        f += amp * _tri((x * dx + y * dy) / period)
    # flat 96x96 patch (textureless -> zero pivots in the solve)
    fx0, fy0 = 0.30 * W, 0.25 * H
    flat = (x >= fx0) & (x < fx0 + 96) & (y >= fy0) & (y < fy0 + 96)
    f = np.where(flat, 600.0, f)
    # hard-edged 64x64 checker block touching the bottom-right border
    bx0, by0 = W - 64.0, H - 64.0
    blk = (x >= bx0) & (y >= by0)
    chk = ((np.floor((x - bx0) / 8.0) + np.floor((y - by0) / 8.0)) % 2.0) == 0.0
    f = np.where(blk, np.where(chk, 980.0, 40.0), f)
    return f


def _pixel_noise(x: np.ndarray, y: np.ndarray, salt: int, amp: int) -> np.ndarray:
    """Uniform integer in [-amp, amp] per pixel from a hash of (x, y, salt)."""
    with np.errstate(over="ignore"):
        h = (x.astype(np.int64).view(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
             + y.astype(np.int64).view(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F)
             + np.uint64(salt & 0xFFFFFFFFFFFFFFFF))
        h = _mix(h)
    return (((h >> np.uint64(32)) * np.uint64(2 * amp + 1)) >> np.uint64(32)).astype(np.int64) - amp


def camera(poc: int):
    """Cumulative camera of POC `poc`: (zoom, cos, sin, tx, ty)."""
    ang = math.radians(0.15) * poc
    return 1.0 + 0.004 * poc, math.cos(ang), math.sin(ang), 1.25 * poc, -0.75 * poc


def synth_frame_np(W: int, H: int, poc: int, seed: int = 0x5EED) -> np.ndarray:
    """Original POC `poc` (H x W uint16) -- the numpy specification."""
    zoom, ca, sa, tx, ty = camera(poc)
    yy, xx = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64),
                         indexing="ij")
    cx, cy = W / 2.0, H / 2.0
    # inverse camera: canvas point seen at pixel (xx, yy)
    px = (xx - cx - tx) / zoom
    py = (yy - cy - ty) / zoom
    sx = ca * px + sa * py + cx
    sy = -sa * px + ca * py + cy
    f = canvas(sx, sy, W, H, seed)
    f = np.floor(f + 0.5) + _pixel_noise(xx, yy, seed * 1000003 + poc, 2)
    return np.clip(f, 0, 1023).astype(np.uint16)


def recon_noise_amp(qp: int) -> int:
    return max(0, (qp - 17) // 5)


def recon_np(frame: np.ndarray, poc: int, qp: int, seed: int = 0x5EED) -> np.ndarray:
    """Reconstructed POC `poc` from its original -- the numpy specification."""
    H, W = frame.shape
    amp = recon_noise_amp(qp)
    yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    r = frame.astype(np.int64) + (_pixel_noise(xx, yy, (seed ^ 0xC0FFEE) * 7919 + poc, amp) if amp else 0)
    return np.clip(r, 0, 1023).astype(np.uint16)


_native = None
_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                         "libvame_synth.so")


_warned = False


def native():
    """ctypes handle of lib/libvame_synth.so, or None when it is not built (or
    VAME_SYNTH_NUMPY is set): the numpy specification is then used, with a
    one-time warning -- it is ~50x slower (4K frames take seconds each)."""
    global _native, _warned
    if _native is None:
        if not os.path.exists(_LIB_PATH) or os.environ.get("VAME_SYNTH_NUMPY"):
            if not _warned and not os.environ.get("VAME_SYNTH_NUMPY"):
                print(f"vame.synth: {_LIB_PATH} not built (make synth); using the numpy generator",
                      file=sys.stderr)
                _warned = True
            return None
        L = ctypes.CDLL(_LIB_PATH)
        I, D, P, U = ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_uint64
        L.vame_synth_frame.argtypes = [I, I, U, I, D, D, D, D, D, P]
        L.vame_synth_frame.restype = None
        L.vame_synth_recon.argtypes = [P, I, I, U, I, I, P]
        L.vame_synth_recon.restype = None
        L.vame_synth_write_csv.argtypes = [ctypes.c_char_p, P, I, I, I]
        _native = L
    return _native


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def synth_frame(W: int, H: int, poc: int, seed: int = 0x5EED) -> np.ndarray:
    """Original POC `poc` (H x W uint16)."""
    L = native()
    if L is None:
        return synth_frame_np(W, H, poc, seed)
    out = np.empty((H, W), np.uint16)
    L.vame_synth_frame(W, H, seed & 0xFFFFFFFFFFFFFFFF, poc, *camera(poc), _p(out))
    return out


def recon_frame(frame: np.ndarray, poc: int, qp: int, seed: int = 0x5EED) -> np.ndarray:
    """Reconstructed POC `poc`: its original + uniform noise of +-floor((QP-17)/5)."""
    L = native()
    if L is None:
        return recon_np(frame, poc, qp, seed)
    H, W = frame.shape
    frame = np.ascontiguousarray(frame, np.uint16)
    out = np.empty((H, W), np.uint16)
    L.vame_synth_recon(_p(frame), W, H, seed & 0xFFFFFFFFFFFFFFFF, poc, recon_noise_amp(qp), _p(out))
    return out


def synth_sequence(W: int, H: int, n_frames: int, qp: int = 32, seed: int = 0x5EED):
    """(orig, recon): orig[k] = POC k+1, recon[k] = reconstructed POC k; each
    (n_frames, H, W) uint16."""
    orig = np.empty((n_frames, H, W), np.uint16)
    recon = np.empty((n_frames, H, W), np.uint16)
    prev = synth_frame(W, H, 0, seed)
    for poc in range(n_frames):
        recon[poc] = recon_frame(prev, poc, qp, seed)
        prev = synth_frame(W, H, poc + 1, seed)
        orig[poc] = prev
    return orig, recon


def synth_pocs(W: int, H: int, pocs, ref_pocs, qp: int = 32, seed: int = 0x5EED):
    """Only the frames a frame shard needs: {poc: orig POC} for `pocs` and
    {poc: recon POC} for `ref_pocs` -- the same bytes as synth_sequence."""
    orig = {p: synth_frame(W, H, p, seed) for p in pocs}
    recon = {}
    for p in ref_pocs:
        f = orig[p] if p in orig else synth_frame(W, H, p, seed)
        recon[p] = recon_frame(f, p, qp, seed)
    return orig, recon


def write_csv(path: str, frames: np.ndarray) -> None:
    """Reference CSV layout: one row per frame line, ',' separated, frames stacked
    vertically (main.cpp:313-328)."""
    n, H, W = frames.shape
    L = native()
    if L is not None:
        fr = np.ascontiguousarray(frames, np.uint16)
        if L.vame_synth_write_csv(path.encode(), _p(fr), n, W, H) != 0:
            raise OSError(f"cannot write {path}")
        return
    with open(path, "w") as f:
        for k in range(n):
            np.savetxt(f, frames[k], fmt="%d", delimiter=",")
