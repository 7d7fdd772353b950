"""Deterministic synthetic 10-bit luma sequences (the reference's data/*.csv are
absent from its repository).

Every value is built from integer hashing and +,-,*,/ on float64 only -- no
transcendental numpy ufuncs -- so the same seed yields the same bytes on any
x86 host (numpy's SIMD sin/cos dispatch differs between CPUs; these do not).

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

import math

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


def synth_frame(W: int, H: int, poc: int, seed: int = 0x5EED) -> np.ndarray:
    """Original POC `poc` (H x W uint16)."""
    zoom = 1.0 + 0.004 * poc
    ang = math.radians(0.15) * poc
    ca, sa = math.cos(ang), math.sin(ang)
    tx, ty = 1.25 * poc, -0.75 * poc
    yy, xx = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64),
                         indexing="ij")
    cx, cy = W / 2.0, H / 2.0
    # inverse camera: canvas point seen at pixel (xx, yy)
    px = (xx - cx - tx) / zoom
    py = (yy - cy - ty) / zoom
    sx = ca * px + sa * py + cx
    sy = -sa * px + ca * py + cy
    f = canvas(sx, sy, W, H, seed)
    rng = np.random.Generator(np.random.PCG64(seed * 1000003 + poc))
    f = np.floor(f + 0.5) + rng.integers(-2, 3, size=f.shape)
    return np.clip(f, 0, 1023).astype(np.uint16)


def recon_noise_amp(qp: int) -> int:
    return max(0, (qp - 17) // 5)


def synth_sequence(W: int, H: int, n_frames: int, qp: int = 32, seed: int = 0x5EED):
    """(orig, recon): orig[k] = POC k+1, recon[k] = reconstructed POC k; each
    (n_frames, H, W) uint16."""
    frames = [synth_frame(W, H, poc, seed) for poc in range(n_frames + 1)]
    orig = np.stack(frames[1:])
    amp = recon_noise_amp(qp)
    recon = []
    for poc in range(n_frames):
        rng = np.random.Generator(np.random.PCG64((seed ^ 0xC0FFEE) * 7919 + poc))
        r = frames[poc].astype(np.int32) + rng.integers(-amp, amp + 1, size=(H, W))
        recon.append(np.clip(r, 0, 1023).astype(np.uint16))
    return orig, np.stack(recon)


def write_csv(path: str, frames: np.ndarray) -> None:
    """Reference CSV layout: one row per frame line, ',' separated, frames stacked
    vertically (main.cpp:313-328)."""
    n, H, W = frames.shape
    with open(path, "w") as f:
        for k in range(n):
            np.savetxt(f, frames[k], fmt="%d", delimiter=",")
