"""Work and algorithmic-byte accounting of the hot path.

Unit of work: one decision-log row = one (POC, ref, alignment, nCP, CU)
candidate.  Algorithmic bytes of one candidate CU evaluation:
    B_alg = n_pred * n_sb * 162   (9x9 int16 reference window per 4x4 sub-block
                                   per prediction: the 6-tap support)
          + n_sb * 32             (the original CU, read once)
          + 36                    (result: int64 cost + 28-byte CPMVs)
with n_sb counted over in-frame CUs only (out-of-frame candidates are logged
but never predicted, affine.cl:192-208) and n_pred = 6 (2 CP) / 5 (3 CP)
plus ExtraGradientIter.
"""
from __future__ import annotations

from .hostlogic import geometry

N_PRED = {2: 6, 3: 5}


def cu_inventory(W: int, H: int):
    """[(align, w, h, inframe, big_class)] for every candidate CU of one frame."""
    ctus_per_row = (W + 127) // 128
    rows = (H + 127) // 128
    out = []
    for align in (0, 1):
        for (w, h, xs, ys, _) in geometry(align):
            for ctu in range(ctus_per_row * rows):
                cx, cy = (ctu % ctus_per_row) * 128, (ctu // ctus_per_row) * 128
                for x, y in zip(xs, ys):
                    inframe = cx + x + w <= W and cy + y + h <= H
                    out.append((align, w, h, inframe, align == 0 and (w == 128 or h == 128)))
    return out


def pair_accounting(W: int, H: int, ncps=(2,), extra: int = 0):
    """Per (POC, ref) pair: rows, in-frame rows, and B_alg split by kernel class
    ('quad' = the quadrant CUs: 'quad1' = those of affine_me_quad -- 16
    sub-blocks, and the 64x64 CUs -- and 'quad2' = those of affine_me_quad2 --
    32 to 128 sub-blocks; 'big' = the 128-class CUs: 'ctu' = the 128x128 CUs of
    affine_me_ctu2, 'half' = the 128x64 / 64x128 CUs of affine_me_half2w /
    _half2h)."""
    acc = {"rows": 0, "rows_inframe": 0, "bytes_quad": 0, "bytes_quad1": 0, "bytes_quad2": 0, "bytes_big": 0,
           "bytes_ctu": 0, "bytes_half": 0, "bytes_half_w": 0, "bytes_half_h": 0, "sb_pred": 0, "sb_pred_quad": 0,
           "sb_pred_big": 0}
    inv = cu_inventory(W, H)
    for ncp in ncps:
        npred = N_PRED[ncp] + extra
        for (_, w, h, inframe, big) in inv:
            acc["rows"] += 1
            b = 36
            if inframe:
                acc["rows_inframe"] += 1
                nsb = (w // 4) * (h // 4)
                b += npred * nsb * 162 + nsb * 32
                acc["sb_pred"] += npred * nsb
                acc["sb_pred_big" if big else "sb_pred_quad"] += npred * nsb
            acc["bytes_big" if big else "bytes_quad"] += b
            if not big:
                acc["bytes_quad2" if 32 <= (w // 4) * (h // 4) <= 128 else "bytes_quad1"] += b
            if big:
                acc["bytes_ctu" if w == h else "bytes_half"] += b
                if w != h:  # 128x64 (affine_me_half2w) / 64x128 (affine_me_half2h)
                    acc["bytes_half_w" if w > h else "bytes_half_h"] += b
    acc["bytes"] = acc["bytes_quad"] + acc["bytes_big"]
    return acc
