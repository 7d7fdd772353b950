#!/usr/bin/env python3
"""Executed fraction of the algorithmic sub-block predictions (the exact early
exit of vame_kernel.h skips the rest), per kernel class, on one step of a
bench config, with the instrumentation build (make count):

    VAME_LIB=vvc-affine-gpu_amd/lib/libvame_count.so python3 profiles/count_preds.py --config c2

Prints one JSON object; pmc_summary.py folds it into profiles/pmc_<config>.json
(bench.py reports it as roofline.executed_pred_frac)."""
import argparse
import ctypes
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "vvc-affine-gpu_amd"))
sys.path.insert(0, R)

import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from vame import _lib  # noqa: E402
from vame.engine import Engine  # noqa: E402
from vame.metrics import pair_accounting  # noqa: E402
from vame.seqrun import ShardRun  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--qp", type=int, default=None)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--rank-only", type=int, default=0, help="count rank K's block of a --gpus N job")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    qp = cfg["qp"] if args.qp is None else args.qp
    L = _lib.lib()
    if not hasattr(L, "vame_debug_pred_count"):
        raise SystemExit("VAME_LIB must point at the instrumentation build (make count)")
    L.vame_debug_pred_count.argtypes = [ctypes.c_void_p, ctypes.c_int]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = Engine(cfg["W"], cfg["H"], 0)
    n_pairs = None
    if cfg["scaling"] == "weak":  # bench.py's weak-scaling prefix of the sequence
        from vame.shard import frames_for_pairs, sequence_pairs
        n_pairs = sequence_pairs(cfg["frames"]) * args.gpus
    frames = cfg["frames"] if n_pairs is None else frames_for_pairs(n_pairs)
    run = ShardRun(eng, cfg["W"], cfg["H"], qp, frames, cfg["modes"], args.gpus, args.rank_only, dev,
                   n_pairs=n_pairs)
    cnt = (ctypes.c_ulonglong * 20)()
    L.vame_debug_pred_count(cnt, 1)
    run.step()
    torch.cuda.synchronize()
    L.vame_debug_pred_count(cnt, 1)
    acc = pair_accounting(cfg["W"], cfg["H"], (2, 3) if cfg["modes"] & 2 else (2,))
    alg_q, alg_b = acc["sb_pred_quad"] * run.pairs, acc["sb_pred_big"] * run.pairs
    out = {"config": args.config, "qp": qp, "pairs": run.pairs, "rank": [args.rank_only, args.gpus],
           "executed_quad": cnt[0], "algorithmic_quad": alg_q, "executed_pred_frac_quad": cnt[0] / alg_q,
           "executed_ctu": cnt[1], "algorithmic_ctu": alg_b, "executed_pred_frac_ctu": cnt[1] / alg_b,
           "executed_pred_frac": (cnt[0] + cnt[1]) / (alg_q + alg_b),
           # executed predictions whose 9x9 window left the staged tile (clamped global loads)
           "outside_tile_frac_quad": (cnt[2] + cnt[3]) / max(cnt[0], 1),
           "outside_tile_frac_ctu": (cnt[4] + cnt[5]) / max(cnt[1], 1),
           "outside_tile_quad_2cp_3cp": [cnt[2], cnt[3]], "outside_tile_ctu_2cp_3cp": [cnt[4], cnt[5]],
           # of the outside windows, those a margin wider by 4 / 8 / 16 px would hold
           "outside_held_by_wider_margin_quad": [cnt[6], cnt[7], cnt[8]],
           "outside_held_by_wider_margin_ctu": [cnt[9], cnt[10], cnt[11]],
           # lane use of the prediction steps: predictions run / 64 lane slots of
           # the waves that ran the step; and the same over the waves holding
           # several CUs (lanes of settled CUs idle while the wave iterates)
           "lane_use_quad": cnt[0] / max(cnt[12], 1), "lane_use_ctu": cnt[1] / max(cnt[13], 1),
           "multi_cu_wave_slots_frac_quad": cnt[14] / max(cnt[12], 1),
           "multi_cu_wave_lane_use_quad": cnt[16] / max(cnt[14], 1)}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
