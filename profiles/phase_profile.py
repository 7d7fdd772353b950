#!/usr/bin/env python3
"""Per-phase shader-clock breakdown of both kernels (profiling-only build).

    make phase && VAME_LIB=vvc-affine-gpu_amd/lib/libvame_phase.so \\
        python profiles/phase_profile.py [--config c2] [--steps 5]

Runs bench.py's workload, then prints, per kernel, the share of wave-clock
spent in each phase (summed over all waves: it weights phases by how long
waves sit in them, including barrier / wave-sync waits at the phase's end).
Since the quadrant items run several tasks (round 4), the timing registers
push this build's 3-CP quadrant instances past 128 VGPRs (3 waves per SIMD
instead of 4): their shares describe a slower kernel; the 2-CP-only (c2)
instance keeps 4.
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-affine-gpu_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PHASES = ("stage", "predict", "cost", "gradient+reduce", "solve", "pass tail")
# slots [kernel][phase + 6 * (3-CP pass)], 12 / 13: SIMD-slot use


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    from bench import CONFIGS
    from vame import _lib
    from vame.engine import Engine
    from vame.seqrun import ShardRun
    from vame.shard import frames_for_pairs, sequence_pairs
    cfg = CONFIGS[args.config]
    W, H, qp, nf, modes = cfg["W"], cfg["H"], cfg["qp"], cfg["frames"], cfg["modes"]
    L = _lib.lib()
    fn = L.vame_debug_phase_cycles
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    eng = Engine(W, H, 0)
    # bench.py's step at N = 1: the config's pairs in one vame_affine_me_batch call
    n_pairs = sequence_pairs(nf) if cfg["scaling"] == "weak" else None
    run = ShardRun(eng, W, H, qp, frames_for_pairs(n_pairs) if n_pairs else nf, modes, 1, 0, dev,
                   n_pairs=n_pairs, streams=cfg["scaling"] == "weak")
    buf = np.zeros(48, np.uint64)
    run.step()
    torch.cuda.synchronize()
    fn(buf.ctypes.data, 1)
    for _ in range(args.steps):
        run.step()
    torch.cuda.synchronize()
    fn(buf.ctypes.data, 1)
    out = {}
    for k, name in enumerate(("affine_me_quad", "affine_me_ctu", "affine_me_half")):
        v = buf[16 * k:16 * k + 12].astype(np.float64)
        tot = v.sum()
        if not tot:
            continue
        e = {}
        for off, pas in ((0, "2cp"), (6, "3cp")):
            e[pas] = {p: round(float(x / tot), 4) for p, x in zip(PHASES, v[off:off + 6])}
        e["wave_clock_total"] = float(tot)
        slot, life = float(buf[16 * k + 12]), float(buf[16 * k + 13])
        e["simd_slot_use"] = round(life / slot, 4) if slot else 0.0
        out[name] = e
    print(json.dumps({"config": args.config, "steps": args.steps, "pairs_per_step": run.pairs,
                      "phases": out}, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
