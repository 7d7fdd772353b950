#!/usr/bin/env python3
"""Per-phase shader-clock breakdown of both kernels (profiling-only build).

    make phase && VAME_LIB=vvc-affine-gpu_amd/lib/libvame_phase.so \\
        python profiles/phase_profile.py [--config c2] [--steps 5]

Runs bench.py's workload, then prints, per kernel, the share of wave-clock
spent in each phase (summed over all waves: it weights phases by how long
waves sit in them, including barrier / wave-sync waits at the phase's end).
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
    from vame import synth, _lib
    from vame.engine import Engine
    from vame.hostlogic import lambda_for_poc, ref_list
    cfg = CONFIGS[args.config]
    W, H, qp, nf, modes = cfg["W"], cfg["H"], cfg["qp"], cfg["frames"], cfg["modes"]
    L = _lib.lib()
    fn = L.vame_debug_phase_cycles
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    orig, recon = synth.synth_sequence(W, H, nf, qp, seed=0x5EED)
    d_o = [torch.from_numpy(orig[k].view(np.int16)).to(dev) for k in range(nf)]
    d_r = [torch.from_numpy(recon[k].view(np.int16)).to(dev) for k in range(nf)]
    eng = Engine(W, H, 0)
    buf = np.zeros(32, np.uint64)

    def run():
        for poc in range(1, nf + 1):
            eng.affine_me_poc(d_o[poc - 1], [d_r[r] for r in ref_list(poc)], lambda_for_poc(qp, poc), modes)
        torch.cuda.synchronize()

    run()
    fn(buf.ctypes.data, 1)
    for _ in range(args.steps):
        run()
    fn(buf.ctypes.data, 1)
    out = {}
    for k, name in enumerate(("affine_me_quad", "affine_me_ctu")):
        v = buf[16 * k:16 * k + 12].astype(np.float64)
        tot = v.sum()
        e = {}
        for off, pas in ((0, "2cp"), (6, "3cp")):
            e[pas] = {p: round(float(x / tot), 4) if tot else 0.0 for p, x in zip(PHASES, v[off:off + 6])}
        e["wave_clock_total"] = float(tot)
        slot, life = float(buf[16 * k + 12]), float(buf[16 * k + 13])
        e["simd_slot_use"] = round(life / slot, 4) if slot else 0.0
        out[name] = e
    print(json.dumps({"config": args.config, "steps": args.steps, "phases": out}, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
