"""Where each kernel class's waves spend their time, phase by phase.

Runs a bench config's step through the profiling-only build
`vvc-affine-gpu_amd/lib/libvame_phase.so` (`make phase`: every wave sums the
shader clock per phase, vame_kernel.h VAME_PHASE_TIMING) and prints, per
kernel class and pass, the share of wave cycles in each phase -- staging,
prediction (+ SATD), cost, gradient sums, equation reduction, solve + CPMV
update, results -- where a phase includes the wait at the barrier that ends it; the
SIMD-slot use (wave lifetimes / waves x workgroup lifetime) and the mean
workgroup lifetime in cycles.  The counters cost ~10 % of wave cycles; the
shares, not the times, are the result.
  VAME_LIB=vvc-affine-gpu_amd/lib/libvame_phase.so python3 profiles/phase_profile.py [c2|c3|c4] [steps]
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "vvc-affine-gpu_amd"))

KINDS = ["affine_me_quad", "affine_me_ctu", "affine_me_half", "affine_me_ctu2", "affine_me_half2w",
         "affine_me_half2h"]
PHASES = ["stage", "predict", "cost", "gradient", "solve", "tail", "reduce"]
NP = len(PHASES)
SLOTS = 2 * NP + 4


def main():
    import torch

    import bench
    from vame import _lib
    from vame.engine import Engine
    from vame.seqrun import ShardRun
    from vame.shard import frames_for_pairs, sequence_pairs
    if "libvame_phase" not in _lib.LIB_PATH:
        sys.exit("set VAME_LIB to the phase build (make phase)")
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    cfg = bench.CONFIGS[cfg_name]
    L = _lib.lib()
    L.vame_debug_phase_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * (6 * SLOTS))()
    dev = torch.device("cuda", 0)
    n_pairs = sequence_pairs(cfg["frames"])
    eng = Engine(cfg["W"], cfg["H"], 0)
    run = ShardRun(eng, cfg["W"], cfg["H"], cfg["qp"], frames_for_pairs(n_pairs), cfg["modes"], 1, 0, dev,
                   n_pairs=n_pairs, streams=True)
    for _ in range(3):
        run.step()
    torch.cuda.synchronize()
    _lib.check(L.vame_debug_phase_cycles(buf, 1))
    for _ in range(steps):
        run.step()
    torch.cuda.synchronize()
    _lib.check(L.vame_debug_phase_cycles(buf, 1))
    out = {"config": cfg_name, "steps": steps, "env": {k: v for k, v in os.environ.items() if k.startswith("VAME_")},
           "kernels": {}}
    for k, name in enumerate(KINDS):
        v = list(buf[SLOTS * k:SLOTS * k + SLOTS])
        total = sum(v[:2 * NP])
        if not total:
            continue
        rec = {"wave_cycles": total}
        for p in range(2):
            part = v[NP * p:NP * p + NP]
            if sum(part):
                rec["pass%dcp" % (p + 2)] = {ph: round(c / total, 4) for ph, c in zip(PHASES, part)}
        w = 2 * NP
        rec["simd_slot_use"] = round(v[w + 1] / v[w], 4) if v[w] else None
        rec["workgroups_per_step"] = v[w + 2] / steps
        rec["mean_wg_lifetime_cycles"] = round(v[w + 3] / v[w + 2]) if v[w + 2] else None
        out["kernels"][name] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
