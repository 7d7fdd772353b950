#!/usr/bin/env python3
"""Phase split of a kernel's dynamic VALU instructions from the VAME_DUP
builds' SQ passes (profiles/run_dup_sq.sh: gpurun_out/<tag>_dup<N>/summary.txt;
a duplicated phase adds exactly its own instructions).
   python3 profiles/dup_split.py <tag> <kernel substring>"""
import glob
import os
import re
import sys

PHASES = {1: "prediction (predict_sb: orig rows, MV, window, filter, SATD)", 2: "gradient (grad_sb)",
          4: "equation values + reduction", 16: "solve (system build, elimination, back-substitution)",
          64: "tile staging round trip", 128: "MV field (mv_field, spread test)",
          256: "extended rows (DPP neighbour columns, edge-row stores / reads)", 512: "SATD segment sum",
          1024: "cost / best (lane 7)", 2048: "CPMV update (scaleDeltaMvs, clamp, clip, rate bits, flags)"}


def valu(tag, n, kern):
    f = os.path.join("gpurun_out", f"{tag}_dup{n}", "summary.txt")
    cur, out = None, {}
    for line in open(f):
        if not line.startswith(" "):
            cur = line.strip()
        elif "SQ_INSTS_VALU" in line:
            out[cur] = float(line.split()[-1])
    return next(v for k, v in out.items() if kern in k)


def main():
    tag, kern = sys.argv[1], sys.argv[2]
    base = valu(tag, 0, kern)
    print(f"{kern} ({tag}): SQ_INSTS_VALU per launch {base:,.0f}")
    rest = base
    for n, name in PHASES.items():
        d = valu(tag, n, kern) - base
        rest -= d
        print(f"  dup{n:<5d} {name:62s} {d / 1e6:8.1f} M  {d / base:6.1%}")
    print(f"  {'':8s} {'everything else (task switch / claim, init, results, loop, live checks)':62s} "
          f"{rest / 1e6:8.1f} M  {rest / base:6.1%}")


if __name__ == "__main__":
    main()
