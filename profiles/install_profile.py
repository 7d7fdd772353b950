"""Copy a run_profile.sh output (gpurun_out/prof_<config>) into the committed
records the bench line and DESIGN read: profiles/pmc_<config>.json and the
round's kernel stats, prediction count and profiled bench line.
    python3 profiles/install_profile.py <round tag, e.g. r05> <config>..."""
import json
import os
import shutil
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
for c in sys.argv[2:]:
    O = os.path.join(R, "gpurun_out", f"prof_{tag}_{c}")  # run_profile.sh <tag>_<config> <config>
    if not os.path.isdir(O):
        O = os.path.join(R, "gpurun_out", f"prof_{c}")
    s = json.load(open(os.path.join(O, "summary.json")))
    s["source"] = f"{os.path.relpath(O, R)} (profiles/run_profile.sh, {tag})"
    json.dump(s, open(os.path.join(R, "profiles", f"pmc_{c}.json"), "w"), indent=1)
    shutil.copy(os.path.join(O, "trace", "run_kernel_stats.csv"), os.path.join(R, "profiles", f"{tag}_{c}_kernel_stats.csv"))
    shutil.copy(os.path.join(O, "count.json"), os.path.join(R, "profiles", f"{tag}_{c}_pred_count.json"))
    shutil.copy(os.path.join(O, "bench.json"), os.path.join(R, "profiles", f"{tag}_{c}_profile_bench.json"))
    print("installed", c)
