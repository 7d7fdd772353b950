#!/bin/bash
# round 6 records: the profiles bench.py's roofline reads (profiles/pmc_<config>.json
# inputs) for the given configs, each a run_profile.sh pass.  gpurun only.
#   bash profiles/run_r06_prof.sh c2 c3     (c5: PSTEPS=1 PWARM=0 CLEAN=1)
set -o pipefail
for c in "$@"; do
  if [ $c = c5 ]; then
    PSTEPS=1 PWARM=0 CLEAN=1 bash profiles/run_profile.sh r06_$c $c --steps 2 --warmup 1 > gpurun_out/prof_r06_$c.log 2>&1 || exit 1
  elif [ $c = c4 ]; then
    CLEAN=1 PSTEPS=3 PWARM=1 bash profiles/run_profile.sh r06_$c $c > gpurun_out/prof_r06_$c.log 2>&1 || exit 1
  else
    bash profiles/run_profile.sh r06_$c $c > gpurun_out/prof_r06_$c.log 2>&1 || exit 1
  fi
  tail -2 gpurun_out/prof_r06_$c.log
done
echo prof-done
