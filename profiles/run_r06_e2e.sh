#!/bin/bash
# round 6: end to end C5 (the CLI, one rank of 8 under both log paths), the
# 24-frame byte-identity check of the 2-rank paths, then the frame-shard
# forecast.  gpurun only.
set -o pipefail
mkdir -p gpurun_out
bash profiles/run_e2e_c5.sh e2e_r06 240 > gpurun_out/e2e_r06.log 2>&1 || { tail -20 gpurun_out/e2e_r06.log; exit 1; }
grep -E "cli run|rank|OVERALL|DISTRUN" gpurun_out/e2e_r06.log | cut -c1-200
bash profiles/run_e2e_c5.sh e2e_r06_24 24 > gpurun_out/e2e_r06_24.log 2>&1 || { tail -20 gpurun_out/e2e_r06_24.log; exit 1; }
tail -6 gpurun_out/e2e_r06_24.log
timeout -k 10 900 python3 profiles/scale_forecast.py > gpurun_out/r06_scale_forecast.txt 2>&1 || { tail -20 gpurun_out/r06_scale_forecast.txt; exit 1; }
grep -v "^{" gpurun_out/r06_scale_forecast.txt | tail -30
echo r06-e2e-done
