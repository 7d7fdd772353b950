#!/bin/bash
# GPU-box profiling recipe (gpurun): bench line, rocprofv3 kernel trace + stats,
# then the two PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs,
# MI355X_MICROARCH.md §HBM) and their per-kernel summary.
#   bash profiles/run_profile.sh <tag> [bench args...]
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=${1:-c2}; shift || true
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py "$@" > $O/bench.json 2> $O/bench.err
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline > $O/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch -o run -- \
    python3 $R/bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_write -o run -- \
    python3 $R/bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1
python3 $R/profiles/pmc_summary.py $O $O/summary.json > /dev/null
echo profile-done
