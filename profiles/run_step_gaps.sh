#!/bin/bash
# Step-boundary idle time of the c2 bench step under each
# engine stream mode: a rocprofv3 kernel trace of bench.py --no-spans, the
# gaps between one step's last kernel and the next step's first
# (step_gaps.py), and an untraced bench line per mode.
#   bash profiles/run_step_gaps.sh <tag> [modes...]     (modes: VAME_STREAMS values, default "2 1")
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=${1:-gaps}; shift || true
MODES=${*:-2 1}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for M in $MODES; do
  echo "[gaps] VAME_STREAMS=$M bench"
  VAME_STREAMS=$M timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --fs-frames 0 > $O/bench_s$M.json 2> $O/bench_s$M.err
  echo "[gaps] VAME_STREAMS=$M trace"
  VAME_STREAMS=$M VAME_BENCH_KTIMING=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
      -d $O/trace_s$M -o run -- python3 $R/bench.py --no-cpu-baseline --fs-frames 0 --no-spans --steps 100 --warmup 10 \
      > $O/tr_s$M.json 2> $O/tr_s$M.err
  T=$(find $O/trace_s$M -name "*kernel_trace.csv" -print -quit)
  python3 $R/profiles/step_gaps.py $T --last 100 | tee $O/gaps_s$M.txt
done
echo gaps-done
