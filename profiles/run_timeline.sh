#!/bin/bash
# Kernel timeline of the bench step under each "name:VAR=v,..." setting
# (gpurun only): a rocprofv3 kernel trace of bench.py --no-spans and, per
# kernel, its median start / end within the step (step_gaps.py).
#   bash profiles/run_timeline.sh <tag> "<name>:<vars>" ... [-- bench args]
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=$1; shift
SETS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do SETS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for s in "${SETS[@]}"; do
  name=${s%%:*}; vars=${s#*:}
  env ${vars//,/ } VAME_BENCH_KTIMING=0 timeout -k 10 ${TMO:-300} rocprofv3 --kernel-trace --output-format csv \
      -d $O/trace_$name -o run -- python3 $R/bench.py --no-cpu-baseline --fs-frames 0 --no-spans --steps 100 --warmup 10 "$@" \
      > $O/tr_$name.json 2> $O/tr_$name.err || { tail -5 $O/tr_$name.err; exit 1; }
  T=$(find $O/trace_$name -name "*kernel_trace.csv" -print -quit)
  echo "== $name"
  python3 $R/profiles/step_gaps.py $T --last 80 --skip 20 | tee $O/timeline_$name.txt
done
echo timeline-done
