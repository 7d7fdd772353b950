#!/bin/bash
# A/B of engine / bench environment knobs on one build (gpurun only): the bench
# line under each setting, interleaved over REPS repetitions, then ms/step and
# the per-kernel dispatch averages per setting.
#   bash profiles/run_bench_env.sh <tag> "<name>:<VAR=v,VAR=v>" ... [-- bench args]
# e.g. run_bench_env.sh ktiming "both:VAME_BENCH_KTIMING=1" "quad:VAME_BENCH_KTIMING=2" \
#          "off:VAME_BENCH_KTIMING=0" -- --no-spans
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=$1; shift
SETS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do SETS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
O=$R/gpurun_out/$TAG; mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for s in "${SETS[@]}"; do
    name=${s%%:*}; vars=${s#*:}
    env ${vars//,/ } timeout -k 10 ${TMO:-300} python3 $R/bench.py --no-cpu-baseline --fs-frames 0 "$@" \
        > $O/$name.$rep.json 2> $O/$name.$rep.err || { tail -5 $O/$name.$rep.err; exit 1; }
    python3 - "$O/$name.$rep.json" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]
extra = {k: round(v["avg_launch_ms"], 4) for k, v in r.items() if isinstance(v, dict) and "avg_launch_ms" in v}
print(sys.argv[2], "ms/step", round(d["ms_per_step"], 4), "quad", round(r["avg_launch_ms"], 4), extra,
      "parity", d.get("parity_sample", {}).get("bit_exact"))
PY
  done
done
echo env-done
