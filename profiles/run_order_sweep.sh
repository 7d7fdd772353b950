#!/bin/bash
# Block-order sweep (gpurun only): CTU-chunk group size (VAME_GROUP_COMBOS) and
# XCD slot order (VAME_XCD_ORDER) at c4 and c2: the bench line and one
# FETCH_SIZE pass per variant.   bash profiles/run_order_sweep.sh <tag> "G:O G:O ..."
set -uo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=${1:-order}; VARS=${2:-"408:1 408:0 272:1 136:1"}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in $VARS; do
  G=${v%%:*}; X=${v##*:}
  export VAME_GROUP_COMBOS=$G VAME_XCD_ORDER=$X
  for cfg in c2 c4; do
    timeout -k 10 300 python3 $R/bench.py --config $cfg --no-cpu-baseline --no-spans \
        > $O/${cfg}_g${G}_x${X}.json 2> $O/${cfg}_g${G}_x${X}.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['roofline']['frac'],4), d['roofline']['avg_launch_ms'], d['roofline']['affine_me_ctu']['avg_launch_ms'], d['gather']['check']['byte_identical'])" $O/${cfg}_g${G}_x${X}.json ${cfg}_g${G}_x${X}
  done
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_g${G}_x${X} -o run -- \
      python3 $R/bench.py --config c4 --no-cpu-baseline --no-spans --steps 2 --warmup 1 > $O/fetch_g${G}_x${X}.log 2>&1 || exit 1
  python3 - $O/fetch_g${G}_x${X} <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0].split("<")[0]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print("  ", k, "FETCH bytes/launch (x2 corrected) %.3f GB" % (2 * 1024 * sum(v) / len(v) / 1e9), "n", len(v))
PY
done
echo sweep-done
