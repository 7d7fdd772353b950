#!/bin/bash
# Block-order sweep (gpurun only): CTU-chunk group sizes of the quadrant and
# 128-class kernels (VAME_GROUP_COMBOS / VAME_GROUP_COMBOS_BIG) and the XCD
# dealing (VAME_XCD_ORDER) at c2 and c4: the bench line and one FETCH_SIZE pass
# per variant.   bash profiles/run_order_sweep.sh <tag> "Gq:Gb:X ..."
set -uo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=${1:-order}; VARS=${2:-"408:408:0"}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in $VARS; do
  IFS=: read G GB X <<< "$v"
  export VAME_GROUP_COMBOS=$G VAME_GROUP_COMBOS_BIG=$GB VAME_XCD_ORDER=$X
  n=g${G}_b${GB}_x${X}
  for cfg in c2 c4; do
    timeout -k 10 300 python3 $R/bench.py --config $cfg --no-cpu-baseline --fs-frames 0 --no-spans \
        > $O/${cfg}_$n.json 2> $O/${cfg}_$n.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'ms/step', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4), 'quad', round(d['roofline']['avg_launch_ms'],3), 'ctu', round(d['roofline']['affine_me_ctu']['avg_launch_ms'],3), d['gather']['check']['byte_identical'])" $O/${cfg}_$n.json ${cfg}_$n
  done
  [ -n "${NOFETCH:-}" ] && continue
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$n -o run -- \
      python3 $R/bench.py --config c4 --no-cpu-baseline --fs-frames 0 --no-spans --steps 2 --warmup 1 > $O/fetch_$n.log 2>&1 || exit 1
  python3 - $O/fetch_$n <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "vame::" in k:
            acc[k.split("(")[0].split("<")[0]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print("  ", k, "c4 FETCH GB/launch (x2 corrected) %.3f" % (2 * 1024 * sum(v) / len(v) / 1e9), "n", len(v))
PY
done
echo sweep-done
