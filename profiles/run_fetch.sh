#!/bin/bash
# FETCH_SIZE pass for one library build (gpurun only): bash profiles/run_fetch.sh <tag> <lib.so>
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=$1; LIB=$(readlink -f $2); shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
VAME_LIB=$LIB timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit $?
python3 - $O <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/pmc_fetch/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(k, "FETCH_SIZE KiB/launch (raw)", round(sum(v) / len(v)))
PY
