#!/bin/bash
# A/B timing of library builds (gpurun only): for each lib and each bench
# config, one bench line (no CPU baseline, no spans); prints ms/step, the
# quadrant / 128-class launch times and frac.
#   bash profiles/run_ab.sh <tag> "<lib names>" "<config args>;<config args>;..."
set -uo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=$1; LIBS=$2; CFGS=$3
O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra CS <<< "$CFGS"
for rep in 1 2; do
for c in "${CS[@]}"; do
  for lib in $LIBS; do
    VAME_LIB=$R/vvc-affine-gpu_amd/lib/$lib.so timeout -k 10 300 python3 $R/bench.py $c --no-cpu-baseline --no-spans > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('$lib', '$c', round(d['ms_per_step'],3), 'quad', round(d['roofline']['avg_launch_ms'],3), 'ctu', round(d['roofline']['affine_me_ctu']['avg_launch_ms'],3), 'frac', round(d['roofline']['frac'],4))"
  done
done
done
echo ab-done
