#!/bin/bash
# A/B of the `vame` CLI end to end (gpurun only): synthetic CSVs once, then the
# CLI under each "name:VAR=v,..." setting, interleaved over REPS repetitions.
#   bash profiles/run_cli_ab.sh <tag> <WxH> <frames> "<name>:<vars>" ...
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=$1; SIZE=$2; F=$3; shift 3
W=${SIZE%x*}; H=${SIZE#*x}
O=$R/gpurun_out/$TAG; mkdir -p $O
T=$(mktemp -d /tmp/vame_cli.XXXXXX)
trap 'rm -rf $T' EXIT
export PYTHONPATH=$R/vvc-affine-gpu_amd
python3 -c "
from vame.synth import synth_sequence, write_csv
o, r = synth_sequence($W, $H, $F, 32)
write_csv('$T/orig.csv', o); write_csv('$T/recon.csv', r)
" || exit 1
mkdir -p $T/log
for rep in $(seq 1 ${REPS:-2}); do
  for s in "$@"; do
    name=${s%%:*}; vars=${s#*:}
    rm -f $T/log/*
    env ${vars//,/ } timeout -k 10 300 $R/vvc-affine-gpu_amd/bin/vame -f $F -s $SIZE -q 32 -o $T/orig.csv \
        -r $T/recon.csv -l $T/log/x > $O/$name.$rep.txt || { echo "$name failed"; exit 1; }
    echo "$name $rep: $(grep -E 'TOTAL_EXEC|OVERALL|READ_CSV|LOG_WRITE' $O/$name.$rep.txt | tr '\n' ' ')"
  done
done
echo cli-ab-done
