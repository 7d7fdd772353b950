#!/bin/bash
# End-to-end timing of the `vame` CLI (the drop-in for the reference's ./main):
# CSV ingest, kernel time and the 40-file decision-log write, for BASELINE
# configs[2] (C3: 1920x1080 QP32, 30 frames, 2+3 CP) and configs[3] at QP32
# (C4: 3840x2160, 30 frames), inputs written in the reference CSV layout
# (main.cpp:313-328) by the native generator.  gpurun only.
#   bash profiles/run_e2e.sh <tag>
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=${1:-e2e}
O=$R/gpurun_out/$TAG
mkdir -p $O
T=$(mktemp -d /tmp/vame_e2e.XXXXXX)
trap 'rm -rf $T' EXIT
for cfg in "c3 1920 1080" "c4 3840 2160"; do
  set -- $cfg
  name=$1; W=$2; H=$3
  R=$R python3 -c "
import sys, time, os
sys.path.insert(0, os.path.join('$R', 'vvc-affine-gpu_amd'))
from vame.synth import synth_sequence, write_csv
t = time.time()
o, r = synth_sequence($W, $H, 30, 32)
write_csv('$T/orig.csv', o); write_csv('$T/recon.csv', r)
print('csv written in %.1f s, %d + %d bytes' % (time.time() - t, os.path.getsize('$T/orig.csv'), os.path.getsize('$T/recon.csv')))
"
  mkdir -p $T/logs
  # two runs: the first pages the CSVs in (cold file cache on a fresh box)
  for run in 1 2; do
    rm -f $T/logs/*
    timeout -k 10 300 $R/vvc-affine-gpu_amd/bin/vame -f 30 -s ${W}x${H} -q 32 -o $T/orig.csv \
        -r $T/recon.csv -l $T/logs/log > $O/${name}_run$run.txt
  done
  echo "== $name ($W x $H, 30 frames, QP32, 2+3 CP): $(ls $T/logs | wc -l) log files, $(du -sb $T/logs | cut -f1) bytes"
  grep -E "_EXEC|OVERALL|READ_CSV|LOG_WRITE|LOG_BYTES" $O/${name}_run2.txt
  rm -rf $T/logs $T/orig.csv $T/recon.csv
done
echo e2e-done
