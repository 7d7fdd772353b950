#!/bin/bash
# End-to-end C5 (BASELINE configs[4]: 3840x2160 QP32, 240 frames) on one
# MI355X (gpurun only): CSV inputs in the reference layout, then
#   1. the `vame` CLI (one process, the drop-in for ./main): READ_CSV_TIME,
#      TOTAL_EXEC_TIME, LOG_WRITE_TIME, OVERALL for the whole sequence;
#   2. `vame.distrun --gpus 8 --rank-only K` for K = 0 and 7: one rank's share
#      of the 8-GPU frame shard alone on this GPU and its 16-CPU share --
#      ingest of its frames, its kernel time and the formatting of its own
#      log block, under the default log path and under --shard-logs (part
#      files written as it goes), twice each: what each rank of an 8-GPU node does;
#   3. the 40 files of a 2-rank distrun (gloo, one GPU) compared
#      byte for byte with the CLI's.
#   bash profiles/run_e2e_c5.sh <tag> [frames]
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=${1:-e2e_c5}; F=${2:-240}
O=$R/gpurun_out/$TAG
mkdir -p $O
T=$(mktemp -d /tmp/vame_c5.XXXXXX)
trap 'rm -rf $T' EXIT
export PYTHONPATH=$R/vvc-affine-gpu_amd
python3 -c "
import time, os
from vame.synth import synth_sequence, write_csv
t = time.time()
o, r = synth_sequence(3840, 2160, $F, 32)
write_csv('$T/orig.csv', o); write_csv('$T/recon.csv', r)
print('csv written in %.1f s, %d + %d bytes' % (time.time() - t, os.path.getsize('$T/orig.csv'), os.path.getsize('$T/recon.csv')), flush=True)
" | tee $O/inputs.txt
mkdir -p $T/cli
for run in 1 2; do  # the first run pages the CSVs in
  rm -f $T/cli/*
  timeout -k 10 400 $R/vvc-affine-gpu_amd/bin/vame -f $F -s 3840x2160 -q 32 -o $T/orig.csv \
      -r $T/recon.csv -l $T/cli/log > $O/cli_run$run.txt
  echo "cli run $run: $(grep -E 'TOTAL_EXEC|OVERALL|READ_CSV|LOG_WRITE|LOG_BYTES' $O/cli_run$run.txt | tr '\n' ' ')"
done
echo "cli logs: $(ls $T/cli | wc -l) files, $(du -sb $T/cli | cut -f1) bytes"
for rep in 1 2; do
for K in 0 7; do
  for P in place shard; do  # the default log path, then --shard-logs (part files as it goes)
    X=""; [ $P = shard ] && X="--shard-logs"
    mkdir -p $T/r$K
    timeout -k 10 400 python3 -m vame.distrun -f $F -s 3840x2160 -q 32 -o $T/orig.csv -r $T/recon.csv \
        -l $T/r$K/log --gpus 8 --rank-only $K $X > $O/rank${K}_of8_${P}_$rep.txt
    echo "rank $K of 8, $P, run $rep:"
    grep -E "EXEC|OVERALL|READ_CSV|LOG_WRITE|LOG_BYTES|DISTRUN" $O/rank${K}_of8_${P}_$rep.txt
    rm -rf $T/r$K
  done
done
done
if [ "$F" -le 60 ]; then
  mkdir -p $T/d2
  VAME_DIST_BACKEND=gloo timeout -k 10 600 python3 -m vame.distrun -f $F -s 3840x2160 -q 32 -o $T/orig.csv \
      -r $T/recon.csv -l $T/d2/log --gpus 2 > $O/distrun2_shard.txt
  grep -E "EXEC|OVERALL|READ_CSV|LOG_WRITE|LOG_MERGE|LOG_BYTES" $O/distrun2_shard.txt
  for f in $(ls $T/cli); do cmp -s $T/cli/$f $T/d2/$f || { echo "MISMATCH $f"; exit 1; }; done
  echo "distrun --gpus 2: $(ls $T/d2 | wc -l) files byte-identical to the CLI's"
  mkdir -p $T/d2s
  VAME_DIST_BACKEND=gloo timeout -k 10 600 python3 -m vame.distrun -f $F -s 3840x2160 -q 32 -o $T/orig.csv \
      -r $T/recon.csv -l $T/d2s/log --gpus 2 --shard-logs --merge-parts > $O/distrun2_parts.txt
  grep -E "OVERALL|LOG_MERGE" $O/distrun2_parts.txt
  for f in $(ls $T/cli); do cmp -s $T/cli/$f $T/d2s/$f || { echo "MISMATCH $f (--shard-logs)"; exit 1; }; done
  echo "distrun --gpus 2 --shard-logs --merge-parts: $(ls $T/d2s | wc -l) files byte-identical to the CLI's"
fi
echo e2e-c5-done
