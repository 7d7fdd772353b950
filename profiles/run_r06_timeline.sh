#!/bin/bash
# round 6: the c2 step's kernel timeline under each packing / stream placement
# (rocprofv3 kernel trace, profiles/step_timeline.py), then SQ passes of the
# default build at c2 and c4 (VALU instructions per kernel).  gpurun only.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
O=$R/gpurun_out/r06_tl; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
L=$R/vvc-affine-gpu_amd/lib
for v in ${VARIANTS:-default nosplit q1side}; do
  lib=$L/libvame_$v.so; [ $v = default ] && lib=$L/libvame.so
  VAME_LIB=$lib VAME_BENCH_KTIMING=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
      -d $O/trace_$v -o run -- python3 $R/bench.py --no-cpu-baseline --fs-frames 0 --no-spans --steps 100 --warmup 10 \
      > $O/tr_$v.json 2> $O/tr_$v.err || exit 1
  T=$(find $O/trace_$v -name "*kernel_trace.csv" -print -quit)
  echo "== $v"; python3 $R/profiles/step_timeline.py $T --last 80 | tee $O/timeline_$v.txt
  rm -f $T
done
for c in ${SQCFG:-c2 c4}; do
  bash $R/profiles/run_sq_lib.sh r06sq_$c $L/libvame.so --no-spans --config $c || exit 1
done
echo tl-done
