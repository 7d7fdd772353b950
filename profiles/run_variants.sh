#!/bin/bash
# Bench several experiment builds (make variant NAME=x DEFS=...) back to back.
# gpurun only.   bash profiles/run_variants.sh "base x y" [bench args]
# "base" = lib/libvame.so.  Prints ms/step and the two kernels' average launch times.
R="$(cd "$(dirname "$0")/.." && pwd)"
O=$R/gpurun_out/variants
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${1:-base}; do
  shift_done=1
  if [ "$v" = base ]; then lib=$R/vvc-affine-gpu_amd/lib/libvame.so; else lib=$R/vvc-affine-gpu_amd/lib/libvame_$v.so; fi
  VAME_LIB=$lib timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-spans "${@:2}" > $O/$v.out 2> $O/$v.err
  rc=$?
  case $rc in 124|134|137|139) echo "$v crash-like exit $rc, stopping"; exit $rc;; esac
  tail -n 1 $O/$v.out | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],4), 'quad', round(d['roofline']['avg_launch_ms'],4), 'ctu', round(d['roofline']['affine_me_ctu']['avg_launch_ms'],4))" || echo "$v rc=$rc"
done
echo variants-done
