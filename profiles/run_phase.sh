#!/bin/bash
# Phase shares per kernel class (gpurun only): profiles/phase_profile.py on the
# phase build under each "name:VAR=v,VAR=v" setting.
#   bash profiles/run_phase.sh <tag> <config> "<name>:<vars>" ...
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=$1; CFG=$2; shift 2
O=$R/gpurun_out/$TAG; mkdir -p $O
for s in "$@"; do
  name=${s%%:*}; vars=${s#*:}
  env ${vars//,/ } VAME_LIB=$R/vvc-affine-gpu_amd/lib/libvame_phase.so timeout -k 10 ${TMO:-240} \
      python3 $R/profiles/phase_profile.py $CFG ${STEPS:-20} > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  echo "== $name"; cat $O/$name.json
done
echo phase-done
