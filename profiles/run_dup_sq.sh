#!/bin/bash
# Dynamic VALU instruction split by phase: one SQ pass (SQ_INSTS_VALU, ...)
# per build -- the product library and the VAME_DUP builds that run one phase
# twice (make variant NAME=dupN DEFS=-DVAME_DUP=N; a duplicated phase adds
# exactly its own instructions, the trajectories are unchanged).  gpurun only.
#   bash profiles/run_dup_sq.sh <tag> "<dup ids>" [bench args]
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=$1; IDS=$2; shift 2
for v in 0 $IDS; do
  if [ "$v" = 0 ]; then lib=$R/vvc-affine-gpu_amd/lib/libvame.so; else lib=$R/vvc-affine-gpu_amd/lib/libvame_dup$v.so; fi
  bash $R/profiles/run_sq_lib.sh ${TAG}_dup$v $lib --no-spans "$@" || exit 1
done
echo dup-done
