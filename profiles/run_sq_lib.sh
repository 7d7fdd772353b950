#!/bin/bash
# SQ pass 1 (instruction counts, wave cycles) for one library build.
#   bash profiles/run_sq_lib.sh <tag> <lib.so> [bench args]      (gpurun only)
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=$1; LIB=$(readlink -f $2); shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
VAME_LIB=$LIB timeout -k 10 300 rocprofv3 --pmc $G1 --output-format csv -d $O/p1 -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --fs-frames 0 "$@" > $O/p1.log 2>&1
rc=$?; echo "$TAG rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
python3 $R/profiles/sq_summary.py $O > $O/summary.txt && cat $O/summary.txt
