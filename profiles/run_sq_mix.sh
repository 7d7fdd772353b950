#!/bin/bash
# The VALU instruction mix per kernel (gpurun only): two SQ passes of the c2
# bench (or the given config) with the per-type instruction counters.
#   bash profiles/run_sq_mix.sh <tag> [bench args]
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH"
G2="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_SMEM"
i=1
for G in "$G1" "$G2"; do
  timeout -s KILL 300 rocprofv3 --pmc $G --output-format csv -d $O/p$i -o run -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-spans --fs-frames 0 "$@" > $O/p$i.log 2>&1
  rc=$?; echo "$TAG pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  i=$((i + 1))
done
python3 $R/profiles/sq_summary.py $O > $O/summary.txt && cat $O/summary.txt
