#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run per group; no tracing domains).
#   bash profiles/run_sq.sh <tag> [bench args]      (gpurun only)
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=${1:-sq}; shift || true
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU"
G2="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32"
G3="SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
i=0
for G in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G --output-format csv -d $O/p$i -o run -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
python3 $R/profiles/sq_summary.py $O > $O/summary.txt && cat $O/summary.txt
