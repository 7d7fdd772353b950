#!/bin/bash
# GPU-box profiling recipe (gpurun): the bench line, a rocprofv3 kernel trace +
# stats, then separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ/GRBM counters;
# MI355X_MICROARCH.md §HBM and §rocprofv3 PMC slots), the executed-prediction
# count of the instrumentation build (make count), and their summary.
#   bash profiles/run_profile.sh <tag> <config> [bench args...]
# Every profiled run uses --no-spans: each kernel's dispatches are then the
# step's batched launches only, so per-launch averages are of identical work.
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TAG=${1:-c2}; CFG=${2:-c2}; shift 2 || true
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --config $CFG --fs-frames 0"
P="--no-spans --no-cpu-baseline --steps ${PSTEPS:-10} --warmup ${PWARM:-2}"  # c5: PSTEPS=1 PWARM=0
echo "[prof] bench line"
timeout -k 10 600 $B "$@" > $O/bench.json 2> $O/bench.err
cat $O/bench.json
echo "[prof] kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- \
    $B "$@" $P > $O/trace.log 2>&1
echo "[prof] FETCH_SIZE"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
    $B "$@" $P > $O/pmc_fetch.log 2>&1
echo "[prof] WRITE_SIZE"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
    $B "$@" $P > $O/pmc_write.log 2>&1
echo "[prof] SQ"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
    SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $O/pmc_sq -o run -- $B "$@" $P > $O/pmc_sq.log 2>&1
echo "[prof] prediction count"
if [ -f $R/vvc-affine-gpu_amd/lib/libvame_count.so ]; then
  VAME_LIB=$R/vvc-affine-gpu_amd/lib/libvame_count.so timeout -k 10 300 \
      python3 $R/profiles/count_preds.py --config $CFG ${COUNT_ARGS:-} > $O/count.json 2> $O/count.err
  cat $O/count.json
fi
python3 $R/profiles/pmc_summary.py $O $O/summary.json > /dev/null
if [ -n "${CLEAN:-}" ]; then  # big configs: keep the summary, stats and logs (gpurun returns <= 64 MiB)
  rm -f $O/trace/run_kernel_trace.csv $O/pmc_*/run_counter_collection.csv
fi
echo profile-done
