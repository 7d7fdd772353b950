#!/bin/bash
# Phase ablations (timing-only builds) + SQ counter passes.  gpurun only.
#   bash profiles/run_ablate.sh [bench args]
R="$(cd "$(dirname "$0")/.." && pwd)"
O=$R/gpurun_out/ablate
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
step() {  # name, command...; stop on crash-like exit codes, continue on ordinary failure
  local name=$1; shift
  timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 124|134|137|139) echo "crash-like exit, stopping"; exit $rc;; esac
  return 0
}
for v in "" 1 2 4 6 7 8 11 13 14 15; do
  lib=$R/vvc-affine-gpu_amd/lib/libvame${v:+_ablate$v}.so
  VAME_LIB=$lib step bench_ablate${v:-0} python3 $R/bench.py --no-cpu-baseline "$@"
  tail -c 900 $O/bench_ablate${v:-0}.out | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ablate${v:-0}', round(d['ms_per_step'],3), 'quad', round(d['roofline']['avg_launch_ms'],3), 'ctu', round(d['roofline']['big_kernel_avg_launch_ms'],3))" || true
done
step pmc_sq1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_sq1 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@"
step pmc_sq2 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@"
echo ablate-done
