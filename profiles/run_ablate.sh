#!/bin/bash
# Phase ablations (timing-only builds from `make ablate`, results are wrong) + SQ
# counter passes.  gpurun only.
#   bash profiles/run_ablate.sh "<ablate ids>" [bench args]
R="$(cd "$(dirname "$0")/.." && pwd)"
O=$R/gpurun_out/ablate
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
IDS=${1:-"1 16 32"}; shift || true
step() {  # name, command...; stop on crash-like exit codes, continue on ordinary failure
  local name=$1; shift
  timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 124|134|137|139) echo "crash-like exit, stopping"; exit $rc;; esac
  return 0
}
for v in 0 $IDS; do
  if [ "$v" = 0 ]; then lib=$R/vvc-affine-gpu_amd/lib/libvame.so; else lib=$R/vvc-affine-gpu_amd/lib/libvame_ablate$v.so; fi
  VAME_LIB=$lib step bench_ablate$v python3 $R/bench.py --no-cpu-baseline --fs-frames 0 "$@"
  tail -c 1200 $O/bench_ablate$v.out | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ablate$v', round(d['ms_per_step'],3), 'quad', round(d['roofline']['avg_launch_ms'],3), 'ctu', round(d['roofline']['affine_me_ctu']['avg_launch_ms'],3))" || true
done
if [ -n "$SQ" ]; then
step pmc_sq1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_sq1 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --fs-frames 0 "$@"
step pmc_sq2 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --fs-frames 0 "$@"
fi
echo ablate-done
