#!/bin/bash
# round 6: the GPU suite on the default build (one affine_me_quad kernel over
# the SBL1 and SBL2 items), then A/B lines at c2 / c4 of the quadrant
# packings, then c2 timelines.  gpurun only.
set -o pipefail
O=gpurun_out/check; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
L=vvc-affine-gpu_amd/lib
V=(merged:VAME_LIB=$L/libvame.so split:VAME_LIB=$L/libvame_split.so split3:VAME_LIB=$L/libvame_split3.so
   q2t8:VAME_LIB=$L/libvame_q2t8.so nosplit:VAME_LIB=$L/libvame_nosplit.so)
REPS=2 bash profiles/run_bench_env.sh r06ab2_c2 "${V[@]}" -- --no-spans || exit 1
REPS=1 bash profiles/run_bench_env.sh r06ab2_c4 "${V[@]}" -- --no-spans --config c4 || exit 1
VARIANTS="merged split3" SQCFG=c2 bash profiles/run_r06_timeline.sh || exit 1
echo r06-done
