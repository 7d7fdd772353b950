#!/bin/bash
# round 6: the GPU suite on the default build (quadrant structure by launch
# mode, the 128x64 / 64x128 CUs in one affine_me_half2 launch), then A/B
# lines at c2 / c4 and the c2 timeline.  gpurun only.
set -o pipefail
O=gpurun_out/check; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
L=vvc-affine-gpu_amd/lib
V=(default:VAME_LIB=$L/libvame.so halfsep:VAME_LIB=$L/libvame_halfsep.so merged:VAME_LIB=$L/libvame_merged.so
   split:VAME_LIB=$L/libvame_split.so nosplit:VAME_LIB=$L/libvame_nosplit.so)
REPS=2 bash profiles/run_bench_env.sh r06ab3_c2 "${V[@]}" -- --no-spans || exit 1
REPS=1 bash profiles/run_bench_env.sh r06ab3_c4 "${V[@]}" -- --no-spans --config c4 || exit 1
VARIANTS="default halfsep" SQCFG=" " bash profiles/run_r06_timeline.sh || exit 1
echo r06-done
