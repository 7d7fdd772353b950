#!/bin/bash
# round 6: the split build (the 2-CP-only kernels in a unit of their own, built without
# SimplifyCFG common-code hoisting and sinking; the rest without sinking; default) against
# the one-unit build of before (prev): the GPU suite on default, then A/B lines at c2 / c3 / c4.
# gpurun only.
set -o pipefail
L=vvc-affine-gpu_amd/lib
O=gpurun_out/check_tu; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
case $rc in 0) ;; 1) grep -E "FAILED|Error" $O/pytest.log | head -5; exit 1;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
V=(default:VAME_LIB=$L/libvame.so prev:VAME_LIB=$L/libvame_prev.so)
REPS=3 bash profiles/run_bench_env.sh r06ab8_c2 "${V[@]}" -- --no-spans || exit 1
REPS=2 bash profiles/run_bench_env.sh r06ab8_c3 "${V[@]}" -- --no-spans --config c3 || exit 1
REPS=1 bash profiles/run_bench_env.sh r06ab8_c4 "${V[@]}" -- --no-spans --config c4 || exit 1
echo r06-done
