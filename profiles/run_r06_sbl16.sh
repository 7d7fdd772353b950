#!/bin/bash
# round 6: the 16-sub-block quadrant CUs two sub-blocks per lane too
# (VAME_SBL2_16 build): the GPU suite on it, then A/B lines at c2 / c4 against
# the default build.  gpurun only.
set -o pipefail
L=vvc-affine-gpu_amd/lib
O=gpurun_out/check16; mkdir -p $O
VAME_LIB=$L/libvame_sbl16.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread -k "not under_torchrun" > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
case $rc in 0) ;; 1) grep -E "FAILED|Error" $O/pytest.log | head -5; exit 1;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
V=(default:VAME_LIB=$L/libvame.so sbl16:VAME_LIB=$L/libvame_sbl16.so)
REPS=3 bash profiles/run_bench_env.sh r06ab4_c2 "${V[@]}" -- --no-spans || exit 1
REPS=1 bash profiles/run_bench_env.sh r06ab4_c4 "${V[@]}" -- --no-spans --config c4 || exit 1
echo r06-done
