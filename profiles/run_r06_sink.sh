#!/bin/bash
# round 6: the kernels built without SimplifyCFG's common-code sinking
# (nosink: -mllvm -simplifycfg-sink-common=false) and without sinking and
# hoisting (nohs), which drop most spill slots, against the
# default build: the GPU suite on nohs, then interleaved A/B lines.  gpurun only.
set -o pipefail
L=vvc-affine-gpu_amd/lib
O=gpurun_out/check_sink; mkdir -p $O
VAME_LIB=$L/libvame_nohs.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread -k "not under_torchrun" > $O/pytest.log 2>&1
rc=$?
tail -1 $O/pytest.log
case $rc in 0) ;; 1) grep -E "FAILED|Error" $O/pytest.log | head -5; exit 1;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
V=(default:VAME_LIB=$L/libvame.so nosink:VAME_LIB=$L/libvame_nosink.so nohs:VAME_LIB=$L/libvame_nohs.so)
REPS=3 bash profiles/run_bench_env.sh r06ab7_c2 "${V[@]}" -- --no-spans || exit 1
REPS=2 bash profiles/run_bench_env.sh r06ab7_c3 "${V[@]}" -- --no-spans --config c3 || exit 1
REPS=1 bash profiles/run_bench_env.sh r06ab7_c4 "${V[@]}" -- --no-spans --config c4 || exit 1
echo r06-done
