#!/bin/bash
# round 6: the split build with uniform regions left unstructurized (default) against it
# without (prev) and with two-entry phi folding threshold 1 on top (sp1): the GPU suite on
# default, then interleaved A/B lines at c2 / c3 / c4.
# gpurun only.
set -o pipefail
L=vvc-affine-gpu_amd/lib
O=gpurun_out/check_skipuni; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
case $rc in 0) ;; 1) grep -E "FAILED|Error" $O/pytest.log | head -5; exit 1;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
V=(default:VAME_LIB=$L/libvame.so prev:VAME_LIB=$L/libvame_prev.so sp1:VAME_LIB=$L/libvame_sp1.so)
REPS=3 bash profiles/run_bench_env.sh r06ab10_c2 "${V[@]}" -- --no-spans || exit 1
REPS=2 bash profiles/run_bench_env.sh r06ab10_c3 "${V[@]}" -- --no-spans --config c3 || exit 1
REPS=1 bash profiles/run_bench_env.sh r06ab10_c4 "${V[@]}" -- --no-spans --config c4 || exit 1
echo r06-done
