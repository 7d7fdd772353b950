#!/bin/bash
# round 6: the GPU suite on the split packing (affine_me_quad + affine_me_quad2),
# then A/B lines at c2 / c4: default, the packing of rounds 4-5 (nosplit),
# quad2 with its stash in LDS, affine_me_quad on the quadrant stream.  gpurun only.
set -o pipefail
O=gpurun_out/check; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
L=vvc-affine-gpu_amd/lib
V=(default:VAME_LIB=$L/libvame.so nosplit:VAME_LIB=$L/libvame_nosplit.so stash:VAME_LIB=$L/libvame_stash.so q1side:VAME_LIB=$L/libvame_q1side.so)
REPS=2 bash profiles/run_bench_env.sh r06ab_c2 "${V[@]}" -- --no-spans || exit 1
REPS=2 bash profiles/run_bench_env.sh r06ab_c4 "${V[@]}" -- --no-spans --config c4 || exit 1
echo r06-done
