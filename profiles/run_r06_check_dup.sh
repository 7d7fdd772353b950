#!/bin/bash
# round 6: the GPU suite, then the VALU phase split (dup builds) at c2 / c4.
# Stops at a GPU fault / abort / time limit; a plain test failure does not
# stop the profiling.  gpurun only.
set -o pipefail
O=gpurun_out/check; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
IDS="1 2 4 16 64 128 256 512 1024 2048"
bash profiles/run_dup_sq.sh r06c2 "$IDS" > gpurun_out/r06_dup_c2.log 2>&1 || exit 1
bash profiles/run_dup_sq.sh r06c4 "$IDS" --config c4 > gpurun_out/r06_dup_c4.log 2>&1 || exit 1
echo r06-done
