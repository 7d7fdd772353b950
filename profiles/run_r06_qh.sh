#!/bin/bash
# round 6: the 2-CP-only launch's 128x64 / 64x128 items inside the one
# affine_me_quad launch (qh: VAME_QUAD_HALF=1, the half items first in its
# item order; affine_me_ctu2 alone on the caller's stream) against the default
# (affine_me_half2 after affine_me_ctu2 on the caller's stream).  The 2-CP
# parity tests on qh, then interleaved c2 lines.  gpurun only.
set -o pipefail
L=vvc-affine-gpu_amd/lib
VAME_LIB=$L/libvame_qh.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 \
    --timeout-method thread -m gpu -k "c2 or 2cp or batch or fused or dropin or alignment" > gpurun_out/r06ab15_qh.log 2>&1 \
    || { tail -5 gpurun_out/r06ab15_qh.log; exit 1; }
echo "qh: $(tail -1 gpurun_out/r06ab15_qh.log)"
V=(default:VAME_LIB=$L/libvame.so qh:VAME_LIB=$L/libvame_qh.so)
REPS=4 bash profiles/run_bench_env.sh r06ab15_c2 "${V[@]}" -- --no-spans || exit 1
echo r06-done
