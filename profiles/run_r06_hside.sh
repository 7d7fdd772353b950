#!/bin/bash
# round 6: the c2 step's affine_me_half2 launch on a second side stream (hside,
# starts beside affine_me_ctu2) or ahead of affine_me_ctu2 on the caller's
# stream (hfirst) vs the default (after affine_me_ctu2).  Interleaved lines,
# then a parity check of each build on the c2 step.  gpurun only.
set -o pipefail
L=vvc-affine-gpu_amd/lib
V=(default:VAME_LIB=$L/libvame.so hside:VAME_LIB=$L/libvame_hside.so hfirst:VAME_LIB=$L/libvame_hfirst.so)
REPS=3 bash profiles/run_bench_env.sh r06ab6_c2 "${V[@]}" -- --no-spans || exit 1
for v in hside hfirst; do
  VAME_LIB=$L/libvame_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
      --timeout-method thread -m gpu -k "c2 or batch" > gpurun_out/r06ab6_$v.log 2>&1 || { tail -5 gpurun_out/r06ab6_$v.log; exit 1; }
  tail -1 gpurun_out/r06ab6_$v.log
done
echo r06-done
