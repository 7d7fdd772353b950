#!/bin/bash
# round 6: the caller's-stream order of a 2+3-CP launch: affine_me_ctu2, the
# half kernels, affine_me_quad (default) vs the half kernels first (bo1) vs
# affine_me_quad first (bo2); affine_me_quad2 on the side stream in all.  A
# parity subset of the 2+3-CP paths per variant, then interleaved c3 / c4
# lines.  gpurun only.
set -o pipefail
L=vvc-affine-gpu_amd/lib
for v in bo1 bo2; do
  VAME_LIB=$L/libvame_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 \
      --timeout-method thread -m gpu -k "fused_vs_oracle or batch_equals or live_reference_1080p or property" \
      > gpurun_out/r06ab14_$v.log 2>&1 || { tail -5 gpurun_out/r06ab14_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r06ab14_$v.log)"
done
V=(default:VAME_LIB=$L/libvame.so bo1:VAME_LIB=$L/libvame_bo1.so bo2:VAME_LIB=$L/libvame_bo2.so)
REPS=2 bash profiles/run_bench_env.sh r06ab14_c3 "${V[@]}" -- --no-spans --config c3 || exit 1
REPS=2 bash profiles/run_bench_env.sh r06ab14_c4 "${V[@]}" -- --no-spans --config c4 || exit 1
echo r06-done
