#!/bin/bash
# round 6: the two-body kernels in 2+3-CP launches too, now that the build
# flags leave them (nearly) without spill slots: affine_me_quad over every
# quadrant item (qm: VAME_SPLIT=2), affine_me_half2 over both orientations
# (hm: VAME_HALF_MERGE=2), both (qhm), against the by-mode default.  A parity
# subset per variant (2+3-CP paths at 1080p / 2160p), then interleaved A/B
# lines at c3 / c4.  gpurun only.
set -o pipefail
L=vvc-affine-gpu_amd/lib
for v in qm hm qhm; do
  VAME_LIB=$L/libvame_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 \
      --timeout-method thread -m gpu -k "fused_vs_oracle or batch_equals or live_reference_1080p or property" \
      > gpurun_out/r06ab11_$v.log 2>&1 || { tail -5 gpurun_out/r06ab11_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r06ab11_$v.log)"
done
V=(default:VAME_LIB=$L/libvame.so qm:VAME_LIB=$L/libvame_qm.so hm:VAME_LIB=$L/libvame_hm.so qhm:VAME_LIB=$L/libvame_qhm.so)
REPS=2 bash profiles/run_bench_env.sh r06ab11_c3 "${V[@]}" -- --no-spans --config c3 || exit 1
REPS=1 bash profiles/run_bench_env.sh r06ab11_c4 "${V[@]}" -- --no-spans --config c4 || exit 1
echo r06-done
