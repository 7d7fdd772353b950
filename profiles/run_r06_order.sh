#!/bin/bash
# round 6: the item order of the 2-CP-only affine_me_quad launch: cooperative
# chains, SBL2 items, 16-sub-block items (default) vs SBL2 items first (o1) vs
# SBL2 items last (o2).  A c2 / batch parity subset per variant, then
# interleaved c2 lines.  gpurun only.
set -o pipefail
L=vvc-affine-gpu_amd/lib
for v in o1 o2; do
  VAME_LIB=$L/libvame_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
      --timeout-method thread -m gpu -k "c2 or batch or 2cp" > gpurun_out/r06ab13_$v.log 2>&1 || { tail -5 gpurun_out/r06ab13_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r06ab13_$v.log)"
done
V=(default:VAME_LIB=$L/libvame.so o1:VAME_LIB=$L/libvame_o1.so o2:VAME_LIB=$L/libvame_o2.so)
REPS=4 bash profiles/run_bench_env.sh r06ab13_c2 "${V[@]}" -- --no-spans || exit 1
echo r06-done
