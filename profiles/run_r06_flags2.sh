#!/bin/bash
# round 6: more LLVM option variants of the final build against it: relaxed uniform-region
# checks (relax), no SLP vectorizer (noslp), the engine unit without common-code hoisting too
# (hoistall).  A c2 / batch parity subset per variant, then interleaved A/B lines.  gpurun only.
set -o pipefail
L=vvc-affine-gpu_amd/lib
for v in relax noslp hoistall; do
  VAME_LIB=$L/libvame_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
      --timeout-method thread -m gpu -k "c2 or batch" > gpurun_out/r06ab12_$v.log 2>&1 || { tail -5 gpurun_out/r06ab12_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r06ab12_$v.log)"
done
V=(default:VAME_LIB=$L/libvame.so relax:VAME_LIB=$L/libvame_relax.so noslp:VAME_LIB=$L/libvame_noslp.so hoistall:VAME_LIB=$L/libvame_hoistall.so)
REPS=3 bash profiles/run_bench_env.sh r06ab12_c2 "${V[@]}" -- --no-spans || exit 1
REPS=1 bash profiles/run_bench_env.sh r06ab12_c3 "${V[@]}" -- --no-spans --config c3 || exit 1
REPS=1 bash profiles/run_bench_env.sh r06ab12_c4 "${V[@]}" -- --no-spans --config c4 || exit 1
echo r06-done
