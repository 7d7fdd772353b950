#!/bin/bash
# round 6: LLVM option variants of the split build against it: uniform
# regions left unstructurized (skipuni), two-entry phi folding threshold 1 /
# 8 (phi1 / phi8), no AMDGPU VGPR live-range optimisation (noliv).  A c2 / batch
# parity subset per variant, then interleaved A/B lines.  gpurun only.
set -o pipefail
L=vvc-affine-gpu_amd/lib
for v in skipuni phi1 noliv phi8; do
  VAME_LIB=$L/libvame_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
      --timeout-method thread -m gpu -k "c2 or batch" > gpurun_out/r06ab9_$v.log 2>&1 || { tail -5 gpurun_out/r06ab9_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r06ab9_$v.log)"
done
V=(default:VAME_LIB=$L/libvame.so skipuni:VAME_LIB=$L/libvame_skipuni.so phi1:VAME_LIB=$L/libvame_phi1.so noliv:VAME_LIB=$L/libvame_noliv.so phi8:VAME_LIB=$L/libvame_phi8.so)
REPS=3 bash profiles/run_bench_env.sh r06ab9_c2 "${V[@]}" -- --no-spans || exit 1
REPS=1 bash profiles/run_bench_env.sh r06ab9_c4 "${V[@]}" -- --no-spans --config c4 || exit 1
echo r06-done
