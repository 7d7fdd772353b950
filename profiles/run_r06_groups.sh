#!/bin/bash
# round 6: the block-order group size (VAME_GROUP_COMBOS: (CTU, pair)
# combinations per group, default 408) at c3 / c4 with the final kernels.
# gpurun only.
set -o pipefail
V=(g408:VAME_GROUP_COMBOS=408 g204:VAME_GROUP_COMBOS=204 g816:VAME_GROUP_COMBOS=816 g1632:VAME_GROUP_COMBOS=1632)
REPS=1 bash profiles/run_bench_env.sh r06ab16_c3 "${V[@]}" -- --no-spans --config c3 || exit 1
REPS=1 bash profiles/run_bench_env.sh r06ab16_c4 "${V[@]}" -- --no-spans --config c4 || exit 1
echo r06-done
