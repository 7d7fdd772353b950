# CLI at C5 cut to 60 frames with the timeline: is the constant ~5 ms gap
# between batches the result download (285 MB at ~56 GB/s) serialised with
# the compute stream?  Variants: default; copy streams at low / high priority
# (VAME_CLI_COPY_PRIO=1 / -1); more hardware queues (GPU_MAX_HW_QUEUES=8).
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
O=$R/gpurun_out/r3aa; mkdir -p $O
T=$(mktemp -d /tmp/vame_c5.XXXXXX)
trap 'rm -rf $T' EXIT
export PYTHONPATH=$R/vvc-affine-gpu_amd
python3 -c "
from vame.synth import synth_sequence, write_csv
o, r = synth_sequence(3840, 2160, 60, 32)
write_csv('$T/orig.csv', o); write_csv('$T/recon.csv', r)
print('csv written', flush=True)
"
mkdir -p $T/cli
run() {  # name, env...
  local name=$1; shift
  rm -f $T/cli/*
  env "$@" VAME_CLI_TRACE=1 timeout -k 10 200 $R/vvc-affine-gpu_amd/bin/vame -f 60 -s 3840x2160 -q 32 -o $T/orig.csv \
      -r $T/recon.csv -l $T/cli/log > $O/$name.txt 2> $O/$name.err
  echo "$name: $(grep -E 'TOTAL_EXEC|OVERALL' $O/$name.txt | tr '\n' ' ')"
  grep 'kernels' $O/$name.err | sed 's/.*GPU:/GPU:/'
  grep 'gaps (ms)' $O/$name.err | cut -c1-260
}
run warm VAME_X=0
run base VAME_X=0
run prio_lo VAME_CLI_COPY_PRIO=1
run prio_hi VAME_CLI_COPY_PRIO=-1
run hwq8 GPU_MAX_HW_QUEUES=8
run base2 VAME_X=0
