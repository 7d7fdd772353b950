# CLI timeline (VAME_CLI_TRACE=1) at C5: where OVERALL goes beyond the kernel time
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
O=$R/gpurun_out/r3w; mkdir -p $O
T=$(mktemp -d /tmp/vame_c5.XXXXXX)
trap 'rm -rf $T' EXIT
export PYTHONPATH=$R/vvc-affine-gpu_amd
python3 -c "
from vame.synth import synth_sequence, write_csv
o, r = synth_sequence(3840, 2160, 240, 32)
write_csv('$T/orig.csv', o); write_csv('$T/recon.csv', r)
print('csv written', flush=True)
"
mkdir -p $T/cli
for run in 1 2; do
  rm -f $T/cli/*
  VAME_CLI_TRACE=1 timeout -k 10 400 $R/vvc-affine-gpu_amd/bin/vame -f 240 -s 3840x2160 -q 32 -o $T/orig.csv \
      -r $T/recon.csv -l $T/cli/log > $O/cli_run$run.txt 2> $O/cli_run$run.err
  echo "cli run $run: $(grep -E 'TOTAL_EXEC|OVERALL|READ_CSV|LOG_WRITE' $O/cli_run$run.txt | tr '\n' ' ')"
  grep trace $O/cli_run$run.err
done
rm -f $T/cli/*
VAME_CLI_TRACE=1 timeout -k 10 400 $R/vvc-affine-gpu_amd/bin/vame -f 240 -s 3840x2160 -q 32 -o $T/orig.csv \
    -r $T/recon.csv > $O/cli_nolog.txt 2> $O/cli_nolog.err
echo "cli without logs: $(grep -E 'TOTAL_EXEC|OVERALL' $O/cli_nolog.txt | tr '\n' ' ')"
grep trace $O/cli_nolog.err
