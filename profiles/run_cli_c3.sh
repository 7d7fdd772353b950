set -e
python - <<'PY'
import sys; sys.path.insert(0,'vvc-affine-gpu_amd')
from vame.synth import synth_sequence
o,r=synth_sequence(1920,1080,30,32)
o.tofile('gpurun_out/o.u16'); r.tofile('gpurun_out/r.u16')
PY
for i in 1 2; do
timeout -k 10 120 vvc-affine-gpu_amd/bin/vame -f 30 -s 1920x1080 -q 32 -o gpurun_out/o.u16 -r gpurun_out/r.u16 > gpurun_out/cli_fused.txt
grep -E "FUSED_POC_EXEC|TOTAL_EXEC|OVERALL" gpurun_out/cli_fused.txt
done
rm -f gpurun_out/o.u16 gpurun_out/r.u16
