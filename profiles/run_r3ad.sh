# c5 strong-scaling forecast: every rank's block of the 8-GPU (and 2-, 4-GPU) job alone on this GPU
set -o pipefail
O=gpurun_out/r3ad; mkdir -p $O
for N in 8 4 2; do
  for K in $(seq 0 $((N - 1))); do
    timeout -k 10 240 python bench.py --config c5 --no-cpu-baseline --no-spans --gpus $N --rank-only $K > $O/n${N}_r$K.json 2> $O/n${N}_r$K.err || { tail -5 $O/n${N}_r$K.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/n${N}_r$K.json')); print($N, $K, d['config']['pairs_per_step_rank0'], round(d['ms_per_step'],2), d['gather']['check']['byte_identical'])"
  done
done
