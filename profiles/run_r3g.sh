set -o pipefail
O=gpurun_out/r3g; mkdir -p $O
VAME_LIB=vvc-affine-gpu_amd/lib/libvame_count.so timeout -k 10 300 python3 profiles/count_preds.py --config c5 --gpus 8 --rank-only 7 > $O/count_c5r7.json 2> $O/count.err || { tail $O/count.err; exit 1; }
cat $O/count_c5r7.json
for lib in libvame libvame_ablate512; do
  for args in "--config c5 --gpus 8 --rank-only 7" "--config c4"; do
    VAME_LIB=vvc-affine-gpu_amd/lib/$lib.so timeout -k 10 300 python3 bench.py $args --no-cpu-baseline --no-spans > $O/b.json 2> $O/b.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('$lib', '$args', round(d['ms_per_step'],2), 'quad', round(d['roofline']['avg_launch_ms'],2), 'ctu', round(d['roofline']['affine_me_ctu']['avg_launch_ms'],2), 'frac', round(d['roofline']['frac'],4))"
  done
done
