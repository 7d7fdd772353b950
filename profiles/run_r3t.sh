# lane use of the prediction steps (instrumentation build): c2, c3, c4
set -o pipefail
O=gpurun_out/r3t; mkdir -p $O
for c in c2 c3 c4; do
  VAME_LIB=vvc-affine-gpu_amd/lib/libvame_count.so timeout -k 10 300 python3 profiles/count_preds.py --config $c > $O/count_$c.json 2> $O/count_$c.err || { tail -5 $O/count_$c.err; exit 1; }
  cat $O/count_$c.json
done
