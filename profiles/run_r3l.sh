set -o pipefail
O=gpurun_out/r3l; mkdir -p $O
for a in "--config c4" "--config c5 --gpus 8 --rank-only 7"; do
  VAME_LIB=vvc-affine-gpu_amd/lib/libvame_count.so timeout -k 10 300 python3 profiles/count_preds.py $a > $O/c.json 2> $O/c.err || { tail $O/c.err; exit 1; }
  cat $O/c.json
done
