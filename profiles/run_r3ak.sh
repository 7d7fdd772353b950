# c3 / c4 / c5 bench lines at HEAD (final round-3 engine)
set -o pipefail
O=gpurun_out/r3ak; mkdir -p $O
for c in c3 c4 c5; do
  timeout -k 10 500 python bench.py --config $c > $O/$c.json 2> $O/$c.err || { tail -10 $O/$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$c.json')); r=d['roofline']; print('$c', round(d['ms_per_step'],2), round(d['value']/1e6,1), 'frac', round(r['frac'],4), 'parity', d.get('parity_sample'), d['gather']['check']['byte_identical'])"
done
