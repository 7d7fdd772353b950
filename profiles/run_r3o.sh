set -o pipefail
O=gpurun_out/r3o; mkdir -p $O
for c in c2 c3 c4 c5; do
  bash profiles/heartbeat.sh timeout -k 10 400 python3 bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', round(d['ms_per_step'],3), round(d['value']/1e6,1), 'frac', round(d['roofline']['frac'],4), d['parity_sample'], d['cpu_baseline']['value'])"
done
