# timing only the quadrant kernel in the timed steps (VAME_BENCH_KTIMING=2) vs both (1) vs none (0)
set -o pipefail
O=gpurun_out/r3al; mkdir -p $O
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-spans > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$name.json')); r=d['roofline']; print('$name', round(d['ms_per_step'],4), 'quad', round(r['avg_launch_ms'],4))"
}
for rep in 1 2 3; do run both$rep VAME_BENCH_KTIMING=1; run quad$rep VAME_BENCH_KTIMING=2; run off$rep VAME_BENCH_KTIMING=0; done
